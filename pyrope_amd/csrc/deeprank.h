// deeprank.h -- the k > 60 merge + certified refine's select and rank, shared by deep_refine_kernel (filter.hip,
// the IVF_FLAT / FLAT stream scans) and pq_deep_refine_kernel (pq32.hip, the IVF_PQ matrix-core scan).  Internal;
// include inside an anonymous namespace of a .hip file's pyr namespace, after candmerge.h.
//
// One 256-thread block per query.  The candidates are the K1 best emitted rows by rank key merged with K1 copies of
// the floor placeholder max(T_q, floor) -- the rows above the floor first, then floors (every row left out scores
// at most the K1-th); their exact scores come from 8-lane groups (the caller's scorer, in the reference's order);
// the ranks by better() (score desc, key asc).  A NaN score fails the query (the exact scan decides).
// Round 6: the K1 best rows are SELECTED, not sorted out of the whole emitted set -- an MSB-first
// radix select over the 64-bit rank keys (8-bit digits, stopping at the first digit whose bin is taken whole),
// then one compaction; the K1 exact scores are ranked by a bitonic sort of K1 (score, key) words instead of K1^2
// pairwise counts.  (Round 5 sorted up to 8,192 emitted keys and counted 512 x 512 pairs per query: 8.9 of the
// 13.4 ms of a k = 256 search at I1, profiles/r6_deepk.)
#pragma once

constexpr int DEEP_MAX = 512;

struct DeepRank {
  const uint64_t *sk;  // the candidates' (score, key) words, ranked (sk[0] the best)
  const float *ex;     // candidate c's exact score (c < j) and its storage key
  const uint32_t *ky;
  int j;               // real candidates (rows); the other K1 - j are floor copies
  bool excluded;       // rows (or the floor) were left out of the K1
  float bound;         // what every row left out scores at most
  bool nan;            // a candidate's exact score is NaN
};

// dk: dynamic LDS of max(cap, 256) rank keys (deep_refine_lds_bytes).  exact(key, l) is called by the 8 lanes
// l = 0..7 of a group together and returns the row's exact score (at least in lane 0).
template <class Exact>
__device__ __forceinline__ DeepRank deep_select_rank(const CandMergeArgs &m, int64_t q, int d, uint64_t *dk,
                                                     Exact exact) {
  __shared__ uint64_t sk[DEEP_MAX];  // the exact (score, key) words being ranked
  __shared__ float ex[DEEP_MAX];
  __shared__ uint32_t ky[DEEP_MAX];
  __shared__ int hist[256];
  __shared__ uint64_t sel_s, kmin_s;  // the select's key prefix; the smallest candidate key
  __shared__ int need_s, done_s, above_s, nsel_s, nan_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tot = min(m.cand_n[q], m.cap);
  const uint32_t fk = m.cand_f[q];
  float F = m.thr ? m.thr[q] : -INFINITY;
  if (fk != 0u) F = fmaxf(F, key_score(fk));
  const uint64_t fkey = F > -INFINITY ? pack_cand(F, KEY_FLOOR) : 0ull;
  if (tid == 0) {
    above_s = 0;
    nsel_s = 0;
    nan_s = 0;
    sel_s = 0ull;
    kmin_s = ~0ull;
    need_s = d;
    done_s = 0;
  }
  __syncthreads();
  // 1. the rows' rank keys into LDS; how many lie above the floor
  const uint2 *cq = m.cand + (size_t)q * m.cap;
  int above = 0;
  for (int i = tid; i < tot; i += 256) {
    const uint2 e = cq[i];
    const uint64_t v = pack_cand(__uint_as_float(e.x), e.y);
    dk[i] = v;
    above += v > fkey ? 1 : 0;
  }
  if (above) atomicAdd(&above_s, above);
  __syncthreads();
  const int na = above_s;
  // 2. the threshold T: the candidates are the rows with key >= T.  na < d: every row above the floor (the rest
  // of the K1 are floor copies); else the d-th largest key (keys are distinct: the low word is ~storage key)
  uint64_t T = fkey + 1ull;
  if (na >= d) {
    uint64_t mask = 0ull;
#pragma unroll 1
    for (int shift = 56; shift >= 0; shift -= 8) {
      hist[tid] = 0;
      __syncthreads();
      const uint64_t pre = sel_s;
      for (int i = tid; i < tot; i += 256) {
        const uint64_t v = dk[i];
        if ((v & mask) == pre) atomicAdd(&hist[(int)(v >> shift) & 255], 1);
      }
      __syncthreads();
      if (w == 0) {  // the digit b whose bin holds the need-th largest: a suffix sum over bins 255 .. 0
        const int need = need_s;
        int c4[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c4[u] = hist[255 - 4 * lane - u];
          sum += c4[u];
        }
        int incl = sum;  // inclusive prefix over lanes (lane 0 = the highest bins)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int t = __shfl_up(incl, off);
          if (lane >= off) incl += t;
        }
        const int excl = incl - sum;
        const uint64_t hit = __builtin_amdgcn_ballot_w64(excl < need && incl >= need);
        const int L = (int)__builtin_ctzll(hit);  // (one lane: the counts reach need exactly once)
        if (lane == L) {
          int before = excl, b = 0, cb = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (before + c4[u] >= need) {
              b = 255 - 4 * lane - u;
              cb = c4[u];
              break;
            } else {
              before += c4[u];
            }
          sel_s = pre | ((uint64_t)b << shift);
          need_s = need - before;
          done_s = cb == need - before;  // the whole bin is taken: every key with this prefix is a candidate
        }
      }
      __syncthreads();
      mask |= 0xFFull << shift;
      if (done_s) break;  // (block-uniform)
    }
    T = sel_s;  // keys >= the prefix (its lower digits zero) are exactly the d largest
  }
  // 3. the candidates, compacted (order free: they are ranked below), and the smallest of their keys
  uint64_t kmin = ~0ull;
  for (int i = tid; i < tot; i += 256) {
    const uint64_t v = dk[i];
    if (v >= T && v > fkey) {
      const int c = atomicAdd(&nsel_s, 1);
      if (c < DEEP_MAX) ky[c] = ~(uint32_t)v;
      kmin = v < kmin ? v : kmin;
    }
  }
  if (kmin != ~0ull) atomicMin(reinterpret_cast<unsigned long long *>(&kmin_s), (unsigned long long)kmin);
  __syncthreads();
  DeepRank R;
  R.j = min(nsel_s, d);
  // the K1-th entry exists: rows (or the floor) were left out; every one of them scores at most its bound --
  // the K1-th row (na >= K1: the rows left out rank below it, the floor too) or the floor
  R.excluded = na >= d || fkey != 0ull;
  R.bound = na >= d ? key_score((uint32_t)(kmin_s >> 32)) : (fkey != 0ull ? F : -INFINITY);
  // 4. exact scores: group g of the block's 32 takes candidates g, g + 32, ... (every lane of a group ends with it)
  const int g = tid >> 3, l = tid & 7;
  for (int c = g; c < R.j; c += 32) {
    const float sc = exact(ky[c], l);
    if (l == 0) {
      ex[c] = sc;
      if (isnan(sc)) nan_s = 1;
    }
  }
  __syncthreads();
  // 5. rank by better(): a descending bitonic sort of the (score, key) words (-0 as +0: better() ties them)
  int P = 128;
  while (P < d) P <<= 1;
  for (int c = tid; c < P; c += 256) sk[c] = c < R.j ? pack_cand(ex[c] == 0.0f ? 0.0f : ex[c], ky[c]) : 0ull;
  __syncthreads();
  for (int sz = 2; sz <= P; sz <<= 1)
    for (int jj = sz >> 1; jj >= 1; jj >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int o = i ^ jj;
        if (o > i) {
          const uint64_t x = sk[i], y = sk[o];
          if ((i & sz) == 0 ? x < y : x > y) {
            sk[i] = y;
            sk[o] = x;
          }
        }
      }
      __syncthreads();
    }
  R.sk = sk;
  R.ex = ex;
  R.ky = ky;
  R.nan = nan_s != 0;
  return R;
}

// the k-th ranked exact score (-inf when fewer than k candidates)
__device__ __forceinline__ float deep_kth(const DeepRank &R, int k) {
  return min(R.j, k) == k ? key_score((uint32_t)(R.sk[k - 1] >> 32)) : -INFINITY;
}

// the top k (labels[key], or the key itself when labels is null), -inf / -1 past the candidates; the count; a
// failed query listed for the caller's exact scan
__device__ __forceinline__ void deep_write(const DeepRank &R, int64_t q, int k, bool ok, const int64_t *labels,
                                           float *out_s, int64_t *out_l, int32_t *out_c, int32_t *fail_list,
                                           int32_t *fail_cnt) {
  const int tid = threadIdx.x, nout = min(R.j, k);
  for (int r = tid; r < k; r += 256) {
    if (r < nout) {
      const uint64_t v = R.sk[r];
      const uint32_t kr = ~(uint32_t)v;
      float sc = key_score((uint32_t)(v >> 32));
      if (sc == 0.0f)  // the exact zero's own sign (the word holds +0 for both)
        for (int c = 0; c < R.j; ++c)
          if (R.ky[c] == kr) sc = R.ex[c];
      out_s[(size_t)q * k + r] = sc;
      out_l[(size_t)q * k + r] = labels ? labels[kr] : (int64_t)kr;
    } else {
      out_s[(size_t)q * k + r] = -INFINITY;
      out_l[(size_t)q * k + r] = -1;
    }
  }
  if (tid == 0) {
    if (out_c) out_c[q] = nout;
    if (!ok) fail_list[atomicAdd(fail_cnt, 1)] = (int32_t)q;
  }
}
