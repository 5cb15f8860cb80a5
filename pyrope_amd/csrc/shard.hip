// shard.hip -- the device side of the list-sharded multi-GPU search (IVF lists shard
// whole across the GPUs; pyrope_amd/dist.py ListShardedIvf drives it).
//
// A query's home rank ranks the coarse quantizer and computes its threshold T_q from a replicated sample of
// every list (the plan: P probe ids + T_q as float bits); every rank scans the (query, list) pairs whose
// list it owns against the gathered plans and writes one RECORD per query: its exact local top-k and the
// bound B_r every row it left out scores at most.  The home merges the records of all ranks and
// certifies: the k-th merged score must beat every B_r, else the query is re-run exactly on every rank.
//
// Records (ShardEntry x k, then ShardTrailer; shard_record_bytes(k) = 16 (k + 1)): entries in the order
// (score desc, list asc, label asc) -- the unsharded index's tie order, since a list keeps its rows in label
// order on the rank that owns it and lists are laid out by id.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <stdexcept>

#include "kernels.h"

namespace pyr {
namespace {

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

// (score desc, list asc, label asc); NaN ranks below every number (as better() in the scans)
__device__ __forceinline__ bool entry_better(float s1, int32_t l1, int64_t b1, float s2, int32_t l2, int64_t b2) {
  if (isnan(s2) && !isnan(s1)) return true;
  if (isnan(s1)) return false;
  return s1 > s2 || (s1 == s2 && (l1 < l2 || (l1 == l2 && b1 < b2)));
}

// plan [nq][S] = P probe ids, T_q's float bits, then (a MaxScans budget: S = 2P + 1) the P remaining budgets
__global__ void pack_plan_kernel(const int32_t *probes, const float *thr, const int32_t *rem, int64_t nq, int P,
                                 int32_t *plan) {
  const int S = P + 1 + (rem ? P : 0);
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nq * S) return;
  const int64_t q = e / S;
  const int c = (int)(e - q * S);
  plan[e] = c < P ? probes[q * P + c] : c == P ? __float_as_int(thr[q]) : rem[q * P + c - P - 1];
}
__global__ void unpack_plan_kernel(const int32_t *plan, int64_t nq, int P, int S, int32_t *probes, float *thr) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nq * (P + 1)) return;
  const int64_t q = e / (P + 1);
  const int c = (int)(e - q * (P + 1));
  if (c < P) probes[q * P + c] = plan[q * S + c];
  else thr[q] = __int_as_float(plan[q * S + P]);
}

// MaxScans on the home rank (IvfFlatVectorIndex.cs:202-212: the lists in probe order, each scanned until
// `scanned` reaches maxScans; the list-sharded index has no buffer).  One thread per query.
__global__ void shard_budget_kernel(const int32_t *probes, int64_t nq, int P, int64_t max_scans, const int32_t *glive,
                                    const int32_t *slb, const int32_t *sle, int32_t *rem, uint32_t *slimits) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  int64_t r = max_scans;
  for (int p = 0; p < P; ++p) {
    const int lst = probes[q * P + p];
    const int64_t left = r > 0 ? r : 0;
    rem[q * P + p] = (int32_t)min(left, (int64_t)INT32_MAX);
    const int64_t ns = sle[lst] - slb[lst];
    slimits[q * P + p] = (uint32_t)(slb[lst] + min(left, ns));
    r = left - glive[lst];
  }
}

// One wave per record index i: a k-step merge of the nparts sorted entry lists (lane s holds the head of
// part s), then the certificate.  Up to SM_LDS entries (N = 8, k = 10: 80) are first copied into the wave's
// LDS with independent loads, so the k steps read LDS instead of a chain of k dependent global loads.
constexpr int SM_LDS = 256;
__global__ __launch_bounds__(256) void shard_merge_kernel(ShardMergeArgs a) {
  __shared__ ShardEntry sent[4][SM_LDS];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + w;
  int64_t n = a.nrec;
  if (a.qsel) n = min((int64_t)a.qsel[0], (int64_t)a.cap);
  if (i >= n) return;
  const int64_t q = a.qsel ? a.qsel[1 + i] : i;
  const int k = a.k;
  const int64_t rb = shard_record_bytes(k);
  const bool mine = lane < a.nparts;
  const uint8_t *rec = a.rec + ((size_t)(mine ? lane : 0) * a.nrec + i) * rb;
  const ShardEntry *ent = reinterpret_cast<const ShardEntry *>(rec);
  const bool lds = a.nparts * k <= SM_LDS;
  if (lds) {
    for (int e = lane; e < a.nparts * k; e += 64) {
      const int s = e / k, j = e - s * k;
      sent[w][e] = reinterpret_cast<const ShardEntry *>(a.rec + ((size_t)s * a.nrec + i) * rb)[j];
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  const ShardTrailer tr = *reinterpret_cast<const ShardTrailer *>(rec + 16 * (size_t)k);
  float bound = mine ? tr.bound : -INFINITY;
  const int cnt = mine ? min(tr.n, k) : 0;
  int head = 0;
  int produced = 0;
  int lvl = 1;  // the largest butterfly offset that covers lanes 0 .. nparts - 1
  while (2 * lvl < a.nparts) lvl <<= 1;
  float kth = -INFINITY;
  for (int r = 0; r < k; ++r) {
    const bool has = head < cnt;
    ShardEntry e;
    if (has) e = lds ? sent[w][lane * k + head] : ent[head];
    float s = has ? e.score : -INFINITY;
    int32_t l = has ? e.list : 0x7FFFFFFF;
    int64_t b = has ? e.label : INT64_MAX;
    int src = has ? lane : 64;
    // wave argmax under entry_better (ties between parts cannot happen: a row lives on one rank) over the
    // lanes that hold a part: log2(nparts) butterfly levels (N = 8: 3, not 6), then lane 0's winner to all
    for (int off = lvl; off >= 1; off >>= 1) {
      const float s2 = __shfl_xor(s, off);
      const int32_t l2 = __shfl_xor(l, off);
      const int64_t b2 = __shfl_xor(b, off);
      const int src2 = __shfl_xor(src, off);
      const bool take = src2 < 64 && (src == 64 || entry_better(s2, l2, b2, s, l, b) ||
                                      (!entry_better(s, l, b, s2, l2, b2) && src2 < src));
      if (take) {
        s = s2;
        l = l2;
        b = b2;
        src = src2;
      }
    }
    s = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s)));  // (lane 0 is active: a uniform loop)
    b = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)b >> 32)) << 32) |
                  (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)b));
    src = __builtin_amdgcn_readfirstlane(src);
    if (src == 64) break;  // every part is exhausted
    if (lane == src) ++head;
    if (lane == 0) {
      a.out_s[(size_t)q * k + r] = s;
      a.out_l[(size_t)q * k + r] = b;
    }
    kth = s;
    ++produced;
  }
  if (lane == 0)
    for (int r = produced; r < k; ++r) {
      a.out_s[(size_t)q * k + r] = -INFINITY;
      a.out_l[(size_t)q * k + r] = -1;
    }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) bound = fmaxf(bound, __shfl_xor(bound, off));
  if (lane == 0) {
    if (a.out_c) a.out_c[q] = produced;
    if (a.fail) {
      // every row a rank left out scores <= its bound: the merged top-k is exact when its k-th score beats
      // every bound (or nothing was left out anywhere)
      const bool ok = bound == -INFINITY || (produced == k && kth > bound);
      if (!ok) {
        const int at = atomicAdd(a.fail, 1);
        if (at < a.fcap) a.fail[1 + at] = (int32_t)q;
      }
    }
  }
}

// gathered fail lists [nranks][1 + fcap] (home-local query ids) -> the global failing queries in rank
// order: fail[i] = s * nq_home + id, pos[i] = s * fcap + j (the record slot of the re-run's answer for
// home s), *nfail = their count.  One block.
__global__ __launch_bounds__(256) void shard_fail_compact_kernel(const int32_t *fails, int nranks, int fcap,
                                                                int64_t nq_home, int32_t *fail, int32_t *pos,
                                                                int32_t *nfail) {
  __shared__ int base[65];
  if (threadIdx.x == 0) {
    int t = 0;
    for (int s = 0; s < nranks; ++s) {
      base[s] = t;
      t += min(max(fails[(size_t)s * (1 + fcap)], 0), fcap);
    }
    base[nranks] = t;
    *nfail = t;
  }
  __syncthreads();
  for (int s = 0; s < nranks; ++s) {
    const int c = base[s + 1] - base[s];
    for (int j = threadIdx.x; j < c; j += blockDim.x) {
      fail[base[s] + j] = (int32_t)(s * nq_home + fails[(size_t)s * (1 + fcap) + 1 + j]);
      pos[base[s] + j] = s * fcap + j;
    }
  }
}

// the multi-device index's shards label their rows by the stage's storage positions: back to the caller's
// labels (table: the stage's per-position labels; -1 stays -1)
__global__ void map_positions_kernel(int64_t *l, int64_t n, const int64_t *table) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && l[i] >= 0) l[i] = table[l[i]];
}

// round j of the failures past fcap: entries [off, off + fcap) of every home's whole fail list
// (full [W][stride], stride = 1 + the home's batch) in the re-run's [W][1 + fcap] form
__global__ void fail_round_kernel(const int32_t *full, int W, int64_t stride, int off, int fcap, int32_t *out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)W * (1 + fcap)) return;
  const int s = (int)(e / (1 + fcap)), j = (int)(e - (int64_t)s * (1 + fcap));
  const int c = min(max(full[(size_t)s * stride] - off, 0), fcap);
  out[e] = j == 0 ? c : (j <= c ? full[(size_t)s * stride + off + j] : 0);
}

}  // namespace

void launch_map_positions(int64_t *l, int64_t n, const int64_t *table, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(map_positions_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, l, n, table);
}
void launch_fail_round(const int32_t *full, int W, int64_t stride, int off, int fcap, int32_t *out, hipStream_t st) {
  const int64_t n = (int64_t)W * (1 + fcap);
  if (n <= 0) return;
  hipLaunchKernelGGL(fail_round_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, full, W, stride, off, fcap, out);
}

void launch_pack_plan(const int32_t *probes, const float *thr, const int32_t *rem, int64_t nq, int P, int32_t *plan,
                      hipStream_t st) {
  if (nq <= 0) return;
  const int S = shard_plan_stride(P, rem != nullptr);
  hipLaunchKernelGGL(pack_plan_kernel, dim3(nblk(nq * S, 256)), dim3(256), 0, st, probes, thr, rem, nq, P, plan);
}
void launch_unpack_plan(const int32_t *plan, int64_t nq, int P, int stride, int32_t *probes, float *thr,
                        hipStream_t st) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(unpack_plan_kernel, dim3(nblk(nq * (P + 1), 256)), dim3(256), 0, st, plan, nq, P, stride, probes,
                     thr);
}
void launch_shard_budget(const int32_t *probes, int64_t nq, int P, int64_t max_scans, const int32_t *glive,
                         const int32_t *slb, const int32_t *sle, int32_t *rem, uint32_t *slimits, hipStream_t st) {
  if (nq <= 0 || P <= 0) return;
  hipLaunchKernelGGL(shard_budget_kernel, dim3(nblk(nq, 256)), dim3(256), 0, st, probes, nq, P, max_scans, glive, slb,
                     sle, rem, slimits);
}
void launch_shard_merge(const ShardMergeArgs &a, int64_t max_rec, hipStream_t st) {
  if (max_rec <= 0 || a.k <= 0) return;
  if (a.nparts < 1 || a.nparts > 64) throw std::invalid_argument("shard merge: 1 to 64 parts");
  hipLaunchKernelGGL(shard_merge_kernel, dim3(nblk(max_rec, 4)), dim3(256), 0, st, a);
}
void launch_shard_fail_compact(const int32_t *fails, int nranks, int fcap, int64_t nq_home, int32_t *fail, int32_t *pos,
                               int32_t *nfail, hipStream_t st) {
  if (nranks < 1 || nranks > 64) throw std::invalid_argument("shard re-run: 1 to 64 ranks");
  hipLaunchKernelGGL(shard_fail_compact_kernel, dim3(1), dim3(256), 0, st, fails, nranks, fcap, nq_home, fail, pos,
                     nfail);
}

}  // namespace pyr
