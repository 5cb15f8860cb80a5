// stream16.hip -- the IVF list scan as stream-and-emit over fp16 residual tiles (gfx950).
//
// Same contract as the round-2 list scan (filter16.hip: approximate scores over the lists' fp16
// residual tiles -> candidates -> certified exact refine, filter.hip refine_kernel), reorganised so
// that no wave ever waits on another wave's candidates and every tile is read from HBM once per
// (list chunk, <= 512 queries):
//
//  1. sprep_kernel: per (list, query) pair (the work lists' qlist order) the query's residual
//     q - c (L2) or q (IP), scaled by a power of two and rounded to fp16 (one term, or a hi/lo pair),
//     plus the score factor f and the per-(query, list) constant cq -- once, instead of in every
//     block that scans the list.
//  2. stream16_kernel<SAMPLE>: persistent blocks (one per CU, 8 waves) take work items (list, row
//     chunk, <= 512 queries) from a counter.  The item's query operands go to LDS (LDS-DMA, 128 KiB at
//     D = 128); then each wave streams its own 32-row tiles (t = w, w + 8, ...) from HBM straight into
//     registers (double-buffered, no LDS ring, no block barrier in the loop) and scores them against
//     every query group of the item on v_mfma_f32_16x16x32_f16 with the ROWS as the A operand: lane
//     (c, g) gets query c's scores of rows 4g..4g+3 of each 16-row half, so a query's factor and
//     threshold are lane scalars.
//       SAMPLE: the first 2 x 8 tiles of every list; each (wave, lane group) keeps the best score it
//     saw per query -> 32 values per (query, probe), each the score of a distinct row.
//  3. sselect_kernel: T_q = the K1-th largest of the query's sample values (radix select).  At least
//     K1 rows of its probed lists score >= T_q, so every row of its true top-K1 does.
//  4. stream16_kernel<MAIN>: every row with score >= T_q is emitted to its (query, part) region
//     (slot from an LDS counter, no list maintenance); a region that fills keeps the largest score it
//     had to drop as a floor.
//  5. cand_merge_kernel: per query the best KO (64) of its emitted rows, ranked with KO copies of the
//     floor placeholder max(T_q, floors) (KEY_FLOOR): every row left out scores <= the merged KO-th.
//  6. refine_kernel (filter.hip) certifies at depth K1, and the failures again at depth KO from the
//     same candidates -- no re-scan.
//
// Cost per (query group, tile): 8 MFMAs (one fp16 term; 16 with the split), 8 fma + 4 max3 + one
// compare per lane, and an emit branch taken for ~1 row in 1,000.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

#include "f16util.h"
#include "wselect.h"

constexpr int SNW = 8;         // waves per stream block
constexpr int SV = SNW * 4;    // sample values per (query, probe)
constexpr int SAMPLE_TILES = 2 * SNW;

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }

// ---- 1. query operands per (list, query) pair ----
// A lane group of D / 8 lanes per query (8 dims a lane, the centroid's 8 dims held in registers for
// the whole list), 64 / (D / 8) queries per wave at a time.
template <int D, int MET>
__global__ __launch_bounds__(256) void sprep_kernel(StreamArgs a) {
  const int item = blockIdx.x;
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  if (it.part != 0) return;  // chunk-0 items cover every qlist position of their list once
  constexpr int LQ = D / 8, QW = 64 / LQ;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane % LQ, qsl = lane / LQ;
  const float4 *cp = reinterpret_cast<const float4 *>(a.cents + (size_t)it.list * D + 8 * sub);
  const float4 c0 = cp[0], c1 = cp[1];
  const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  for (int qi0 = QW * w; qi0 < it.qcnt; qi0 += 4 * QW) {
    const int qi = qi0 + qsl;
    const bool act = qi < it.qcnt;
    const int pos = it.qbeg + (act ? qi : 0);
    const int q = a.qlist[pos] / a.nparts;
    const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)q * D + 8 * sub);
    const float4 q0 = qp[0], q1 = qp[1];
    const float qv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    float r[8], cq = 0.0f, amax = 0.0f, q2 = 0.0f, c2 = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (MET == L2) {
        r[u] = qv[u] - cv[u];
        cq += r[u] * r[u];
      } else {
        r[u] = qv[u];
        cq += qv[u] * cv[u];
        q2 += qv[u] * qv[u];
        c2 += cv[u] * cv[u];
      }
      amax = fmaxf(amax, fabsf(r[u]));
    }
#pragma unroll
    for (int off = 1; off < LQ; off <<= 1) {
      cq += __shfl_xor(cq, off);
      amax = fmaxf(amax, __shfl_xor(amax, off));
      if (MET == IP) {
        q2 += __shfl_xor(q2, off);
        c2 += __shfl_xor(c2, off);
      }
    }
    // the pair's share of the error bound (stream_ub_terms), rounded up by the 1e-3 in its constants
    float ep = 0.0f;
    if (MET == L2) {
      ep = a.kq * cq + a.kqa * sqrtf(cq);
    } else {
      const float qn = sqrtf(q2);
      ep = a.kq * q2 + a.kqa * qn + a.kqc * qn * sqrtf(c2);
    }
    const float sq = pow2_scale(amax);
    if (act) {
      h8v hv, lv;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float v = r[u] * sq;  // exact (power of two)
        hv[u] = (_Float16)v;
        lv[u] = (_Float16)(v - (float)hv[u]);
      }
      *reinterpret_cast<h8v *>(a.bq + (size_t)pos * D + 8 * sub) = hv;
      if (a.bql) *reinterpret_cast<h8v *>(a.bql + (size_t)pos * D + 8 * sub) = lv;
      if (sub == 0) a.qsc[pos] = make_float2((MET == L2 ? 2.0f : 1.0f) / (sq * a.sx), (MET == L2 ? -cq : cq) + ep);
    }
  }
}

// ---- 2. / 4. the list scan ----
template <int D, int MET, bool Q2, bool SAMPLE, bool AB = false>
__global__ __launch_bounds__(64 * SNW, 1) void stream16_kernel(StreamArgs a) {
  constexpr int KS = D / 32;            // 16x16x32 k-steps
  constexpr int TB = 64 * D;            // h16 bytes per 32-row tile
  constexpr int QMAX = Q2 ? 256 : 512;  // queries per item
  constexpr int PIECES = QMAX / 16 * KS;
  __shared__ __attribute__((aligned(16))) char bl[(Q2 ? 2 : 1) * PIECES * 1024];
  __shared__ float4 qr[QMAX];     // per query slot: {f, threshold in y = f acc + meta space, cq (score = y + cq),
                                  //  region (MAIN) / sample row (SAMPLE) as int bits}
  __shared__ int cnt_l[QMAX];     // rows emitted
  __shared__ uint32_t flr_l[QMAX];  // score_key of the best row a full region dropped (0: none)
  __shared__ int item_sh;
  const uint32_t bl_base = (uint32_t)(size_t)(lds_void *)bl;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const char *hsrc = reinterpret_cast<const char *>(a.h16);

  for (;;) {
    if (tid == 0) item_sh = atomicAdd(a.work, 1);
    __syncthreads();
    const int item = item_sh;
    __syncthreads();  // every thread has read item_sh before thread 0 may rewrite it
    if (item >= *a.n_items) return;
    const ScanItem it = a.items[item];
    if (SAMPLE && it.part != 0) continue;
    const int qcnt = it.qcnt, ng = (qcnt + 15) >> 4;
    const int ng2 = SAMPLE ? ng : (ng + 1) & ~1;  // MAIN runs groups in pairs (an odd count gets an empty one)

    // ---- prologue: query operands (LDS-DMA; a lane of piece (j, s) carries dims 32s + 8g .. +7 of
    // query 16j + c, the 16x16x32 B layout) and per-query scalars ----
    {
      const int npc = ng * KS;
      for (int p = w; p < (Q2 ? 2 : 1) * npc; p += SNW) {
        const int term = p >= npc ? 1 : 0, pp = p - term * npc;
        const int j = pp / KS, s = pp - j * KS;
        const int qi = min(16 * j + c, qcnt - 1);
        const _Float16 *src = (term ? a.bql : a.bq) + (size_t)(it.qbeg + qi) * D + 32 * s + 8 * g;
        glds<16>(src, bl_base + (uint32_t)((term * PIECES + pp) * 1024));
      }
      // records of every slot of the (even-padded) groups; an unused slot's threshold is NaN, so no
      // row is ever emitted for it (not even a +inf-meta row, whose y would reach a +inf threshold)
      for (int i = tid; i < ng2 * 16; i += 64 * SNW) {
        float2 v = make_float2(0.0f, __builtin_nanf(""));
        float cqv = 0.0f;
        int o = -1;
        if (i < qcnt) {
          const int pos = it.qbeg + i;
          const int slot = a.qlist[pos];
          const float2 fc = a.qsc[pos];
          const int q = slot / a.nparts;
          const float T = (!SAMPLE && a.thr) ? a.thr[q] + a.thr_bias : -INFINITY;
          v = make_float2(fc.x, lower_thr(T, fc.y));
          cqv = fc.y;
          o = SAMPLE ? q * a.nprobe + (slot % a.nparts) / a.cmax : slot + it.part;
        }
        qr[i] = make_float4(v.x, v.y, cqv, __int_as_float(o));
        cnt_l[i] = 0;
        flr_l[i] = 0u;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces landed
      __syncthreads();
    }

    const int r0 = it.row_begin;  // multiple of 32
    int nt = (it.row_end - r0 + 31) >> 5;
    if (SAMPLE) nt = min(nt, SAMPLE_TILES);
    const int rlim = (int)min((int64_t)it.row_end, (int64_t)a.row_limit);

    // tile t: A fragments (rows 16b + c, dims 32s + 8g .. +7) and the meta of rows 16b + 4g .. +3
    auto load = [&](int t, h8v (&A)[KS][2], f4v (&M)[2]) {
      const char *tb = hsrc + (size_t)(r0 / 32 + t) * TB + (g * 32 + c) * 16;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        A[s][0] = *reinterpret_cast<const h8v *>(tb + s * 2048);
        A[s][1] = *reinterpret_cast<const h8v *>(tb + s * 2048 + 256);
      }
      const size_t mo = (size_t)(r0 + 32 * t) + 4 * g;
      const f4v m0 = *reinterpret_cast<const f4v *>(a.meta + mo), m1 = *reinterpret_cast<const f4v *>(a.meta + mo + 16);
      const f4v x0 = *reinterpret_cast<const f4v *>(a.rsq16 + mo), x1 = *reinterpret_cast<const f4v *>(a.rsq16 + mo + 16);
      // the row's share of the error bound (stream_ub_terms): -inf (dead, NaN) and +inf (Inf) meta stay
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        M[0][i] = fmaf(a.kr, x0[i], m0[i]);
        M[1][i] = fmaf(a.kr, x1[i], m1[i]);
      }
      if constexpr (MET == IP) {
        const f4v n0 = *reinterpret_cast<const f4v *>(a.rsq + mo), n1 = *reinterpret_cast<const f4v *>(a.rsq + mo + 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          M[0][i] = fmaf(a.kx, n0[i], M[0][i]);
          M[1][i] = fmaf(a.kx, n1[i], M[1][i]);
        }
      }
    };
    // query group j's operands from LDS (one term: 4 x ds_read_b128 at D = 128; the split adds 4)
    auto read_b = [&](int j, h8v (&B)[KS], h8v (&B2)[KS]) {
      const char *bp = bl + j * KS * 1024 + lane * 16;
#pragma unroll
      for (int s = 0; s < KS; ++s) B[s] = *reinterpret_cast<const h8v *>(bp + s * 1024);
      if constexpr (Q2) {
#pragma unroll
        for (int s = 0; s < KS; ++s) B2[s] = *reinterpret_cast<const h8v *>(bp + PIECES * 1024 + s * 1024);
      }
    };
    // acc = rows x queries of the tile: two independent chains (16-row halves)
    auto mma = [&](const h8v (&A)[KS][2], const h8v (&B)[KS], const h8v (&B2)[KS], f4v (&acc)[2]) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[b][i] = 0.0f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (Q2) {  // small term first (filter16.hip)
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][0], B2[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][1], B2[s], acc[1], 0, 0, 0);
        }
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][0], B[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][1], B[s], acc[1], 0, 0, 0);
      }
    };
    // y = f acc + meta of query group j against the tile (8 values per lane)
    auto scores = [&](const h8v (&A)[KS][2], const float (&mr)[8], int j, float f, float (&y)[8]) {
      h8v bh[KS], bo[KS];
      read_b(j, bh, bo);
      f4v acc[2];
      mma(A, bh, bo, acc);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) y[4 * b + i] = fmaf(f, acc[b][i], mr[4 * b + i]);
    };
    auto row_terms = [&](const f4v (&M)[2], int t, float (&mr)[8]) {
      const int rt = r0 + 32 * t;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) mr[4 * b + i] = rt + 16 * b + 4 * g + i < rlim ? M[b][i] : -INFINITY;
    };

    if constexpr (SAMPLE) {
      // at most two tiles per wave: both stay in registers while every group is scored
      h8v A0[KS][2], A1[KS][2];
      f4v M0[2], M1[2];
      const bool h0 = w < nt, h1 = w + SNW < nt;
      if (h0) load(w, A0, M0);
      if (h1) load(w + SNW, A1, M1);
      float mr0[8], mr1[8];
      if (h0) row_terms(M0, w, mr0);
      if (h1) row_terms(M1, w + SNW, mr1);
      for (int j = 0; j < ng; ++j) {
        const int qi = 16 * j + c;
        const float4 rq = qr[qi];
        const float f = rq.x;
        float mx = -INFINITY;
        if (h0) {
          float y[8];
          scores(A0, mr0, j, f, y);
          mx = fmaxf(mx, max3f(max3f(y[0], y[1], y[2]), max3f(y[3], y[4], y[5]), fmaxf(y[6], y[7])));
        }
        if (h1) {
          float y[8];
          scores(A1, mr1, j, f, y);
          mx = fmaxf(mx, max3f(max3f(y[0], y[1], y[2]), max3f(y[3], y[4], y[5]), fmaxf(y[6], y[7])));
        }
        if (qi < qcnt) a.samp[(size_t)__float_as_int(rq.w) * SV + w * 4 + g] = mx + rq.z;
      }
    } else {
      // rows whose score can reach T_q -> the query's region of the part: the lane counts its passing
      // rows, reserves that many slots with ONE returning LDS atomic, then stores them (a region that
      // is full keeps the best score it had to drop as its floor)
      auto emit = [&](const float (&y)[8], const float4 rq, int qi, int rt) {
        uint32_t m = 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) m |= (y[e] >= rq.y ? 1u : 0u) << e;
        if (m == 0u) return;
        int slot = atomicAdd(&cnt_l[qi], __builtin_popcount(m));
        const size_t rb = (size_t)__float_as_int(rq.w) * a.cap;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (m & (1u << e)) {
            const float s = y[e] + rq.z;
            if (slot < a.cap) {
              a.cand_s[rb + slot] = s;
              a.cand_k[rb + slot] = a.key_base | (uint32_t)(rt + 16 * (e >> 2) + 4 * g + (e & 3));
            } else {
              atomicMax(&flr_l[qi], score_key(s));
            }
            ++slot;
          }
        }
      };
      // group j's scores from its accumulators (rq: the group's query record, read one group ahead);
      // the emit branch when a row of the wave can reach its query's T_q
      auto epi = [&](const f4v (&acc)[2], const float (&mr)[8], int j, const float4 rq, int rt) {
        float y[8];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i) y[4 * b + i] = fmaf(rq.x, acc[b][i], mr[4 * b + i]);
        const float mx = max3f(max3f(y[0], y[1], y[2]), max3f(y[3], y[4], y[5]), fmaxf(y[6], y[7]));
        if constexpr (AB) {  // measurement only (PYR_FILTER_ABLATE=64): no emission
          if (mx == 12345.0f) cnt_l[0] = 1;  // keep the scores live
          return;
        }
        // rare (about 1 group-tile in 4 at I1): the emit code is laid out off the fall-through path
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(mx >= rq.y) != 0ull, 0)) emit(y, rq, 16 * j + c, rt);
      };
      // one tile against every group, software-pipelined over pairs of groups with two fixed register
      // sets: group j + 1's record and operands are read while group j's MFMAs run (the record first,
      // so waiting for it never waits for operand reads issued after it), group j - 1's epilogue runs
      // behind group j's MFMAs.  The group count is even (a padded group has NaN thresholds) and the
      // reads ahead are unconditional (clamped): no exit or conditional read inside the pipeline, which
      // the compiler otherwise rotates into a one-group loop that waits for its reads at the back edge.
      auto tile = [&](const h8v (&A)[KS][2], const f4v (&M)[2], int t) {
        float mr[8];
        row_terms(M, t, mr);
        const int rt = r0 + 32 * t;
        h8v b0[KS], b1[KS], o0[KS], o1[KS];
        f4v a0[2], a1[2];
        float4 q0 = qr[c], q1 = q0, qp = q0;
        read_b(0, b0, o0);
        for (int j = 0; j < ng2; j += 2) {
          q1 = qr[16 * (j + 1) + c];
          read_b(j + 1, b1, o1);
          mma(A, b0, o0, a0);
          if (j > 0) epi(a1, mr, j - 1, qp, rt);
          const float4 qj = q0;
          const int jn = min(j + 2, ng2 - 1);
          q0 = qr[16 * jn + c];
          read_b(jn, b0, o0);
          mma(A, b1, o1, a1);
          epi(a0, mr, j, qj, rt);
          qp = q1;
        }
        epi(a1, mr, ng2 - 1, qp, rt);
      };
      // double-buffered tiles; the prefetch of tile t + 8 is unconditional (the last tile is re-read when
      // there is none): a conditional load makes the compiler's vmcnt accounting wait for the
      // prefetch itself before the current tile, which serialised every tile behind an HBM round trip
      h8v A0[KS][2], A1[KS][2];
      f4v M0[2], M1[2];
      int t = w;
      if (t < nt) load(t, A0, M0);
      while (t < nt) {
        load(min(t + SNW, nt - 1), A1, M1);
        tile(A0, M0, t);
        t += SNW;
        if (t >= nt) break;
        load(min(t + SNW, nt - 1), A0, M0);
        tile(A1, M1, t);
        t += SNW;
      }
      __syncthreads();
      for (int i = tid; i < qcnt; i += 64 * SNW) {
        const int o = __float_as_int(qr[i].w);
        a.cand_n[o] = min(cnt_l[i], a.cap);
        a.cand_f[o] = flr_l[i];
      }
    }
  }
}

// ---- 3. T_q = the R-th largest sample value (radix select over score keys, wselect.h) ----
// The sample holds min(len, 512) rows of each probed list, so about R / f rows of the probed lists
// reach T_q (f = the sampled fraction of the query's probed rows).  R adapts to f: the rows it
// guarantees (R) stay at least rmin, the rows it emits (~R / f) near et, R <= rmax -- short lists
// (f ~ 1) take R = rmax = K1 so the k-th row sits well above T_q, long ones R = rmin (I1: f ~ 0.05).
__global__ __launch_bounds__(256) void sselect_kernel(StreamSelectArgs a) {
  __shared__ int hist[4][256];
  __shared__ int buf[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  if (q >= a.nq) return;
  int K = a.rmax;
  if (a.rmin < a.rmax) {
    int64_t tot = 0, smp = 0;
    for (int p = lane; p < a.nprobe; p += 64) {
      const int l = a.probes[(size_t)q * a.nprobe + p];
      if (l < 0) continue;
      const int64_t len = a.le[l] - a.lb[l];
      tot += len;
      smp += min(len, (int64_t)(SAMPLE_TILES * 32));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      tot += __shfl_xor(tot, off);
      smp += __shfl_xor(smp, off);
    }
    const double f = tot > 0 ? (double)smp / (double)tot : 1.0;
    K = (int)fmin((double)a.rmax, fmax((double)a.rmin, ceil(a.et * f)));
  }
  const int n = a.n;
  if (n < K) {
    if (lane == 0) a.thr[q] = -INFINITY;
    return;
  }
  float cv[16];
  const uint32_t key = K <= 64 ? wave_kth_key_lm<16>(a.samp + (size_t)q * n, n, K, hist[w], buf[w], lane, cv)
                               : wave_kth_key<16>(a.samp + (size_t)q * n, n, K, hist[w], lane, cv);
  if (lane == 0) a.thr[q] = key_score(key);
}

// ---- 5. per query: the best KO emitted rows (+ floor placeholders), wave bitonic sort ----
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
// rank key: score desc, then storage key asc (~key); 0 = no entry
__device__ __forceinline__ uint64_t pack_cand(float s, uint32_t k) { return ((uint64_t)score_key(s) << 32) | (uint32_t)~k; }

__device__ __forceinline__ uint64_t sort64_desc(uint64_t v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j >= 1; j >>= 1) {
      const uint64_t o = shfl_xor64(v, j);
      const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == desc) ? (v > o ? v : o) : (v < o ? v : o);
    }
  return v;
}
__device__ __forceinline__ uint64_t merge64_desc(uint64_t v, int lane) {  // v bitonic -> sorted desc
#pragma unroll
  for (int j = 32; j >= 1; j >>= 1) {
    const uint64_t o = shfl_xor64(v, j);
    v = (lane & j) == 0 ? (v > o ? v : o) : (v < o ? v : o);
  }
  return v;
}

template <int KO>
__global__ __launch_bounds__(256) void cand_merge_kernel(CandMergeArgs m) {
  __shared__ int pre[4][MAX_PARTS + 1];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  if (q >= m.nq) return;
  const size_t sb = (size_t)q * m.nparts;
  int tot = 0;
  uint32_t fk = 0u;
  for (int base = 0; base < m.nparts; base += 64) {
    const int p = base + lane;
    int n = 0;
    if (p < m.nparts) {
      n = m.cand_n[sb + p];
      fk = max(fk, m.cand_f[sb + p]);
    }
    int x = n;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (p < m.nparts) pre[w][p] = tot + x - n;
    tot += __shfl(x, 63);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) fk = max(fk, (uint32_t)__shfl_xor((int)fk, off));
  float F = m.thr ? m.thr[q] : -INFINITY;
  if (fk != 0u) F = fmaxf(F, key_score(fk));
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint64_t cur = F > -INFINITY ? pack_cand(F, KEY_FLOOR) : 0ull;
  for (int base = 0; base < tot; base += 64) {
    const int idx = base + lane;
    uint64_t v = 0ull;
    if (idx < tot) {
      int lo = 0, hi = m.nparts;  // pre[lo] <= idx < pre[hi] (pre[nparts] = tot)
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pre[w][mid] <= idx) lo = mid;
        else hi = mid;
      }
      const size_t e = (sb + lo) * m.cap + (idx - pre[w][lo]);
      v = pack_cand(m.cand_s[e], m.cand_k[e]);
    }
    const uint64_t kth = shfl64(cur, KO - 1);
    if (!__builtin_amdgcn_ballot_w64(v > kth)) continue;
    v = sort64_desc(v, lane);
    const uint64_t r = shfl64(v, 63 - lane);
    cur = cur > r ? cur : r;
    cur = merge64_desc(cur, lane);
  }
  if (lane < KO) {
    float s = -INFINITY;
    int32_t k = -1;
    if (cur != 0ull) {
      s = key_score((uint32_t)(cur >> 32));
      const uint32_t kk = ~(uint32_t)cur;
      k = kk == KEY_FLOOR ? -2 : (int32_t)kk;
    }
    m.out_s[(size_t)q * KO + lane] = s;
    m.out_k[(size_t)q * KO + lane] = k;
  }
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }




template <int D, int MET, bool Q2>
void launch_stream_dm(const StreamArgs &a, int max_items, bool sample, hipStream_t st) {
  const int grid = std::max(1, std::min(max_items, device_cus()));
  if (sample) hipLaunchKernelGGL((stream16_kernel<D, MET, Q2, true>), dim3(grid), dim3(64 * SNW), 0, st, a);
  else if (a.ablate & 64) hipLaunchKernelGGL((stream16_kernel<D, MET, Q2, false, true>), dim3(grid), dim3(64 * SNW), 0, st, a);
  else hipLaunchKernelGGL((stream16_kernel<D, MET, Q2, false>), dim3(grid), dim3(64 * SNW), 0, st, a);
}

template <int D>
void launch_stream_d(const StreamArgs &a, int metric, int max_items, bool sample, hipStream_t st) {
  if (metric == L2) a.bql ? launch_stream_dm<D, L2, true>(a, max_items, sample, st)
                          : launch_stream_dm<D, L2, false>(a, max_items, sample, st);
  else a.bql ? launch_stream_dm<D, IP, true>(a, max_items, sample, st)
             : launch_stream_dm<D, IP, false>(a, max_items, sample, st);
}

}  // namespace

int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    cus = hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }
  return cus;
}

bool stream16_supported(int dim, int metric, int k1) {
  if (metric != L2 && metric != IP) return false;
  if (dim != 32 && dim != 64 && dim != 128) return false;
  return k1 >= 1 && k1 <= STREAM_KO;
}
int stream16_qmax(bool q2) { return q2 ? 256 : 512; }
int stream16_sample_values() { return SV; }

void launch_stream_prep(const StreamArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(max_items), dim3(256), 0, st, a); };
  switch (a.dim) {
    case 32: metric == L2 ? go(sprep_kernel<32, L2>) : go(sprep_kernel<32, IP>); return;
    case 64: metric == L2 ? go(sprep_kernel<64, L2>) : go(sprep_kernel<64, IP>); return;
    default: metric == L2 ? go(sprep_kernel<128, L2>) : go(sprep_kernel<128, IP>); return;
  }
}

void launch_stream_scan(const StreamArgs &a, int metric, int max_items, bool sample, hipStream_t st) {
  if (max_items <= 0) return;
  switch (a.dim) {
    case 32: launch_stream_d<32>(a, metric, max_items, sample, st); return;
    case 64: launch_stream_d<64>(a, metric, max_items, sample, st); return;
    default: launch_stream_d<128>(a, metric, max_items, sample, st); return;
  }
}

void stream_ub_terms(int dim, int metric, double c_bf, double c_err, double c_abs, StreamArgs &a) {
  const double u = 5.9604644775390625e-8;         // 2^-24
  const double t = 1.4551915228366852e-11 * std::sqrt((double)dim);  // the query's fp16 subnormals, 2^-36 sqrt(D)
  const double g = (dim / 8.0 + 8.0) * u;         // the reference's own sum (refine_kernel)
  const double up = 1.0 + 1e-3;                   // the fp32 evaluation of the terms themselves
  if (metric == L2) {
    // c_bf u A X + c_err u (A + X)^2 + c_abs A + 2 t A X, and g |q - x|^2 <= g (A + X)^2
    const double k = (c_bf * u / 2.0 + 2.0 * c_err * u + t + 2.0 * g) * up + 8.0 * u;
    a.kr = (float)k;
    a.kq = (float)k;
    a.kqa = (float)(c_abs * up);
    a.kx = 0.0f;
    a.kqc = 0.0f;
  } else {
    // c_bf u |q| X + c_err u |q| X + c_abs |q| + t |q| X + c_err u |q||c| + g |q||x|
    const double k = ((c_bf + c_err) * u + t) / 2.0 * up + 8.0 * u;
    a.kr = (float)k;
    a.kq = (float)(k + g / 2.0 * up);
    a.kx = (float)(g / 2.0 * up + 8.0 * u);
    a.kqa = (float)(c_abs * up);
    a.kqc = (float)(c_err * u * up);
  }
}

namespace {
__global__ void row_terms_kernel(const float *meta, const float *rsq16, const float *rsq, int64_t n, int met, float kr,
                                 float kx, float *out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = fmaf(kr, rsq16[i], meta[i]);
    if (met == IP) v = fmaf(kx, rsq[i], v);
    out[i] = v;
  }
}
}  // namespace

void launch_row_terms(const float *meta, const float *rsq16, const float *rsq, int64_t n, int metric, float kr,
                      float kx, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(row_terms_kernel, dim3(gblk(n)), dim3(256), 0, st, meta, rsq16, rsq, n, metric, kr, kx, out);
}

void launch_stream_select(const StreamSelectArgs &a, hipStream_t st) {
  if (a.nq <= 0) return;
  hipLaunchKernelGGL(sselect_kernel, dim3(nblk(a.nq, 4)), dim3(256), 0, st, a);
}

void launch_cand_merge(const CandMergeArgs &m, hipStream_t st) {
  if (m.nq <= 0) return;
  hipLaunchKernelGGL(cand_merge_kernel<STREAM_KO>, dim3(nblk(m.nq, 4)), dim3(256), 0, st, m);
}

}  // namespace pyr
