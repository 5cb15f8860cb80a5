// sample16.hip -- the stream scan's threshold step and candidate merge (gfx950).
//
// The stream-and-emit scan (scan.hip) emits every row whose approximate score can reach its query's
// threshold T_q.  This file holds the steps around it:
//
//  1. sprep_q_kernel (round 5; query-major over the positions the work lists recorded) / sprep_kernel (list-major;
//     list-sharded ranks): per (list, query) pair the query's residual q - c
//     (L2) or q (IP), scaled by a power of two and rounded to fp16, plus the score factor f and the
//     per-(query, list) constant cq -- once, instead of in every block that scans the list.
//  2. sample16_kernel (since round 5 the A/B path, PYR_SAMPLE16=1: the sample runs on scan.hip's scan_kernel in
//     its SMP mode after sprep; both write the same samp layout): persistent blocks (one per CU, 8 waves) take the chunk-0 work items (list,
//     <= 512 queries) from a counter.  The item's query operands go to LDS (LDS-DMA, 128 KiB at
//     D = 128); each wave holds two of the list's first 16 tiles in registers and scores them against
//     every query group of the item on v_mfma_f32_16x16x32_f16 with the ROWS as the A operand (lane
//     (c, g) gets query c's scores of rows 4g..4g+3 of each 16-row half); each (wave, lane group) keeps
//     the best score it saw per query -> 32 values per (query, probe), each the bound of a distinct row.
//     (Round 3's list scan was this kernel's main mode; scan.hip replaced it, and a scan.hip-shaped
//     sample -- one wave per 32-query group, or the tiles staged in LDS -- measured slower at I1: 0.29 and
//     0.19-0.26 ms against 0.15 ms, profiles/r4_scan/sample_lds_attempt.log.)
//  3. sselect_kernel: T_q = the R-th largest of the query's sample values (radix select).
//  4. cand_merge_kernel: per query the best KO (64) of its emitted rows (its query-major buffer, read
//     64 contiguous entries at a time), ranked with KO copies of the floor placeholder max(T_q, floor)
//     (KEY_FLOOR): every row left out scores <= the merged KO-th.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

#include "kernels.h"

namespace pyr {
namespace {

#include "f16util.h"
#include "wselect.h"
#include "candmerge.h"

constexpr int SNW = 8;         // waves per stream block
constexpr int SV = SNW * 4;    // sample values per (query, probe)
constexpr int SAMPLE_TILES = 2 * SNW;

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }

// ---- 1. query operands per (list, query) pair ----
// A lane group of D / 8 lanes per query (8 dims a lane, the centroid's 8 dims held in registers for
// the whole list), 64 / (D / 8) queries per wave per pass.  A block's loads are a chain (item -> position
// -> query row), so each wave issues the loads of SPREP_U passes before it computes any of them, and an
// item's queries are split over SPREP_SPLIT(D) blocks: more chains in flight, fewer turns each.
// (Round 4: one pass per turn and D / 16 blocks per item, 34-43 us at I1: latency-bound.)
template <int D>
constexpr int SPREP_SPLIT = D >= 128 ? 2 : 1;
constexpr int SPREP_U = 4;
template <int D, int MET>
__device__ void sprep_unit(const StreamArgs &a, int item, int part);

// grid-stride over (item, part) units up to the device item count: the grid is sized for the most items a
// batch can have, and a list-sharded rank's batch has far fewer (only its own lists get items)
template <int D, int MET>
__global__ __launch_bounds__(256) void sprep_kernel(StreamArgs a) {
  constexpr int SPLIT = SPREP_SPLIT<D>;
  const int64_t units = (int64_t)(*a.n_items) * SPLIT;
  for (int64_t u = blockIdx.x; u < units; u += gridDim.x) sprep_unit<D, MET>(a, (int)(u / SPLIT), (int)(u % SPLIT));
}

template <int D, int MET>
__device__ void sprep_unit(const StreamArgs &a, int item, int part) {
  constexpr int SPLIT = SPREP_SPLIT<D>, U = SPREP_U;
  const ScanItem it = a.items[item];
  if (it.part != 0) return;  // chunk-0 items cover every qlist position of their list once
  constexpr int LQ = D / 8, QW = 64 / LQ, STEP = 4 * QW * SPLIT;  // STEP: queries between a wave's passes
  if (4 * QW * part >= it.qcnt) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane % LQ, qsl = lane / LQ;
  const float4 *cp = reinterpret_cast<const float4 *>(a.cents + (size_t)it.list * D + 8 * sub);
  const float4 c0 = cp[0], c1 = cp[1];
  const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  for (int qb = QW * w + 4 * QW * part; qb < it.qcnt; qb += STEP * U) {
    int pos[U], q[U];
    float4 q0[U], q1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qi = qb + u * STEP + qsl;
      pos[u] = it.qbeg + (qi < it.qcnt ? qi : 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = a.qlist[pos[u]] / a.nparts;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)q[u] * D + 8 * sub);
      q0[u] = qp[0];
      q1[u] = qp[1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool act = qb + u * STEP + qsl < it.qcnt;
      const float qv[8] = {q0[u].x, q0[u].y, q0[u].z, q0[u].w, q1[u].x, q1[u].y, q1[u].z, q1[u].w};
      float r[8], cq = 0.0f, amax = 0.0f, q2 = 0.0f, c2 = 0.0f;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        if (MET == L2) {
          r[d] = qv[d] - cv[d];
          cq += r[d] * r[d];
        } else {
          r[d] = qv[d];
          cq += qv[d] * cv[d];
          q2 += qv[d] * qv[d];
          c2 += cv[d] * cv[d];
        }
        amax = fmaxf(amax, fabsf(r[d]));
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
        h8v hv;
#pragma unroll
        for (int d = 0; d < 8; ++d) hv[d] = (_Float16)(r[d] * sq);  // the scaling is exact (a power of two)
        *reinterpret_cast<h8v *>(a.bq + (size_t)pos[u] * D + 8 * sub) = hv;
        if (sub == 0)
          a.qsc[pos[u]] = make_float2((MET == L2 ? 2.0f : 1.0f) / (sq * a.sx), (MET == L2 ? -cq : cq) + ep);
      }
    }
  }
}

// The same operands query-major, when the work lists recorded each (query, probe)'s position (StreamArgs::qpos):
// one wave per query, lane group g of D / 8 lanes takes probes g, g + QW, ...  The query's dims are read
// once and stay in registers across its probes, and the centroids (nlist x D x 4 B) stay L2-resident; the
// list-major pass above re-reads a query row per (list, query) pair: at I1, 10,000 x 32 rows of 512 B
// against L2s of 4 MiB per XCD.  Same arithmetic, same bq / qsc.
template <int D, int MET>
__global__ __launch_bounds__(256) void sprep_q_kernel(StreamArgs a) {
  constexpr int LQ = D / 8, QW = 64 / LQ, PU = 32 / QW > 0 ? 32 / QW : 1;  // probes per lane group per turn
  const int lane = threadIdx.x & 63, sub = lane % LQ, g = lane / LQ;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)q * D + 8 * sub);
  const float4 q0 = qp[0], q1 = qp[1];
  const float qv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  for (int p0 = 0; p0 < a.nprobe; p0 += QW * PU) {
    int pos[PU], lst[PU];
    float4 c0[PU], c1[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int p = p0 + u * QW + g;
      const bool ok = p < a.nprobe;
      pos[u] = ok ? a.qpos[(size_t)q * a.nprobe + p] : -1;
      lst[u] = ok ? a.probes[(size_t)q * a.nprobe + p] : -1;
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      // (a position a list-sharded rank dropped, -1, loads nothing: most of its batch's pairs)
      const float4 *cp = reinterpret_cast<const float4 *>(a.cents + (size_t)max(lst[u], 0) * D + 8 * sub);
      const bool use = pos[u] >= 0 && lst[u] >= 0;
      c0[u] = use ? cp[0] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      c1[u] = use ? cp[1] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const float cv[8] = {c0[u].x, c0[u].y, c0[u].z, c0[u].w, c1[u].x, c1[u].y, c1[u].z, c1[u].w};
      float r[8], cq = 0.0f, amax = 0.0f, q2 = 0.0f, c2 = 0.0f;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        if (MET == L2) {
          r[d] = qv[d] - cv[d];
          cq += r[d] * r[d];
        } else {
          r[d] = qv[d];
          cq += qv[d] * cv[d];
          q2 += qv[d] * qv[d];
          c2 += cv[d] * cv[d];
        }
        amax = fmaxf(amax, fabsf(r[d]));
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
      float ep = 0.0f;  // (as sprep_unit)
      if (MET == L2) {
        ep = a.kq * cq + a.kqa * sqrtf(cq);
      } else {
        const float qn = sqrtf(q2);
        ep = a.kq * q2 + a.kqa * qn + a.kqc * qn * sqrtf(c2);
      }
      const float sq = pow2_scale(amax);
      if (lst[u] >= 0 && pos[u] >= 0) {
        h8v hv;
#pragma unroll
        for (int d = 0; d < 8; ++d) hv[d] = (_Float16)(r[d] * sq);
        *reinterpret_cast<h8v *>(a.bq + (size_t)pos[u] * D + 8 * sub) = hv;
        if (sub == 0)
          a.qsc[pos[u]] = make_float2((MET == L2 ? 2.0f : 1.0f) / (sq * a.sx), (MET == L2 ? -cq : cq) + ep);
      }
    }
  }
}

// ---- 2. the sample ----
template <int D, int MET>
__global__ __launch_bounds__(64 * SNW, 1) void sample16_kernel(StreamArgs a) {
  constexpr int KS = D / 32;            // 16x16x32 k-steps
  constexpr int TB = 64 * D;            // h16 bytes per 32-row tile
  constexpr int QMAX = 512;             // queries per item
  constexpr int PIECES = QMAX / 16 * KS;
  __shared__ __attribute__((aligned(16))) char bl[PIECES * 1024];
  __shared__ float4 qr[QMAX];     // per query slot: {f, -, cq (score = y + cq), sample row as int bits}
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
    if (it.part != 0) continue;  // chunk-0 items cover every (list, query) pair once
    const int qcnt = it.qcnt, ng = (qcnt + 15) >> 4;

    // prologue: query operands (LDS-DMA; a lane of piece (j, s) carries dims 32s + 8g .. +7 of query
    // 16j + c, the 16x16x32 B layout) and per-query scalars
    {
      const int npc = ng * KS;
      for (int p = w; p < npc; p += SNW) {
        const int j = p / KS, s = p - j * KS;
        const int qi = min(16 * j + c, qcnt - 1);
        glds<16>(a.bq + (size_t)(it.qbeg + qi) * D + 32 * s + 8 * g, bl_base + (uint32_t)(p * 1024));
      }
      for (int i = tid; i < ng * 16; i += 64 * SNW) {
        float f = 0.0f, cqv = 0.0f;
        int o = -1;
        if (i < qcnt) {
          const int pos = it.qbeg + i;
          const int slot = a.qlist[pos];
          const float2 fc = a.qsc[pos];
          f = fc.x;
          cqv = fc.y;
          o = (slot / a.nparts) * a.nprobe + (slot % a.nparts) / a.cmax;
        }
        qr[i] = make_float4(f, 0.0f, cqv, __int_as_float(o));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces landed
      __syncthreads();
    }

    const int r0 = it.row_begin;  // multiple of 32
    const int nt = min((it.row_end - r0 + 31) >> 5, SAMPLE_TILES);
    const int rlim = (int)min((int64_t)it.row_end, (int64_t)a.row_limit);

    // tile t: A fragments (rows 16b + c, dims 32s + 8g .. +7) and the row terms of rows 16b + 4g .. +3
    auto load = [&](int t, h8v (&A)[KS][2], f4v (&M)[2]) {
      const char *tb = hsrc + (size_t)(r0 / 32 + t) * TB + (g * 32 + c) * 16;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        A[s][0] = *reinterpret_cast<const h8v *>(tb + s * 2048);
        A[s][1] = *reinterpret_cast<const h8v *>(tb + s * 2048 + 256);
      }
      const size_t mo = (size_t)(r0 + 32 * t) + 4 * g;
      M[0] = *reinterpret_cast<const f4v *>(a.mub + mo);
      M[1] = *reinterpret_cast<const f4v *>(a.mub + mo + 16);
    };
    // y = f acc + row term of query group j against the tile (8 values per lane)
    auto scores = [&](const h8v (&A)[KS][2], const float (&mr)[8], int j, float f, float (&y)[8]) {
      const char *bp = bl + j * KS * 1024 + lane * 16;
      h8v B[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) B[s] = *reinterpret_cast<const h8v *>(bp + s * 1024);
      f4v acc[2] = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][0], B[s], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][1], B[s], acc[1], 0, 0, 0);
      }
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

template <int KO>
__global__ __launch_bounds__(256) void cand_merge_kernel(CandMergeArgs m) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  if (q >= m.nq) return;
  const uint64_t cur = cand_merge_wave<KO>(m, q, lane);
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

bool sample16_supported(int dim, int metric) { return (metric == L2 || metric == IP) && (dim == 32 || dim == 64 || dim == 128); }

void launch_sample16(const StreamArgs &a, int metric, int max_items, hipStream_t st, bool prep_only) {
  if (max_items <= 0) return;
  const int split = a.dim == 32 ? SPREP_SPLIT<32> : a.dim == 64 ? SPREP_SPLIT<64> : SPREP_SPLIT<128>;
  // at most 4 blocks per CU of the grid-stride units (I1: 3.3k items x 8 units; a rank's share of a sharded batch
  // holds far fewer)
  const int64_t pg = std::min<int64_t>((int64_t)max_items * split, 8 * (int64_t)device_cus());
  auto prep = [&](auto kern) { hipLaunchKernelGGL(kern, dim3((unsigned)pg), dim3(256), 0, st, a); };
  // query-major when the work lists recorded the positions (PYR_SPREP_Q=0: the list-major pass; A/B only)
  const bool qmaj = !(knob("PYR_SPREP_Q") && atoi(knob("PYR_SPREP_Q")) == 0);
  if (a.qpos && qmaj && a.nq > 0) {
    const dim3 qg((unsigned)((a.nq + 3) / 4));
    auto prepq = [&](auto kern) { hipLaunchKernelGGL(kern, qg, dim3(256), 0, st, a); };
    auto samp2 = [&](auto kern) {
      if (!prep_only) hipLaunchKernelGGL(kern, dim3(std::max(1, std::min(max_items, device_cus()))), dim3(64 * SNW), 0, st, a);
    };
    switch (a.dim) {
      case 32:
        metric == L2 ? prepq(sprep_q_kernel<32, L2>) : prepq(sprep_q_kernel<32, IP>);
        metric == L2 ? samp2(sample16_kernel<32, L2>) : samp2(sample16_kernel<32, IP>);
        return;
      case 64:
        metric == L2 ? prepq(sprep_q_kernel<64, L2>) : prepq(sprep_q_kernel<64, IP>);
        metric == L2 ? samp2(sample16_kernel<64, L2>) : samp2(sample16_kernel<64, IP>);
        return;
      default:
        metric == L2 ? prepq(sprep_q_kernel<128, L2>) : prepq(sprep_q_kernel<128, IP>);
        metric == L2 ? samp2(sample16_kernel<128, L2>) : samp2(sample16_kernel<128, IP>);
        return;
    }
  }
  const dim3 grid(std::max(1, std::min(max_items, device_cus())));
  auto samp = [&](auto kern) {
    if (!prep_only) hipLaunchKernelGGL(kern, grid, dim3(64 * SNW), 0, st, a);
  };
  switch (a.dim) {
    case 32:
      metric == L2 ? prep(sprep_kernel<32, L2>) : prep(sprep_kernel<32, IP>);
      metric == L2 ? samp(sample16_kernel<32, L2>) : samp(sample16_kernel<32, IP>);
      return;
    case 64:
      metric == L2 ? prep(sprep_kernel<64, L2>) : prep(sprep_kernel<64, IP>);
      metric == L2 ? samp(sample16_kernel<64, L2>) : samp(sample16_kernel<64, IP>);
      return;
    default:
      metric == L2 ? prep(sprep_kernel<128, L2>) : prep(sprep_kernel<128, IP>);
      metric == L2 ? samp(sample16_kernel<128, L2>) : samp(sample16_kernel<128, IP>);
      return;
  }
}

// measurement only (scripts/bound_slack.py): PYR_EB_<BF|ERR|ABS|G|T> scale one constant of the bound, to find
// how far each could shrink before some row's bound falls below its exact score (results may then differ)
static double eb_scale(const char *name) {
  const char *e = knob(name);
  return e ? atof(e) : 1.0;
}
void stream_ub_terms(int dim, int metric, double c_bf, double c_err, double c_abs, StreamArgs &a) {
  const double u = 5.9604644775390625e-8;         // 2^-24
  c_bf *= eb_scale("PYR_EB_BF");
  c_err *= eb_scale("PYR_EB_ERR");
  c_abs *= eb_scale("PYR_EB_ABS");
  // the query's fp16 subnormals, 2^-36 sqrt(D)
  const double t = 1.4551915228366852e-11 * std::sqrt((double)dim) * eb_scale("PYR_EB_T");
  const double g = (dim / 8.0 + 8.0) * u * eb_scale("PYR_EB_G");  // the reference's own sum (refine_kernel)
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
