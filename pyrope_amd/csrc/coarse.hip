// coarse.hip -- the IVF coarse step as a dense score matrix + per-query selection (gfx950).
//
// IvfFlatVectorIndex.Search (:186-198) and IvfPqVectorIndex.Search (:141-150) score every
// centroid with ComputeScore (the safe VectorMath forms: one 8-lane accumulator, horizontal
// tree, then the scalar tail) and keep the first nprobe of the descending sort.  With nlist of
// ~1k the top-k-insertion scan of kernels.hip spends its time inserting (nprobe of every
// chunk's few dozen centroids enter the lists), so here the step is split:
//   coarse_scores_kernel  every (query, centroid) score, exact reference order, 32 x 32 tiles
//                         from LDS, 2 x 2 pairs per thread (8-lane accumulators each);
//   coarse_select_kernel  one wave per query: the row in LDS, nprobe rounds of a wave-wide
//                         argmax by (score desc, centroid asc), i.e. the same ranking.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cfloat>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"

namespace pyr {
namespace {

#include "wselect.h"

constexpr int CT = 32;  // queries / centroids per tile

__device__ __forceinline__ float hsum8(const float *v) {
  float lo = (v[0] + v[1]) + (v[2] + v[3]);
  float hi = (v[4] + v[5]) + (v[6] + v[7]);
  return lo + hi;
}

// out[q][c] = ComputeScore(query q, centroid c).  Block: CT queries x CT centroids, 256
// threads, thread (ty, tx) -> queries 2ty, 2ty+1 x centroids 2tx, 2tx+1.  Dimensions stream
// through LDS KT at a time (KT % 8 == 0), so the 8-lane accumulation order is unchanged.
constexpr int KT = 128;
constexpr int KTP = KT + 1;  // odd row stride: the 16 threads of a row read different banks

template <int MET>
__global__ __launch_bounds__(256) void coarse_scores_kernel(const float *q, const float *c, const float *qn,
                                                            const float *cn, int64_t nq, int nc, int D, float *out) {
  __shared__ float qs[CT * KTP], cs[CT * KTP];
  const int64_t q0 = (int64_t)blockIdx.y * CT;
  const int c0 = blockIdx.x * CT;
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  const float *qa = qs + (2 * ty) * KTP, *qb = qa + KTP;
  const float *ca = cs + (2 * tx) * KTP, *cb = ca + KTP;
  float acc[4][8];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[p][l] = 0.0f;
  const int D8 = D & ~7;
  float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int d0 = 0; d0 < D; d0 += KT) {
    const int kt = min(KT, D - d0);
    __syncthreads();  // the previous tile is consumed
    for (int e = tid; e < CT * kt; e += 256) {
      const int r = e / kt, d = e - r * kt;
      qs[r * KTP + d] = q0 + r < nq ? q[(size_t)(q0 + r) * D + d0 + d] : 0.0f;
      cs[r * KTP + d] = c0 + r < nc ? c[(size_t)(c0 + r) * D + d0 + d] : 0.0f;
    }
    __syncthreads();
    const int g8 = min(kt, D8 - d0);  // full 8-groups of this tile
    for (int i = 0; i < g8; i += 8) {  // VectorMath.cs:8-70, one Vector accumulator
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const float x0 = qa[i + l], x1 = qb[i + l], y0 = ca[i + l], y1 = cb[i + l];
        if (MET == L2) {
          const float d00 = x0 - y0, d01 = x0 - y1, d10 = x1 - y0, d11 = x1 - y1;
          acc[0][l] = acc[0][l] + d00 * d00;
          acc[1][l] = acc[1][l] + d01 * d01;
          acc[2][l] = acc[2][l] + d10 * d10;
          acc[3][l] = acc[3][l] + d11 * d11;
        } else {
          acc[0][l] = acc[0][l] + x0 * y0;
          acc[1][l] = acc[1][l] + x0 * y1;
          acc[2][l] = acc[2][l] + x1 * y0;
          acc[3][l] = acc[3][l] + x1 * y1;
        }
      }
    }
    if (d0 + kt >= D) {  // last tile: horizontal sums, then the scalar tail (it lies in this tile)
#pragma unroll
      for (int p = 0; p < 4; ++p) s[p] = D8 > 0 ? 0.0f + hsum8(acc[p]) : 0.0f;
      for (int i = D8 - d0; i < kt; ++i) {
        const float x0 = qa[i], x1 = qb[i], y0 = ca[i], y1 = cb[i];
        if (MET == L2) {
          const float d00 = x0 - y0, d01 = x0 - y1, d10 = x1 - y0, d11 = x1 - y1;
          s[0] = s[0] + d00 * d00;
          s[1] = s[1] + d01 * d01;
          s[2] = s[2] + d10 * d10;
          s[3] = s[3] + d11 * d11;
        } else {
          s[0] = s[0] + x0 * y0;
          s[1] = s[1] + x0 * y1;
          s[2] = s[2] + x1 * y0;
          s[3] = s[3] + x1 * y1;
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int64_t qi = q0 + 2 * ty + (p >> 1);
    const int ci = c0 + 2 * tx + (p & 1);
    if (qi >= nq || ci >= nc) continue;
    float v;
    if (MET == L2) v = -s[p];
    else if (MET == IP) v = s[p];
    else {  // Cosine (VectorMath.cs:102-109): 0 when either norm < 1e-6
      const float a = qn[qi], b = cn[ci];
      v = (a < 1e-6f || b < 1e-6f) ? 0.0f : s[p] / (a * b);
    }
    out[qi * nc + ci] = v;
  }
}

// order-preserving 64-bit key: higher = better (score desc, centroid asc)
__device__ __forceinline__ uint64_t rank_key(float s, int c) {
  return ((uint64_t)score_key(s) << 32) | (uint32_t)(0x7FFFFFFF - c);
}

__global__ __launch_bounds__(256) void coarse_select_kernel(const float *scores, int64_t nq, int nc, int nprobe,
                                                            int wpb, int32_t *probes) {
  extern __shared__ float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * wpb + w;
  if (q >= nq) return;  // no block barrier below
  uint64_t *row = reinterpret_cast<uint64_t *>(sm) + (size_t)w * nc;
  for (int c = lane; c < nc; c += 64) row[c] = rank_key(scores[q * nc + c], c);
  __builtin_amdgcn_wave_barrier();
  for (int p = 0; p < nprobe; ++p) {
    uint64_t best = 0;
    int bi = -1;
    for (int c = lane; c < nc; c += 64) {
      const uint64_t v = row[c];
      if (v > best) {
        best = v;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint64_t ov = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > best) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      probes[q * nprobe + p] = bi;
      row[bi] = 0;  // taken (every real key is > 0)
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// One pass instead of nprobe: each lane keeps the P best keys of its share of the row (every 64th
// centroid) sorted in registers, then P rounds pop the wave's best head -- the same ranking, O(nlist)
// reads instead of O(nprobe x nlist).  P (>= nprobe) is a compile-time list length.
template <int P>
__device__ __forceinline__ void key_insert(uint64_t (&l)[P], uint64_t v) {
  bool b[P];
#pragma unroll
  for (int j = 0; j < P; ++j) b[j] = v > l[j];
#pragma unroll
  for (int j = P - 1; j >= 1; --j) l[j] = b[j - 1] ? l[j - 1] : (b[j] ? v : l[j]);
  l[0] = b[0] ? v : l[0];
}

// the wave's selection over one score row (every lane holds the P best keys of its 64th share)
template <int P>
__device__ __forceinline__ void select_row_reg(const float *row, int nc, int nprobe, int32_t *out, int lane) {
  uint64_t l[P];
#pragma unroll
  for (int j = 0; j < P; ++j) l[j] = 0;  // below every real key
  constexpr int U = 8;  // independent loads in flight per lane before the (branchy) insertions
  for (int c0 = lane; c0 < nc; c0 += 64 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = c0 + 64 * u < nc ? row[c0 + 64 * u] : 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (c0 + 64 * u >= nc) break;
      const uint64_t kv = rank_key(v[u], c0 + 64 * u);
      if (kv > l[P - 1]) key_insert<P>(l, kv);
    }
  }
  for (int p = 0; p < nprobe; ++p) {
    uint64_t best = l[0];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint64_t ov = __shfl_xor(best, o);
      best = ov > best ? ov : best;
    }
    if (l[0] == best) {  // keys are unique (centroid index in the low half): one lane pops its head
#pragma unroll
      for (int j = 0; j < P - 1; ++j) l[j] = l[j + 1];
      l[P - 1] = 0;
      if (best != 0) out[p] = 0x7FFFFFFF - (int)(uint32_t)best;
    }
    if (best == 0 && lane == 0) out[p] = -1;  // fewer centroids than nprobe (as the LDS kernel)
  }
}

template <int P>
__global__ __launch_bounds__(256) void coarse_select_reg_kernel(const float *scores, int64_t nq, int nc, int nprobe,
                                                                int32_t *probes) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  if (q >= nq) return;  // no block barrier below
  select_row_reg<P>(scores + q * nc, nc, nprobe, probes + q * nprobe, lane);
}

// ---- the coarse ranking on the matrix cores (L2 / IP, D % 16 == 0) ----
// 1. coarse_approx_kernel: fp32 MFMA dot products (v_mfma_f32_16x16x4_f32), one wave per 32 queries x 32
//    centroids; approx = 2 q.c - |c|^2 (L2: the score + |q|^2) or q.c (IP).  The k order inside a
//    16-dim block is permuted the same way for both operands (lane group h, step j -> dim 16s + 4h + j),
//    so every lane feeds its MFMAs from float4 loads.
// 2. coarse_pick_kernel: the nprobe-th largest approximate score aP, the exact ComputeScore of every
//    centroid within 2E of it (E bounds |approx - (score + |q|^2)|) and the first nprobe of those.
// 3. coarse_select_list_kernel: the dense exact ranking of the queries the pick could not settle.
// the search's counters zeroed by the approximate-score launch (its 2D grid, one word per thread at most):
// the stream scan's WordFill without a fill_words launch of its own (engine.cpp stream_counters_fill)
__device__ __forceinline__ void grid_word_fill(const WordFill &f) {
  const int64_t nt = (int64_t)gridDim.x * gridDim.y * blockDim.x;
  const int64_t t = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  int64_t base = 0;
  for (int r = 0; r < f.cnt; ++r) {
    for (int64_t e = t - base; e < f.n[r]; e += nt)
      if (e >= 0) f.p[r][e] = f.v[r];
    base += f.n[r];
  }
}

template <int MET, int DT>
__global__ __launch_bounds__(64) void coarse_approx_kernel(const float *q, const float *c, const float *c2, int64_t nq,
                                                           int nc, int Dr, float *out, int32_t *zero, WordFill zf) {
  if (zero && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *zero = 0;  // the pick's failure count
  grid_word_fill(zf);
  const int D = DT > 0 ? DT : Dr;  // a compile-time D unrolls the loop: every operand load is issued up front
  constexpr int UNS = DT > 0 ? DT / 16 : 1;
  const int64_t q0 = (int64_t)blockIdx.y * 32;
  const int c0 = blockIdx.x * 32;
  const int l = threadIdx.x, r = l & 15, h = l >> 4;
  const float4 *qa[2], *cb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    qa[i] = reinterpret_cast<const float4 *>(q + (size_t)min(q0 + 16 * i + r, nq - 1) * D) + h;
    cb[i] = reinterpret_cast<const float4 *>(c + (size_t)min(c0 + 16 * i + r, nc - 1) * D) + h;
  }
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll UNS
  for (int s = 0; s < D / 16; ++s) {
    const float4 a0 = qa[0][4 * s], a1 = qa[1][4 * s], b0 = cb[0][4 * s], b1 = cb[1][4 * s];
    const float av[2][4] = {{a0.x, a0.y, a0.z, a0.w}, {a1.x, a1.y, a1.z, a1.w}};
    const float bv[2][4] = {{b0.x, b0.y, b0.z, b0.w}, {b1.x, b1.y, b1.z, b1.w}};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][j], bv[t][j], acc[i][t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ci = c0 + 16 * t + r;
    if (ci >= nc) continue;
    const float cc = MET == L2 ? c2[ci] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t qi = q0 + 16 * i + 4 * h + g;
        if (qi < nq) out[qi * nc + ci] = MET == L2 ? 2.0f * acc[i][t][g] - cc : acc[i][t][g];
      }
  }
}

// The same approximate scores with both tiles staged in LDS: a 256-thread block computes 64 queries x 64
// centroids (wave w: the 32 x 32 quadrant (w & 1, w >> 1)), the rows arriving as coalesced 512-B row
// loads, KT = 64 dims at a time (34 KB of LDS: four blocks per CU), in a row stride of KT + 4 floats (the 16 rows a 16-lane group of
// ds_read_b128 touches start 4 banks apart: conflict-free).  Each wave then issues exactly the MFMA
// sequence of coarse_approx_kernel (same operands, same k order), so the approximate scores are the same
// bits; the tiles cross L2 once per block instead of once per wave, as whole rows.
constexpr int AKT = 64, AKS = AKT + 4;
template <int MET>
__global__ __launch_bounds__(256) void coarse_approx_lds_kernel(const float *q, const float *c, const float *c2,
                                                                int64_t nq, int nc, int D, float *out, int32_t *zero,
                                                                WordFill zf) {
  __shared__ __attribute__((aligned(16))) float qs[64 * AKS], cs[64 * AKS];
  if (zero && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *zero = 0;  // the pick's failure count
  grid_word_fill(zf);
  const int64_t q0 = (int64_t)blockIdx.y * 64;
  const int c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, r = l & 15, h = l >> 4;
  const int wq = 32 * (w & 1), wc = 32 * (w >> 1);
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int d0 = 0; d0 < D; d0 += AKT) {
    const int kt = min(AKT, D - d0), k4 = kt / 4;
    __syncthreads();  // the previous chunk is consumed
    for (int e = tid; e < 64 * k4; e += 256) {
      const int row = e / k4, col = 4 * (e - row * k4);
      const float4 qv = *reinterpret_cast<const float4 *>(q + (size_t)min(q0 + row, nq - 1) * D + d0 + col);
      const float4 cv = *reinterpret_cast<const float4 *>(c + (size_t)min(c0 + row, nc - 1) * D + d0 + col);
      *reinterpret_cast<float4 *>(qs + row * AKS + col) = qv;
      *reinterpret_cast<float4 *>(cs + row * AKS + col) = cv;
    }
    __syncthreads();
    const float *qa[2] = {qs + (wq + r) * AKS + 4 * h, qs + (wq + 16 + r) * AKS + 4 * h};
    const float *cb[2] = {cs + (wc + r) * AKS + 4 * h, cs + (wc + 16 + r) * AKS + 4 * h};
#pragma unroll 2
    for (int s = 0; s < kt / 16; ++s) {
      const float4 a0 = *reinterpret_cast<const float4 *>(qa[0] + 16 * s), a1 = *reinterpret_cast<const float4 *>(qa[1] + 16 * s);
      const float4 b0 = *reinterpret_cast<const float4 *>(cb[0] + 16 * s), b1 = *reinterpret_cast<const float4 *>(cb[1] + 16 * s);
      const float av[2][4] = {{a0.x, a0.y, a0.z, a0.w}, {a1.x, a1.y, a1.z, a1.w}};
      const float bv[2][4] = {{b0.x, b0.y, b0.z, b0.w}, {b1.x, b1.y, b1.z, b1.w}};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 2; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][j], bv[t][j], acc[i][t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ci = c0 + wc + 16 * t + r;
    if (ci >= nc) continue;
    const float cc = MET == L2 ? c2[ci] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t qi = q0 + wq + 16 * i + 4 * h + g;
        if (qi < nq) out[qi * nc + ci] = MET == L2 ? 2.0f * acc[i][t][g] - cc : acc[i][t][g];
      }
  }
}

// The same approximate scores on the bf16 matrix cores (round 6): each fp32 operand x is split into
// hi = bf16(x) and lo = bf16(x - hi) (x - hi is exact in fp32), and q.c ~ ch.qh + cl.qh + ch.ql, three
// v_mfma_f32_32x32x16_bf16 per 16-dim k-step (2.5 PF dense against the fp32 MFMA's ~157 TF: the launch
// is bound by its operand loads and score stores instead of the matrix pipe).  Per element,
// q c - (qh ch + qh cl + ql ch) = qr cr - qh dc - dq ch with qr = q - qh, dq = ql - qr (and the same for
// c): |qr| <= 2^-8 |q|, |dq| <= 2^-8 |qr| under round-to-nearest-even (the C++ float -> __bf16
// conversion, an IEEE fptrunc, v_cvt_pk_bf16_f32 in the default rounding mode), so the split costs
// <= 3.02 * 2^-16 |q_i c_i|, <= 773 u |q| |c|
// summed (u = 2^-24, Cauchy-Schwarz); the 3D products accumulate in fp32 inside the matrix core, <= 6 D u
// |q| |c| even at 2 u per addition.  launch_coarse_mfma widens c_err by both (L2: 2 q.c against
// (|q| + |c|)^2 >= 4 |q| |c|, so 3 D + 400; IP: 6 D + 800) on top of the fp32 kernels' constant.
// Wave: 32 queries x 64 centroids (two 32 x 32 accumulators, A = centroid tile, B = the queries: lane
// (r, h) ends with query r's scores of centroids 8b + 4h + i); block: 8 waves, 256 queries x the same 64
// centroids, whose fragments are staged in LDS 8 k-steps at a time (each centroid fragment crosses L2 once per
// 256 queries, not per 32; I1's 10,000 x 1,024 fit one round of resident blocks).
// The centroids come pre-split in fragment order (coarse_split_kernel, once per quantizer): tile T,
// k-step s, lane L -> 8 bf16 at ((T * KS + s) * 64 + L) * 8, hi and lo planes, tiles padded with zeros
// to a multiple of 8.
constexpr int COARSE_BF3_MAX_DIM = 256;
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f16acc __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split_bf16x8(const float4 a, const float4 b, bf8v &hi, bf8v &lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    hi[i] = (__bf16)v[i];
    lo[i] = (__bf16)(v[i] - (float)hi[i]);
  }
}

__global__ void coarse_split_kernel(const float *c, int nc, int D, int ntiles, bf8v *hi, bf8v *lo) {
  const int KS = D / 16;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (T, s, lane)
  if (e >= (int64_t)ntiles * KS * 64) return;
  const int L = (int)(e & 63), s = (int)((e >> 6) % KS), T = (int)((e >> 6) / KS);
  const int row = 32 * T + (L & 31), d0 = 16 * s + 8 * (L >> 5);
  float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = a;
  if (row < nc) {
    a = *reinterpret_cast<const float4 *>(c + (size_t)row * D + d0);
    b = *reinterpret_cast<const float4 *>(c + (size_t)row * D + d0 + 4);
  }
  split_bf16x8(a, b, hi[e], lo[e]);
}

template <int MET, int DT>
__global__ __launch_bounds__(512) void coarse_approx_bf3_kernel(const float *q, const bf8v *chi, const bf8v *clo,
                                                                const float *c2, int64_t nq, int nc, int Dr,
                                                                float *out, int32_t *zero, WordFill zf) {
  __shared__ bf8v cs[2][2][8][64];  // [hi / lo][tile][k-step of the chunk][lane]: 32 KB
  if (zero && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *zero = 0;  // the pick's failure count
  grid_word_fill(zf);
  const int D = DT > 0 ? DT : Dr;
  const int KS = D / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)blockIdx.y * 256 + 32 * w;  // the wave's 32 queries
  const int T0 = 2 * blockIdx.x;                          // the block's two centroid tiles (zero-padded past nc)
  const float *qp = q + (size_t)min(q0 + r, nq - 1) * D + 8 * h;
  f16acc a0 = {}, a1 = {};
  for (int s0 = 0; s0 < KS; s0 += 8) {
    const int kc = min(8, KS - s0);
    // the chunk's query fragments first: their HBM latency overlaps the centroid staging below
    float4 qv[8][2];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s >= kc) break;  // (block-uniform)
      qv[s][0] = *reinterpret_cast<const float4 *>(qp + 16 * (s0 + s));
      qv[s][1] = *reinterpret_cast<const float4 *>(qp + 16 * (s0 + s) + 4);
    }
    __syncthreads();  // the previous chunk is consumed
    for (int i = threadIdx.x; i < 4 * kc * 64; i += 512) {  // the two tiles' fragments, both planes
      const int L = i & 63, u = i >> 6, s = u % kc, t = (u / kc) & 1, pl = u / kc >> 1;
      cs[pl][t][s][L] = (pl ? clo : chi)[((size_t)(T0 + t) * KS + s0 + s) * 64 + L];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s >= kc) break;  // (block-uniform)
      bf8v qh, ql;
      split_bf16x8(qv[s][0], qv[s][1], qh, ql);
      const bf8v ch0 = cs[0][0][s][lane], ch1 = cs[0][1][s][lane], cl0 = cs[1][0][s][lane], cl1 = cs[1][1][s][lane];
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, qh, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, qh, a1, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl0, qh, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl1, qh, a1, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch0, ql, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch1, ql, a1, 0, 0, 0);
    }
  }
  const int64_t qi = q0 + r;
  if (qi >= nq) return;
  float *orow = out + qi * nc;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int cb = 32 * (T0 + t) + 8 * b + 4 * h;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float acc = t == 0 ? a0[4 * b + i] : a1[4 * b + i];
        v[i] = MET == L2 ? 2.0f * acc - (cb + i < nc ? c2[cb + i] : 0.0f) : acc;
      }
      if ((nc & 3) == 0 && cb + 3 < nc) {
        *reinterpret_cast<float4 *>(orow + cb) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cb + i < nc) orow[cb + i] = v[i];
      }
    }
  }
}

// ComputeScore (safe VectorMath form, as coarse_scores_kernel) spread over an 8-lane group: lane j runs
// accumulator j over dims j, j + 8, ...; the group sums as hsum8 does; every lane returns the score
template <int MET, int DT = 0>
__device__ __forceinline__ float exact_cs_l8(const float *qp, const float *cp, int Dr, int j) {
  const int D = DT > 0 ? DT : Dr;
  constexpr int U = DT > 0 ? DT / 8 : 4;
  float acc = 0.0f;
#pragma unroll U
  for (int d = j; d < (D & ~7); d += 8) {
    if (MET == L2) {
      const float t = qp[d] - cp[d];
      acc = acc + t * t;
    } else {
      acc = acc + qp[d] * cp[d];
    }
  }
  acc = acc + __shfl_xor(acc, 1);
  acc = acc + __shfl_xor(acc, 2);
  float sum = (D & ~7) > 0 ? 0.0f + (acc + __shfl_xor(acc, 4)) : 0.0f;
  for (int d = D & ~7; d < D; ++d) {  // the scalar tail (D % 16 == 0 here: none)
    if (MET == L2) {
      const float t = qp[d] - cp[d];
      sum = sum + t * t;
    } else {
      sum = sum + qp[d] * cp[d];
    }
  }
  return MET == L2 ? -sum : sum;
}

// the same for two centroids at once (two independent accumulation chains per lane: twice the work per
// dependent step); each result is bit for bit exact_cs_l8's
template <int MET, int DT = 0>
__device__ __forceinline__ void exact_cs_l8x2(const float *qp, const float *ca, const float *cb, int Dr, int j,
                                              float &ra, float &rb) {
  const int D = DT > 0 ? DT : Dr;
  constexpr int U = DT > 0 ? DT / 8 : 4;
  float acc = 0.0f, bcc = 0.0f;
#pragma unroll U
  for (int d = j; d < (D & ~7); d += 8) {
    const float x = qp[d];
    if (MET == L2) {
      const float t = x - ca[d], v = x - cb[d];
      acc = acc + t * t;
      bcc = bcc + v * v;
    } else {
      acc = acc + x * ca[d];
      bcc = bcc + x * cb[d];
    }
  }
  acc = acc + __shfl_xor(acc, 1);
  bcc = bcc + __shfl_xor(bcc, 1);
  acc = acc + __shfl_xor(acc, 2);
  bcc = bcc + __shfl_xor(bcc, 2);
  float sa = (D & ~7) > 0 ? 0.0f + (acc + __shfl_xor(acc, 4)) : 0.0f;
  float sb = (D & ~7) > 0 ? 0.0f + (bcc + __shfl_xor(bcc, 4)) : 0.0f;
  for (int d = D & ~7; d < D; ++d) {
    if (MET == L2) {
      const float t = qp[d] - ca[d], v = qp[d] - cb[d];
      sa = sa + t * t;
      sb = sb + v * v;
    } else {
      sa = sa + qp[d] * ca[d];
      sb = sb + qp[d] * cb[d];
    }
  }
  ra = MET == L2 ? -sa : sa;
  rb = MET == L2 ? -sb : sb;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
// the best 64 of two descending 64-lane lists: the lane-wise max of a and reversed b is bitonic and holds
// them; a bitonic merge sorts it descending
__device__ __forceinline__ uint64_t top64_merge(uint64_t a, uint64_t b, int lane) {
  const uint64_t br = shfl64(b, 63 - lane);
  uint64_t v = a > br ? a : br;
#pragma unroll
  for (int j = 32; j >= 1; j >>= 1) {
    const uint64_t o = shfl_xor64(v, j);
    v = (lane & j) == 0 ? (v > o ? v : o) : (v < o ? v : o);
  }
  return v;
}

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

// One wave per query: aP = the nprobe-th largest approximate score (wselect.h radix select over score
// keys), the candidates = every centroid whose approximate
// score reaches aP - 2E (at most PICK_MAX = 1024, in index order), their exact ComputeScore and the first
// nprobe of them by (score desc, index asc).  Every centroid left out scores exactly below the nprobe
// centroids whose approximate score reached aP.  More than 1024 candidates, or a non-finite query: the
// exact scores of every centroid go to the row and the query to the fail list (coarse_select_list_kernel).
template <int MET, int DT>
__global__ __launch_bounds__(256) void coarse_pick_kernel(const float *q, const float *c, float *scores, int64_t nq,
                                                          int nc, int Dr, int P, double cnmax, double c_err,
                                                          int32_t *probes, int32_t *fail, int32_t *nfail) {
  const int D = DT > 0 ? DT : Dr;
  __shared__ int hist[4][256];
  constexpr int PICK_MAX = 1024;  // (d = 768 widens 2E: P1 keeps a few hundred)
  __shared__ int cl[4][PICK_MAX];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t qi = (int64_t)blockIdx.x * 4 + w;
  if (qi >= nq) return;  // no block barrier below
  const float *qp = q + (size_t)qi * D;
  float *row = scores + qi * nc;
  float part = 0.0f;
  for (int d = lane; d < D; d += 64) part += qp[d] * qp[d];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
  const double qn = sqrt((double)part) * (1.0 + 1e-5);
  bool ok = isfinite(qn);
  int n = 0;
  if (ok) {
    // 1. the P-th largest score key
    float cv[16];
    const uint32_t prefix = wave_kth_key_lm<16>(row, nc, P, hist[w], cl[w], lane, cv);
    const float aP = key_score(prefix);
    const double u = 5.9604644775390625e-8;  // 2^-24
    const double E = MET == L2 ? c_err * u * (qn + cnmax) * (qn + cnmax) : c_err * u * qn * cnmax;
    const double tb = (double)aP - 2.0 * E;
    float th = (float)tb;
    if ((double)th > tb) th = nextafterf(th, -INFINITY);  // at or below aP - 2E
    ok = ok && isfinite(aP) && isfinite(th);
    // 2. the candidates, in index order
    if (ok) {
      auto take = [&](int cc, float val) {
        const bool pr = cc < nc && val >= th;
        const uint64_t m = __builtin_amdgcn_ballot_w64(pr);
        const int pos = n + (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (pr && pos < PICK_MAX) cl[w][pos] = cc;
        n += (int)__builtin_popcountll(m);
      };
      if (nc <= 64 * 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (64 * u < nc) take(64 * u + lane, cv[u]);
      } else {
        for (int c0 = 0; c0 < nc; c0 += 64) take(c0 + lane, c0 + lane < nc ? row[c0 + lane] : 0.0f);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      ok = n <= PICK_MAX;
    }
  }
  if (ok) {
    // 64 candidates at a time: exact scores (8 per pass, an 8-lane group each), sorted, merged into the best 64
    uint64_t best = 0ull;
    for (int b0 = 0; b0 < n; b0 += 64) {
      const int m = min(64, n - b0);
      const int cid = lane < m ? cl[w][b0 + lane] : -1;
      float sc = -INFINITY;
      for (int p = 0; 8 * p < m; p += 2) {  // passes p and p + 1 together (two chains per lane)
        const int ia = __shfl(cid, 8 * p + (lane >> 3)), ib = __shfl(cid, min(63, 8 * (p + 1) + (lane >> 3)));
        float va, vb;
        exact_cs_l8x2<MET, DT>(qp, c + (size_t)max(ia, 0) * D, c + (size_t)max(ib, 0) * D, D, lane & 7, va, vb);
        const float ta = __shfl(va, 8 * (lane & 7)), tb = __shfl(vb, 8 * (lane & 7));
        if ((lane >> 3) == p) sc = ta;  // lane 8p + g took candidate 8p + g's score from group g
        if ((lane >> 3) == p + 1) sc = tb;
      }
      uint64_t key = cid >= 0 ? rank_key(sc, cid) : 0ull;
      key = sort64_desc(key, lane);
      best = b0 == 0 ? key : top64_merge(best, key, lane);
    }
    if (lane < P) probes[qi * P + lane] = best != 0ull ? 0x7FFFFFFF - (int)(uint32_t)best : -1;
    return;
  }
  // fallback: the exact scores of every centroid into the row, selection by coarse_select_list_kernel
  for (int c0 = 0; c0 < nc; c0 += 8) {
    const int id = c0 + (lane >> 3);
    const float v = exact_cs_l8<MET, DT>(qp, c + (size_t)min(id, nc - 1) * D, D, lane & 7);
    if ((lane & 7) == 0 && id < nc) row[id] = v;
  }
  if (lane == 0) fail[atomicAdd(nfail, 1)] = (int32_t)qi;
}

template <int W>
__global__ __launch_bounds__(256) void coarse_select_list_kernel(const float *scores, const int32_t *fail,
                                                                 const int32_t *nfail, int nc, int nprobe,
                                                                 int32_t *probes) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + w;
  if (i >= *nfail) return;
  const int64_t qi = fail[i];
  select_row_reg<W>(scores + qi * nc, nc, nprobe, probes + qi * nprobe, lane);
}

}  // namespace

// waves (queries) per selection block: the rows of all of them must fit in LDS
static int select_wpb(int nlist) {
  const int64_t row = (int64_t)nlist * sizeof(uint64_t);
  return (int)std::max<int64_t>(0, std::min<int64_t>(4, (160 * 1024) / row));
}
bool coarse_dense_supported(int nlist) { return nlist >= 1 && select_wpb(nlist) >= 1; }

void launch_coarse_dense(const float *q, const float *cents_rm, const float *qn, const float *cn, int64_t nq,
                         int32_t nlist, int32_t dim, int32_t metric, int32_t nprobe, float *scores, int32_t *probes,
                         hipStream_t st) {
  if (nq <= 0 || nlist <= 0 || nprobe <= 0) return;
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&coarse_select_kernel), attr);
  const dim3 grid((unsigned)((nlist + CT - 1) / CT), (unsigned)((nq + CT - 1) / CT));
  if (metric == L2)
    hipLaunchKernelGGL(coarse_scores_kernel<L2>, grid, dim3(256), 0, st, q, cents_rm, qn, cn, nq, nlist, dim, scores);
  else if (metric == IP)
    hipLaunchKernelGGL(coarse_scores_kernel<IP>, grid, dim3(256), 0, st, q, cents_rm, qn, cn, nq, nlist, dim, scores);
  else
    hipLaunchKernelGGL(coarse_scores_kernel<COS>, grid, dim3(256), 0, st, q, cents_rm, qn, cn, nq, nlist, dim,
                       scores);
  // register lists for nprobe <= 64 (PYR_COARSE_SELECT=0: the LDS argmax rounds, measurement knob)
  const bool reg = !knob("PYR_COARSE_SELECT") || atoi(knob("PYR_COARSE_SELECT")) != 0;
  const dim3 g4((unsigned)((nq + 3) / 4));
  // a lane sees every 64th centroid, so its list never needs more than ceil(nlist / 64) entries: the
  // wave's P pops then still find every key (nlist = 1,024: 16-entry lists for nprobe = 32)
  const int per_lane = (nlist + 63) / 64;
  if (reg && nprobe <= 64 && per_lane <= 8) {
    hipLaunchKernelGGL(coarse_select_reg_kernel<8>, g4, dim3(256), 0, st, scores, nq, nlist, nprobe, probes);
  } else if (reg && (nprobe <= 16 || (nprobe <= 64 && per_lane <= 16))) {
    hipLaunchKernelGGL(coarse_select_reg_kernel<16>, g4, dim3(256), 0, st, scores, nq, nlist, nprobe, probes);
  } else if (reg && (nprobe <= 32 || (nprobe <= 64 && per_lane <= 32))) {
    hipLaunchKernelGGL(coarse_select_reg_kernel<32>, g4, dim3(256), 0, st, scores, nq, nlist, nprobe, probes);
  } else if (reg && nprobe <= 64) {
    hipLaunchKernelGGL(coarse_select_reg_kernel<64>, g4, dim3(256), 0, st, scores, nq, nlist, nprobe, probes);
  } else {
    const int wpb = select_wpb(nlist);
    hipLaunchKernelGGL(coarse_select_kernel, dim3((unsigned)((nq + wpb - 1) / wpb)), dim3(64 * wpb),
                       (size_t)wpb * nlist * sizeof(uint64_t), st, scores, nq, nlist, nprobe, wpb, probes);
  }
}

// the register-list capacity for selecting n of nlist centroids (launch_coarse_dense's choice)
template <class F>
static void with_list_cap(int nlist, int n, F &&f) {
  const int per_lane = (nlist + 63) / 64;
  if (per_lane <= 8) f(std::integral_constant<int, 8>{});
  else if (n <= 16 || per_lane <= 16) f(std::integral_constant<int, 16>{});
  else if (n <= 32 || per_lane <= 32) f(std::integral_constant<int, 32>{});
  else f(std::integral_constant<int, 64>{});
}

// measured faster than the dense exact ranking at d = 128 (I1 0.09 vs 0.21 ms, M8 0.80 vs 1.71 ms); at
// d = 768 (P1) the 64-candidate pick of round 3 sent almost every query to the dense fallback (12.1 vs
// 4.2 ms, profiles/r3_p1/coarse_mfma_ab.json), hence the 256-candidate pick
bool coarse_mfma_supported(int nlist, int dim, int metric, int nprobe) {
  return (metric == L2 || metric == IP) && dim > 0 && dim % 16 == 0 && dim <= 1024 && nlist >= 1 && nprobe >= 1 &&
         nprobe <= 64;
}

// the bf16 split kernel up to this dimension: its wider bound (3 D + 400 on top of 4 D + 64) lets more centroids
// into the pick's exact band, which P1 (d = 768, nlist 4,096) paid for: coarse 4.66 vs 2.90 ms with the fp32 kernel
// (profiles/r6_p1/p1_bf3.log); at d = 128 the split kernel wins (I1 coarse 0.075 vs 0.086-0.092 ms)
int coarse_bf3_max_dim() { return COARSE_BF3_MAX_DIM; }

size_t coarse_split_bytes(int nlist, int dim) {
  const int ntiles = ((nlist + 31) / 32 + 7) / 8 * 8;
  return (size_t)2 * ntiles * (dim / 16) * 64 * 16;
}

void launch_coarse_split(const float *cents_rm, int nlist, int dim, void *split, hipStream_t st) {
  if (nlist <= 0 || dim % 16 != 0) return;
  const int ntiles = ((nlist + 31) / 32 + 7) / 8 * 8;
  const int64_t n = (int64_t)ntiles * (dim / 16) * 64;
  bf8v *hi = reinterpret_cast<bf8v *>(split);
  hipLaunchKernelGGL(coarse_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cents_rm, nlist, dim,
                     ntiles, hi, hi + n);
}

void launch_coarse_mfma(const float *q, const float *cents_rm, const float *c2, int64_t nq, int32_t nlist,
                        int32_t dim, int32_t metric, int32_t nprobe, double cnmax, double c_err, float *scores,
                        int32_t *fail, int32_t *nfail, int32_t *probes, hipStream_t st, const WordFill *zero,
                        const void *split) {
  if (nq <= 0 || nlist <= 0 || nprobe <= 0) {
    if (zero) launch_fill_words(*zero, st);
    return;
  }
  const WordFill zf = zero ? *zero : WordFill{};
  const int P = std::min(nprobe, nlist);
  const dim3 ga((unsigned)((nlist + 31) / 32), (unsigned)((nq + 31) / 32));
  const dim3 g4((unsigned)((nq + 3) / 4));
  // the bf16 split kernel when the centroids come pre-split; PYR_COARSE_APPROX=0 / 1: the fp32 one-wave-per-
  // tile / LDS kernels (A/B; approximate scores within their own, tighter bound)
  const char *ae = knob("PYR_COARSE_APPROX");
  const bool bf3 = split != nullptr && !ae && dim <= COARSE_BF3_MAX_DIM;
  const bool lds = !(ae && atoi(ae) == 0);
  if (bf3) c_err += metric == L2 ? 3.0 * dim + 400.0 : 6.0 * dim + 800.0;
  const dim3 gl((unsigned)((nlist + 63) / 64), (unsigned)((nq + 63) / 64));
  const dim3 gb((unsigned)((nlist + 63) / 64), (unsigned)((nq + 255) / 256));
  const int64_t nsplit = (int64_t)(((nlist + 31) / 32 + 7) / 8 * 8) * (dim / 16) * 64;
  auto go = [&](auto met, auto dt) {
    constexpr int M = decltype(met)::value, DT = decltype(dt)::value;
    // the approximate-score kernel also zeroes the pick's failure count (no hipMemsetAsync on a search path:
    // the memset nodes of a captured graph write stale values from their second replay on,
    // scripts/diag/graph_memset.py)
    if (bf3) {
      const bf8v *hi = reinterpret_cast<const bf8v *>(split);
      hipLaunchKernelGGL((coarse_approx_bf3_kernel<M, DT>), gb, dim3(512), 0, st, q, hi, hi + nsplit, c2, nq, nlist,
                         dim, scores, nfail, zf);
    } else if (lds)
      hipLaunchKernelGGL((coarse_approx_lds_kernel<M>), gl, dim3(256), 0, st, q, cents_rm, c2, nq, nlist, dim, scores,
                         nfail, zf);
    else
      hipLaunchKernelGGL((coarse_approx_kernel<M, DT>), ga, dim3(64), 0, st, q, cents_rm, c2, nq, nlist, dim, scores,
                         nfail, zf);
    hipLaunchKernelGGL((coarse_pick_kernel<M, DT>), g4, dim3(256), 0, st, q, cents_rm, scores, nq, nlist, dim, P, cnmax,
                       c_err, probes, fail, nfail);
  };
  auto by_dim = [&](auto met) {
    switch (dim) {
      case 32: go(met, std::integral_constant<int, 32>{}); return;
      case 64: go(met, std::integral_constant<int, 64>{}); return;
      case 128: go(met, std::integral_constant<int, 128>{}); return;
      case 768: go(met, std::integral_constant<int, 768>{}); return;
      default: go(met, std::integral_constant<int, 0>{}); return;
    }
  };
  if (metric == L2) by_dim(std::integral_constant<int, L2>{});
  else by_dim(std::integral_constant<int, IP>{});
  with_list_cap(nlist, P, [&](auto W) {
    hipLaunchKernelGGL(coarse_select_list_kernel<decltype(W)::value>, g4, dim3(256), 0, st, scores, fail, nfail, nlist,
                       P, probes);
  });
}

}  // namespace pyr
