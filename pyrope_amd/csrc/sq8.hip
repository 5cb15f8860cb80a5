// sq8.hip -- the 8-bit search mode of the FLAT index on gfx950.
//
// BruteForceVectorIndex.EnableQuantization (BruteForceVectorIndex.cs:25-40): rows written
// while it is on get ScalarQuantizer codes (per-vector min/max, 0..255, ScalarQuantizer.cs:23-62);
// a search quantizes the query the same way and scores every scanned row with the exact
// integer VectorMath.L2Squared8Bit / DotProduct8Bit (VectorMath.cs:441-681), negated for L2
// and converted long -> float.  Rows written while it was off have no codes: they count as
// scanned (MaxScans) but are skipped (:308-318).
//
// Integer arithmetic makes parity exact: the dot product runs on v_dot4_u32_u8 (4 byte MACs
// per lane op), L2 through sum(a^2) + sum(b^2) - 2 sum(ab) with the per-vector sums of squares
// precomputed at quantization time.  The reference's x64 SIMD path sums the first
// n - n % 32 terms in wrapping int32 lanes and the tail in long; both parts are kept apart
// here (u32 arithmetic for the vector part, int64 for the tail) so even the wrap is the same.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

__device__ __forceinline__ bool better(float s1, uint32_t k1, float s2, uint32_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

// (int)Math.Round(double) as .NET 8 evaluates it on x64: ties to even; NaN and values
// outside int range give int.MinValue (cvttsd2si "integer indefinite")
__device__ __forceinline__ int net_round_to_int(float v) {
  const float r = rintf(v);  // round to nearest even (default mode)
  if (!(r >= -2147483648.0f && r < 2147483648.0f)) return INT_MIN;
  return (int)r;
}

// One wave per vector.  src: blocked row store + slot list (FLAT rows) or row-major vectors
// (queries).  Writes codes [dst][dp] (zero padded), the two sums of squares and has-codes.
__global__ __launch_bounds__(256) void sq8_quantize_kernel(const float *src, const int64_t *slots, int blocked,
                                                           int64_t n, int D, int dp, int sl, uint8_t *codes,
                                                           int2 *sums, uint8_t *ok) {
  const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (v >= n) return;
  const int64_t slot = slots ? slots[v] : v;
  auto at = [&](int d) -> float {
    return blocked ? src[((size_t)(slot >> 3) * D + d) * 8 + (slot & 7)] : src[(size_t)v * D + d];
  };
  // ScalarQuantizer.cs:37-44: min / max by strict comparisons (NaN never selected)
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (int d = lane; d < D; d += 64) {
    const float x = at(d);
    if (x < mn) mn = x;
    if (x > mx) mx = x;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    if (a < mn) mn = a;
    if (b > mx) mx = b;
  }
  const float range = mx - mn;
  const float scale = 255.0f / range;
  uint8_t *out = codes + (size_t)slot * dp;
  uint32_t sv = 0;
  int st = 0;
  for (int d = lane; d < dp; d += 64) {
    int c = 0;
    if (d < D && range != 0.0f) {  // :46-50 range 0 -> all zeros
      const float normalized = (at(d) - mn) * scale;
      const int r = net_round_to_int(normalized);
      c = r < 0 ? 0 : (r > 255 ? 255 : r);  // Math.Clamp(.., 0, 255)
    }
    out[d] = (uint8_t)c;
    if (d < sl) sv += (uint32_t)(c * c);
    else st += c * c;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    sv += __shfl_xor(sv, o);
    st += __shfl_xor(st, o);
  }
  if (lane == 0) {
    sums[slot] = make_int2((int)sv, st);
    if (ok) ok[slot] = 1;
  }
}

// One block (4 waves) per item: rows [row_begin, row_end) x queries [qbeg, qbeg + qcnt),
// qcnt <= SQ8_QG.  Lane = row; the query codes sit in LDS (read as broadcasts).  Each wave
// keeps a top-k per query spread over its lanes (lane j = j-th best, ballot-filtered
// insertion as in kernels.hip pq_adc); the four waves' lists are merged per query at the end
// into the item's partial slot q * nparts + part.
constexpr int SQ8_QG = 8;

__device__ __forceinline__ void lane_list_insert(bool cand, float sc, uint32_t key, float &ls, uint32_t &lk,
                                                 float &kth, uint32_t &kthk, int k, int lane) {
  uint64_t m = __ballot(cand);
  while (m) {
    const int j = __ffsll((unsigned long long)m) - 1;
    const float s = __shfl(sc, j);
    const uint32_t kk = __shfl(key, j);
    const int pos = __popcll(__ballot(lane < k && better(ls, lk, s, kk)));
    const float us = __shfl_up(ls, 1);
    const uint32_t uk = __shfl_up(lk, 1);
    if (lane > pos && lane < k) {
      ls = us;
      lk = uk;
    }
    if (lane == pos) {
      ls = s;
      lk = kk;
    }
    kth = __shfl(ls, k - 1);
    kthk = __shfl(lk, k - 1);
    m &= m - 1;
    m &= __ballot(cand && better(sc, key, kth, kthk));
  }
}

template <int DW, int MET>  // DW: 32-bit code words per row (dp / 4)
__global__ __launch_bounds__(256) void sq8_scan_kernel(Sq8Args a) {
  __shared__ uint32_t qw[SQ8_QG][DW];
  __shared__ int2 qsum[SQ8_QG];
  __shared__ float mrs[SQ8_QG][4][64];
  __shared__ uint32_t mrk[SQ8_QG][4][64];
  if ((int)blockIdx.x >= *a.n_items) return;
  const ScanItem it = a.items[blockIdx.x];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, k = a.k;
  const int swords = a.sl / 4;  // words of the int32-wrapped vector part
  for (int e = tid; e < SQ8_QG * DW; e += 256) {
    const int j = e / DW, d = e - j * DW;
    qw[j][d] = j < it.qcnt ? reinterpret_cast<const uint32_t *>(a.qcodes + (size_t)(it.qbeg + j) * a.dp)[d] : 0u;
  }
  if (tid < SQ8_QG) qsum[tid] = tid < it.qcnt ? a.qsums[it.qbeg + tid] : make_int2(0, 0);
  __syncthreads();

  float ls[SQ8_QG], kth[SQ8_QG];
  uint32_t lk[SQ8_QG], kthk[SQ8_QG];
#pragma unroll
  for (int j = 0; j < SQ8_QG; ++j) {
    ls[j] = kth[j] = -INFINITY;
    lk[j] = kthk[j] = KEY_NONE;
  }
  const int rb = it.row_begin, re = it.row_end;
  for (int r0 = rb + 64 * w; r0 < re; r0 += 256) {
    // the query words are re-read from LDS (broadcasts) per row group: hoisting all
    // SQ8_QG x DW of them into registers would cost the occupancy
    asm volatile("" ::: "memory");
    const int r = r0 + lane;
    const bool valid = r < re && (uint32_t)r < a.row_limit && a.live[r] && a.ok[r];
    uint32_t rw[DW];
    const uint4 *rp = reinterpret_cast<const uint4 *>(a.codes + (size_t)(valid ? r : rb) * a.dp);
#pragma unroll
    for (int c = 0; c < DW / 4; ++c) {
      const uint4 v = rp[c];
      rw[4 * c] = v.x;
      rw[4 * c + 1] = v.y;
      rw[4 * c + 2] = v.z;
      rw[4 * c + 3] = v.w;
    }
    const int2 rs = a.sums[valid ? r : rb];
#pragma unroll
    for (int j = 0; j < SQ8_QG; ++j) {
      uint32_t dv = 0, dt = 0;  // vector part (wraps like the int32 lanes), tail (exact)
#pragma unroll
      for (int d = 0; d < DW; ++d) {
        if (d < swords) dv = __builtin_amdgcn_udot4(rw[d], qw[j][d], dv, false);
        else dt = __builtin_amdgcn_udot4(rw[d], qw[j][d], dt, false);
      }
      int64_t tot;
      if (MET == L2) {
        const uint32_t vpart = (uint32_t)qsum[j].x + (uint32_t)rs.x - 2u * dv;
        tot = (int64_t)(int32_t)vpart + ((int64_t)qsum[j].y + rs.y - 2 * (int64_t)dt);
        tot = -tot;
      } else {
        tot = (int64_t)(int32_t)dv + (int64_t)dt;
      }
      const float score = (float)tot;  // long -> float, round to nearest (BruteForceVectorIndex.cs:325-331)
      const bool cand = valid && j < it.qcnt && better(score, (uint32_t)r, kth[j], kthk[j]);
      lane_list_insert(cand, score, (uint32_t)r, ls[j], lk[j], kth[j], kthk[j], k, lane);
    }
  }
#pragma unroll
  for (int j = 0; j < SQ8_QG; ++j) {
    if (lane < k) {
      mrs[j][w][lane] = ls[j];
      mrk[j][w][lane] = lk[j];
    }
  }
  __syncthreads();
  for (int j = w; j < it.qcnt; j += 4) {  // wave w merges queries w, w + 4, ...
    float s = -INFINITY, kt = -INFINITY;
    uint32_t kk = KEY_NONE, ktk = KEY_NONE;
    for (int v = 0; v < 4; ++v) {
      const float cs = lane < k ? mrs[j][v][lane] : -INFINITY;
      const uint32_t ck = lane < k ? mrk[j][v][lane] : KEY_NONE;
      const bool cand = ck != KEY_NONE && better(cs, ck, kt, ktk);
      lane_list_insert(cand, cs, ck, s, kk, kt, ktk, k, lane);
    }
    if (lane < k) {
      const size_t slot = (size_t)(it.qbeg + j) * a.nparts + it.part;
      a.part_s[slot * k + lane] = s;
      a.part_k[slot * k + lane] = kk;
    }
  }
}

}  // namespace

void launch_sq8_quantize(const float *src, const int64_t *slots, int blocked, int64_t n, int32_t dim, int32_t dp,
                         uint8_t *codes, int2 *sums, uint8_t *ok, hipStream_t st) {
  if (n <= 0) return;
  const int sl = dim >= 32 ? dim - dim % 32 : 0;
  hipLaunchKernelGGL(sq8_quantize_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, src, slots, blocked, n, dim,
                     dp, sl, codes, sums, ok);
}

int sq8_dp(int dim) { return (dim + 15) / 16 * 16; }
int sq8_qgroup() { return SQ8_QG; }
bool sq8_supported(int dim, int k) { return k >= 1 && k <= 64 && sq8_dp(dim) <= 256; }

void launch_sq8_scan(const Sq8Args &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  const int dw = a.dp / 4;
  Sq8Args b = a;
  b.sl = a.dim >= 32 ? a.dim - a.dim % 32 : 0;
#define SQ8_CASE(W)                                                                                       \
  case W:                                                                                                 \
    if (metric == L2) hipLaunchKernelGGL((sq8_scan_kernel<W, L2>), dim3(max_items), dim3(256), 0, st, b); \
    else hipLaunchKernelGGL((sq8_scan_kernel<W, IP>), dim3(max_items), dim3(256), 0, st, b);              \
    break;
  switch (dw) {
    SQ8_CASE(4)
    SQ8_CASE(8)
    SQ8_CASE(12)
    SQ8_CASE(16)
    SQ8_CASE(20)
    SQ8_CASE(24)
    SQ8_CASE(28)
    SQ8_CASE(32)
    SQ8_CASE(36)
    SQ8_CASE(40)
    SQ8_CASE(44)
    SQ8_CASE(48)
    SQ8_CASE(52)
    SQ8_CASE(56)
    SQ8_CASE(60)
    SQ8_CASE(64)
    default: break;
  }
#undef SQ8_CASE
}

}  // namespace pyr
