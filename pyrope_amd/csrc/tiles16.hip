// tiles16.hip -- the fp16 row tiles the stream scan reads (gfx950), written at add / build time.
//
//  * Rows are stored a second time as fp16 in the exact order the MFMA operand wants (h16 tiles: 32
//    rows x Dp, [k-step s][lane half h][row i][8 halves], 64 Dp bytes; Dp = the tile dimension, dims
//    past D zero), as residuals x - c[list] (IVF lists; FLAT: x - mean for L2), scaled by a power of
//    two sx so the store's largest |x| is below 2^14.  The scan reads 2 B per dimension instead of 4
//    and every 1 KiB piece is lane-linear (conflict-free, one global_load per lane).
//  * A per-row additive term (meta: -|x|^2 for L2, 0 for IP, -inf for a dead / padding row) travels
//    with the tile, so a score is one fma per (query, row): approx = f_q * acc + meta, with
//    f_q = (L2 ? 2 : 1) / (sq * sx) and sq the query's own power-of-two scale.
//  * The error |q.x - approx/f| <= (2^-11 + 2D u) sum|q_i x_i| + 2^-25 sum|q_i| / sx (x's and q's fp16
//    rounding, fp32 accumulation, fp16 subnormals) is what the scan's bound and refine_kernel's c_bf /
//    abs terms certify against (kernels.h filter_f16_cerr, filter_f16_abs).
// (Until round 3 this file also held the fp16 tile filters that scan.hip superseded.)
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

#include "f16util.h"

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

// residual mode: cents (row-major) and tile_list (list id of each 32-row tile; null = every tile
// list 0, the FLAT store's single center) -> x - c[list]
__device__ __forceinline__ float resid_val(const float *rows, const float *cents, const int32_t *tile_list, int64_t r,
                                           int d, int D) {
  const float x = rows[((size_t)(r >> 3) * D + d) * 8 + (r & 7)];
  return cents ? x - cents[(size_t)(tile_list ? tile_list[r >> 5] : 0) * D + d] : x;
}

// A row whose norm (rn: |x|^2 or |x - c|^2) is not finite holds an Inf or a NaN: its tile entries are
// zero (an Inf times a zero or opposite-signed query half would make the whole score NaN), and
// meta16_kernel makes it always (Inf) or never (NaN) a candidate.
__global__ void encode16_kernel(const float *rows, const int64_t *slots, int64_t n, int D, float sx,
                                const float *cents, const int32_t *tile_list, const float *rn, _Float16 *h16,
                                int Dp) {
  const int G = Dp / 8;  // Dp >= D: the tile dimension, dims past D zero
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * G;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / G;
    const int g = (int)(e % G);
    const int64_t r = slots ? slots[i] : i;
    h8v v;
    const bool special = rn && !isfinite(rn[r]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = special || 8 * g + j >= D ? (_Float16)0.0f
                                         : (_Float16)(resid_val(rows, cents, tile_list, r, 8 * g + j, D) * sx);
    const size_t off = (((size_t)(r >> 5) * (Dp / 16) + (g >> 1)) * 2 + (g & 1)) * 32 + (r & 31);
    *reinterpret_cast<h8v *>(h16 + off * 8) = v;
  }
}

// meta[r] = live ? (L2 ? -|x|^2 : 0) : -inf; a live row with a non-finite norm: +inf when it holds an
// Inf (approx = +inf: always a candidate; the exact refine gives its real +-inf / NaN score, and the
// certificate's K1-th approximate score still bounds every row left out), -inf when it holds a NaN
// (never a candidate: the reference heap keeps a NaN score only among the first k rows it scans)
__global__ void meta16_kernel(const int64_t *slots, int64_t n, int met, const float *rsq, const uint8_t *live,
                              float *meta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots ? slots[i] : i;
  const float n2 = rsq[r];
  meta[r] = !live[r] || isnan(n2) ? -INFINITY : isinf(n2) ? INFINITY : (met == L2 ? -n2 : 0.0f);
}

// max |x_i| over the given rows (finite values; non-negative floats order as their bits)
__global__ void absmax_kernel(const float *rows, const int64_t *slots, int64_t n, int D, const float *cents,
                              const int32_t *tile_list, uint32_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots ? slots[i] : i;
  float m = 0.0f;
  for (int d = 0; d < D; ++d) {
    const float v = fabsf(resid_val(rows, cents, tile_list, r, d, D));
    if (isfinite(v)) m = fmaxf(m, v);
  }
  atomicMax(out, __float_as_uint(m));
}

// |x - c[list]|^2 per row (fp32, any order: the certificate budgets its rounding) of rows [0, n) or
// of the n rows at slots; out_max (may be null): atomic max of the finite values' score keys
__global__ void resid_sq_kernel(const float *rows, const int64_t *slots, int64_t n, int D, const float *cents,
                                const int32_t *tile_list, float *out, uint32_t *out_max) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots ? slots[i] : i;
  float s = 0.0f;
  for (int d = 0; d < D; ++d) {
    const float v = resid_val(rows, cents, tile_list, r, d, D);
    s += v * v;
  }
  out[r] = s;
  if (out_max && isfinite(s)) atomicMax(out_max, score_key(s));
}

}  // namespace

void launch_encode16(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float sx, void *h16,
                     hipStream_t st, const float *cents, const int32_t *tile_list, const float *rn, int32_t dpad) {
  if (n <= 0) return;
  const int dp = dpad > dim ? dpad : dim;
  hipLaunchKernelGGL(encode16_kernel, dim3(gblk(n * (dp / 8))), dim3(256), 0, st, rows, slots, n, dim, sx, cents,
                     tile_list, rn, reinterpret_cast<_Float16 *>(h16), dp);
}

void launch_resid_sq(const float *rows, int64_t n, int32_t dim, const float *cents, const int32_t *tile_list,
                     float *out, hipStream_t st, const int64_t *slots, uint32_t *out_max) {
  if (n <= 0) return;
  hipLaunchKernelGGL(resid_sq_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, slots, n, dim, cents, tile_list,
                     out, out_max);
}

void launch_meta16(const int64_t *slots, int64_t n, int32_t metric, const float *rsq, const uint8_t *live, float *meta,
                   hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(meta16_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, slots, n, metric, rsq, live, meta);
}

void launch_absmax(const float *rows, const int64_t *slots, int64_t n, int32_t dim, uint32_t *out, hipStream_t st,
                   const float *cents, const int32_t *tile_list) {
  if (n <= 0) return;
  hipLaunchKernelGGL(absmax_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, slots, n, dim, cents, tile_list, out);
}

}  // namespace pyr
