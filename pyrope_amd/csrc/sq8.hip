// sq8.hip -- the 8-bit search mode of the FLAT index on gfx950.
//
// BruteForceVectorIndex.EnableQuantization (BruteForceVectorIndex.cs:25-40): rows written
// while it is on get ScalarQuantizer codes (per-vector min/max, 0..255, ScalarQuantizer.cs:23-62);
// a search quantizes the query the same way and scores every scanned row with the exact
// integer VectorMath.L2Squared8Bit / DotProduct8Bit (VectorMath.cs:441-681), negated for L2
// and converted long -> float.  Rows written while it was off have no codes: they count as
// scanned (MaxScans) but are skipped (:308-318).
//
// The products run on the int8 matrix cores (v_mfma_i32_32x32x32_i8, exact int32 sums).
// Codes are stored shifted, c' = c - 128 in [-128, 127], and zero padded to a multiple of 32,
// so with A = sum(a), B = sum(b) over the real dims:
//     sum(a b)     = sum(a' b') + 128 (A + B) - 16384 n
//     sum((a-b)^2) = sum(a^2) + sum(b^2) - 2 sum(a b)
// all exact in 64-bit integers.  (The reference's x64 SIMD path sums in wrapping int32 lanes;
// no wrap is possible at the supported dims, n <= 512: |sum| <= 512 * 255^2 < 2^31.)
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cfloat>
#include <climits>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

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
// (queries).  Writes codes [dst][dp] (shifted by -128 when `shifted`, zero padded), the sums
// {sum c, sum c^2} over the real dims, and has-codes.
__global__ __launch_bounds__(256) void sq8_quantize_kernel(const float *src, const int64_t *slots, int blocked,
                                                           int64_t n, int D, int dp, int shifted, uint8_t *codes,
                                                           int2 *sums, uint8_t *ok, float2 *minmax) {
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
  if (minmax && lane == 0) minmax[v] = make_float2(mn, mx);  // the out min / out max of Quantize
  const float range = mx - mn;
  const float scale = 255.0f / range;
  uint8_t *out = codes + (size_t)slot * dp;
  int s1 = 0, s2 = 0;
  for (int d = lane; d < dp; d += 64) {
    int c = 0;
    if (d < D && range != 0.0f) {  // :46-50 range 0 -> all zeros
      const float normalized = (at(d) - mn) * scale;
      const int r = net_round_to_int(normalized);
      c = r < 0 ? 0 : (r > 255 ? 255 : r);  // Math.Clamp(.., 0, 255)
    }
    if (d < D) {
      s1 += c;
      s2 += c * c;
      out[d] = (uint8_t)(shifted ? c - 128 : c);
    } else {
      out[d] = 0;  // padding: 0 in the shifted domain contributes nothing to sum(a' b')
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) {
    sums[slot] = make_int2(s1, s2);
    if (ok) ok[slot] = 1;
  }
}

// Insert (v, key) into a register-resident sorted (desc) list of length KR (as filter.hip).
template <int KR>
__device__ __forceinline__ void reg_insert(float (&s)[KR], uint32_t (&kk)[KR], float v, uint32_t key) {
  bool b[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) b[j] = better(v, key, s[j], kk[j]);
#pragma unroll
  for (int j = KR - 1; j >= 1; --j) {
    s[j] = b[j - 1] ? s[j - 1] : (b[j] ? v : s[j]);
    kk[j] = b[j - 1] ? kk[j - 1] : (b[j] ? key : kk[j]);
  }
  s[0] = b[0] ? v : s[0];
  kk[0] = b[0] ? key : kk[0];
}

// One block = 4 independent waves; wave w scores queries qbeg + 32w .. +31 of the item
// against the item's rows, 32 rows per step:
//   A operand (queries, registers for the whole item): lane l holds query (l & 31), code
//     bytes [32s + 16h, 32s + 16h + 16) of k-step s, h = l >> 5;
//   B operand (rows, straight from HBM/L2, one step ahead): lane l holds row (l & 31) of the
//     step, the same bytes;
//   C[query][row] (C/D map: lane = row, register r = query (r&3) + 8(r>>2) + 4h) is turned into
//     exact scores in place (query sums in registers, row sums loaded with the row), moved
//     through a wave-private LDS transpose, and lane i < 32 (the query's owner) filters its 32
//     scores against its list's k-th and inserts survivors (register list, KR >= k).
constexpr int SQ8_RT = 32;
constexpr int SQ8_SCR = SQ8_RT + 4;

template <int NS, int MET, int KR>  // NS: 32-byte k-steps per row (dp / 32)
__global__ __launch_bounds__(256) void sq8_mfma_kernel(Sq8Args a) {
  __shared__ float scw[4][32][SQ8_SCR];
  if ((int)blockIdx.x >= *a.n_items) return;
  const ScanItem it = a.items[blockIdx.x];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, i32 = lane & 31, h = lane >> 5;
  if (32 * w >= it.qcnt) return;  // no block barrier below: idle waves may leave
  float(*sc)[SQ8_SCR] = scw[w];
  const int64_t D = a.dim;

  // A operand and the sums of the 16 queries this lane's C registers hold
  v4i qa[NS];
  {
    const int qi = it.qbeg + 32 * w + i32;
    const bool qv = 32 * w + i32 < it.qcnt;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      qa[s] = qv ? *reinterpret_cast<const v4i *>(a.qcodes + (size_t)qi * a.dp + 32 * s + 16 * h) : v4i{0, 0, 0, 0};
  }
  int qs1[16], qs2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int qq = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * h;
    const int2 v = qq < it.qcnt ? a.qsums[it.qbeg + qq] : make_int2(0, 0);
    qs1[r] = v.x;
    qs2[r] = v.y;
  }
  const bool owner = h == 0 && 32 * w + i32 < it.qcnt;
  float ts[KR];
  uint32_t tk[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) {
    ts[j] = -INFINITY;
    tk[j] = KEY_NONE;
  }

  const int r0 = it.row_begin, re = it.row_end;
  const int nst = (re - r0 + SQ8_RT - 1) / SQ8_RT;
  v4i rb[NS];
  int2 rs = make_int2(0, 0);
  bool rvalid = false;
  auto load_row = [&](int stg) {
    const int r = r0 + stg * SQ8_RT + i32;
    rvalid = r < re && (uint32_t)r < a.row_limit && a.live[r] && a.ok[r];
    const int rr = rvalid ? r : r0;
#pragma unroll
    for (int s = 0; s < NS; ++s) rb[s] = *reinterpret_cast<const v4i *>(a.codes + (size_t)rr * a.dp + 32 * s + 16 * h);
    rs = a.sums[rr];
  };
  if (nst > 0) load_row(0);
  for (int st = 0; st < nst; ++st) {
    v16i acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(qa[s], rb[s], acc, 0, 0, 0);
    const int2 cs = rs;
    const bool cv = rvalid;
    if (st + 1 < nst) load_row(st + 1);  // next step's operand while this one is scored
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t dot = (int64_t)acc[r] + 128 * (int64_t)(qs1[r] + cs.x) - 16384 * D;  // sum(a b)
      const int64_t v = MET == L2 ? -((int64_t)qs2[r] + cs.y - 2 * dot) : dot;
      sc[(r & 3) + 8 * (r >> 2) + 4 * h][i32] = cv ? (float)v : -INFINITY;  // long -> float (:325-331)
    }
    __builtin_amdgcn_wave_barrier();
    if (owner) {
      const float *scp = sc[i32];
      const float lo = ts[KR - 1];
      uint32_t pass = 0;
#pragma unroll
      for (int j = 0; j < SQ8_RT; ++j) {
        const float v = scp[j];
        if (v > -INFINITY && v >= lo) pass |= 1u << j;
      }
      const int rbase = r0 + st * SQ8_RT;
      while (pass) {
        const int j = __builtin_ctz(pass);
        pass &= pass - 1;
        const float v = scp[j];
        const uint32_t key = (uint32_t)(rbase + j);
        if (better(v, key, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, key);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the owners have read sc before the next step rewrites it
  }
  if (owner) {
    const size_t slot = (size_t)(it.qbeg + 32 * w + i32) * a.nparts + it.part;
#pragma unroll
    for (int j = 0; j < KR; ++j)
      if (j < a.k) {
        a.part_s[slot * a.k + j] = ts[j];
        a.part_k[slot * a.k + j] = tk[j];
      }
  }
}

template <int NS, int MET>
void launch_nk(const Sq8Args &a, int max_items, hipStream_t st) {
  if (a.k <= 16) hipLaunchKernelGGL((sq8_mfma_kernel<NS, MET, 16>), dim3(max_items), dim3(256), 0, st, a);
  else if (a.k <= 32) hipLaunchKernelGGL((sq8_mfma_kernel<NS, MET, 32>), dim3(max_items), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((sq8_mfma_kernel<NS, MET, 64>), dim3(max_items), dim3(256), 0, st, a);
}

}  // namespace

void launch_sq8_quantize(const float *src, const int64_t *slots, int blocked, int64_t n, int32_t dim, int32_t dp,
                         int shifted, uint8_t *codes, int2 *sums, uint8_t *ok, hipStream_t st, float2 *minmax) {
  if (n <= 0) return;
  // 64 threads per row: launched in pieces of 2^24 rows so a grid stays below 2^32 work-items (a
  // piece offset is a multiple of 8, so a blocked source moves by whole 8-row groups)
  constexpr int64_t PIECE = int64_t(1) << 24;
  for (int64_t off = 0; off < n; off += PIECE) {
    const int64_t m = n - off < PIECE ? n - off : PIECE;
    const bool rm = slots == nullptr;  // row i of the call -> code row i (else -> code row slots[i])
    // the source row: a blocked store is read at the slot; a row-major source at the call's row
    hipLaunchKernelGGL(sq8_quantize_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, st,
                       src + (blocked && !rm ? 0 : off * dim), slots ? slots + off : nullptr, blocked, m, dim, dp, shifted,
                       codes + (rm ? off * dp : 0), sums + (rm ? off : 0), ok ? ok + (rm ? off : 0) : nullptr,
                       minmax ? minmax + off : nullptr);
  }
}

// ScalarQuantizer.Dequantize (ScalarQuantizer.cs:65-84): range 0 -> min everywhere, else
// min + q * (range / 255) in fp32 (no contraction: the file is compiled with fp-contract off)
__global__ void sq8_dequantize_kernel(const uint8_t *codes, int64_t n, int D, const float *mins, const float *maxs,
                                      float *out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * D) return;
  const int64_t v = e / D;
  const float mn = mins[v], range = maxs[v] - mn;
  if (range == 0.0f) {
    out[e] = mn;
    return;
  }
  const float scale = range / 255.0f;
  const float t = (float)codes[e] * scale;
  out[e] = mn + t;
}

void launch_sq8_dequantize(const uint8_t *codes, int64_t n, int32_t dim, const float *mins, const float *maxs,
                           float *out, hipStream_t st) {
  if (n <= 0 || dim <= 0) return;
  const int64_t piece = std::max<int64_t>(1, (int64_t(1) << 30) / dim);  // rows per launch: < 2^32 work-items
  for (int64_t off = 0; off < n; off += piece) {
    const int64_t m = std::min(piece, n - off);
    hipLaunchKernelGGL(sq8_dequantize_kernel, dim3((unsigned)((m * dim + 255) / 256)), dim3(256), 0, st,
                       codes + off * dim, m, dim, mins + off, maxs + off, out + off * dim);
  }
}

// code row stride: dim rounded up to 32, then to a k-step count the scan is instantiated for
int sq8_dp(int dim) {
  int ns = (dim + 31) / 32;
  if (ns > 8) ns = ns <= 10 ? 10 : (ns <= 12 ? 12 : 16);
  return ns * 32;
}
int sq8_qgroup() { return 128; }
bool sq8_supported(int dim, int k) { return k >= 1 && k <= 64 && dim >= 1 && dim <= 512; }

void launch_sq8_scan(const Sq8Args &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  const bool l2 = metric == L2;
  switch (a.dp / 32) {
#define SQ8_CASE(N)                             \
  case N:                                       \
    if (l2) launch_nk<N, L2>(a, max_items, st); \
    else launch_nk<N, IP>(a, max_items, st);    \
    break;
    SQ8_CASE(1)
    SQ8_CASE(2)
    SQ8_CASE(3)
    SQ8_CASE(4)
    SQ8_CASE(5)
    SQ8_CASE(6)
    SQ8_CASE(7)
    SQ8_CASE(8)
    SQ8_CASE(10)
    SQ8_CASE(12)
    SQ8_CASE(16)
#undef SQ8_CASE
    default: break;
  }
}

}  // namespace pyr
