// pq32.hip -- the IVF_PQ list scan on the matrix cores (gfx950).
//
// IvfPqVectorIndex.Search (src/Pyrope.GarnetServer/Vector/IvfPqVectorIndex.cs:118-212) scores a row of a
// probed list by the ADC sum  distSq = sum_m table[m][code_m]  (:182-194) with
// table[m][j] = L2SquaredUnsafe(r_m, C[m][j]) of the query residual r = q - c(list)
// (ProductQuantizer.cs:98-120) and ranks by -distSq.  One LDS table lookup per (query, row, subspace)
// (pq_adc4_kernel, kernels.hip) is bound by the LDS gather rate.  Here the same score is reached the way
// the IVF_FLAT stream scan reaches its own (scan.hip):
//
//   -distSq  =  -|r - x^|^2  =  2 r.x^ - |x^|^2 - |r|^2        (real arithmetic)
//
// with x^ the decoded residual (the concatenated sub-centroids C[m][code_m]).  r.x^ runs on
// v_mfma_f32_32x32x16_f16 with the rows as the A operand: lane (r, h) of k-step s holds dims
// 16 s + 8 h .. +7 of row r, decoded from the fp16 codebook (cb16 [M][256][dsub], L2-resident) by the
// code(s) of the subspace(s) those 8 dims fall in -- dsub 8: one 16-byte gather; 16 / 32: one 16-byte
// gather at offset (16 s + 8 h) mod dsub; 4: two 8-byte gathers.  |x^|^2 is a per-row term fixed at
// build.  The approximate score plus the error bound of the fp16 filter (stream_ub_terms: the same terms
// as the IVF tiles' -- x^ plays x - c, X = |x^|) bounds the reference's fp32 ADC sum from above; rows whose
// bound reaches the query's sampled threshold are emitted, the best 64 per query merged
// (cand_merge_kernel), and pq_refine_kernel computes the reference's own table sum for them, in m order,
// and certifies the top k (k-th exact > the K1-th bound).  Queries that fail re-run on the LUT scan.
//
// Two tile loops, by the k-step count KS = D / 16:
//   * KS <= 8 (D <= 128, e.g. the registry's d=128 m=4 default): a tile's KS decoded A operands stay in
//     registers while every query group of the item runs against them (up to 16 groups = 512 queries: the
//     query operands fill 128 KiB of LDS);
//   * KS > 8 (P1: D = 768): k-outer -- each decoded k-step feeds PQG groups (<= 144 KiB of query operands:
//     PQG = 4 up to D = 576, 3 up to 768, 2 up to 1152), the accumulators of all groups in registers.
// Items of one list chunk go to one XCD's queue (ivf items in XCD order, IvfChunking::xcd): their blocks
// stream the same codes at about the same time, so the chunk leaves HBM once per XCD L2, not once per item.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <stdexcept>

#include "kernels.h"

namespace pyr {
namespace {

#define PYR_STREAM_EMIT
#include "f16util.h"

__device__ __forceinline__ size_t blk_off(int64_t r, int d, int D) {
  return ((size_t)(r >> 3) * (size_t)D + (size_t)d) * 8 + (size_t)(r & 7);
}
#include "vmath.h"
#include "candmerge.h"
#include "deeprank.h"

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

constexpr int PNW = 16;                 // waves per scan block
constexpr int PSAMPLE_TILES = 2 * PNW;  // the sample pass: the first 32 tiles (1,024 rows) of every list
constexpr int PSV = 2 * PNW;            // sample values per (query, probe): one per (wave, lane half)
constexpr int PEB = 768;                // LDS-staged emitted rows per item
constexpr int PQ_KS_MAX = 72;           // D <= 1152

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }

// ---- geometry ----
struct PqGeo {
  int ks;    // k-steps (D / 16)
  int dsub;  // dims per subspace
  int lw;    // 16-byte code words per lane per tile (the lane's code stream, k-step order)
  int res;   // 1: A-resident tile loop (KS <= 8)
  int kp;    // A-resident: padded k-steps (8); k-outer: query groups per item
  int qmax;  // queries per item
};
PqGeo pq_geo(int dim, int M) {
  PqGeo g{};
  g.ks = dim / 16;
  g.dsub = M > 0 ? dim / M : 0;
  g.lw = (g.ks * (g.dsub == 4 ? 2 : 1) + 15) / 16;
  g.res = g.ks <= 8;  // (16 resident k-steps spill: 64 VGPRs of A besides the accumulator and the row terms)
  if (g.res) {
    g.kp = 8;
    g.qmax = 32 * 16;
  } else {
    g.kp = g.ks <= 36 ? 4 : g.ks <= 48 ? 3 : 2;
    g.qmax = 32 * g.kp;
  }
  return g;
}

// ---- build: the tile layout of the codes, |x^|^2 per row, the fp16 codebook ----
// Lane (r, h) of a 32-row tile reads, k-step by k-step, the code(s) its A fragment (dims 16 s + 8 h .. +7
// of row r) decodes from: dsub 8 -> code[2s + h]; 16 -> code[s]; 32 -> code[s / 2]; 4 -> code[4s + 2h],
// code[4s + 2h + 1].  These bytes, in k-step order, are the lane's code stream: tile t, lane l at
// ((t * 64 + l) * lw * 16), lw 16-byte words (as many bytes as the row has codes at dsub 8 and 4; the
// codes repeat across the two halves at dsub 16 and also across a subspace's two k-steps at 32).
__device__ __forceinline__ int pq_stream_code(int dsub, int h, int b) {  // the subspace of stream byte b
  return dsub == 8 ? 2 * b + h : dsub == 16 ? b : dsub == 32 ? b / 2 : 4 * (b >> 1) + 2 * h + (b & 1);
}
__global__ void pq_pack_kernel(const uint8_t *codes_rm, const int64_t *src, int64_t tot, int M, int ks, int lw,
                               int dsub, const float *cb, int ksub, uint8_t *cpack, float *nrm) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= tot) return;
  const int64_t sr = src[p];
  const int64_t t = p >> 5;
  const int r = (int)(p & 31);
  const int nb = ks * (dsub == 4 ? 2 : 1);  // stream bytes per lane
  for (int h = 0; h < 2; ++h)
    for (int w = 0; w < lw; ++w) {
      uint32_t cw[4] = {0u, 0u, 0u, 0u};
      for (int j = 0; j < 16; ++j) {
        const int bi = 16 * w + j;
        if (bi >= nb || sr < 0) continue;
        const int m = pq_stream_code(dsub, h, bi);
        cw[j >> 2] |= (uint32_t)codes_rm[(size_t)sr * M + m] << (8 * (j & 3));
      }
      *reinterpret_cast<u4v *>(cpack + (((size_t)t * 64 + 32 * h + r) * lw + w) * 16) = (u4v){cw[0], cw[1], cw[2], cw[3]};
    }
  float n = 0.0f;
  if (sr >= 0)
    for (int m = 0; m < M; ++m) {
      const float *v = cb + ((size_t)m * ksub + codes_rm[(size_t)sr * M + m]) * dsub;
      for (int u = 0; u < dsub; ++u) n += v[u] * v[u];
    }
  nrm[p] = n;
}

__global__ void pq_cb16_kernel(const float *cb, int M, int ksub, int dsub, float sc, _Float16 *cb16) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // [M][256][dsub]
  if (e >= (int64_t)M * 256 * dsub) return;
  const int u = (int)(e % dsub);
  const int j = (int)((e / dsub) & 255);
  const int m = (int)(e / ((int64_t)dsub * 256));
  cb16[e] = j < ksub ? (_Float16)(cb[((size_t)m * ksub + j) * dsub + u] * sc) : (_Float16)0.0f;
}

// meta of a position: -|x^|^2 for a visible row, -inf otherwise (a shadowed or padding position)
__global__ void pq_meta_kernel(const float *nrm, const uint8_t *live, int64_t tot, float *meta) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= tot) return;
  const float n = nrm[p];
  meta[p] = !live[p] || isnan(n) ? -INFINITY : isinf(n) ? INFINITY : -n;
}

// ---- the query operands per (list, query) position: one wave per position ----
// r = q - c(list) as the reference forms resQuery (:162-164), its scale, {f, -|r|^2 + E_pair}
__global__ __launch_bounds__(256) void pq_prep_kernel(StreamArgs a, int64_t npos) {
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pos >= npos) return;
  const int D = a.dim;
  const int slot = a.qlist[pos];
  const int q = slot / a.nparts;
  const int lst = a.probes[(size_t)q * a.nprobe + (slot % a.nparts) / a.cmax];
  const float *qp = a.queries + (size_t)q * D, *cp = a.cents + (size_t)lst * D;
  float cq = 0.0f, amax = 0.0f;
  for (int d = lane; d < D; d += 64) {
    const float rv = qp[d] - cp[d];
    cq += rv * rv;
    amax = fmaxf(amax, fabsf(rv));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    cq += __shfl_xor(cq, off);
    amax = fmaxf(amax, __shfl_xor(amax, off));
  }
  const float ep = a.kq * cq + a.kqa * sqrtf(cq);
  const float sq = pow2_scale(amax);
  for (int d = lane; d < D; d += 64) a.bq[(size_t)pos * D + d] = (_Float16)((qp[d] - cp[d]) * sq);  // exact scaling
  if (lane == 0) a.qsc[pos] = make_float2(2.0f / (sq * a.sx), -cq + ep);
}

// ---- decode: the A fragment of k-step s for lane half h; u = its position in the lane's current code
// word (the word's byte u, or bytes 2u, 2u + 1 at dsub 4) ----
template <int DSUB>
constexpr int pq_steps_per_word() { return DSUB == 4 ? 8 : 16; }
template <int DSUB>
__device__ __forceinline__ h8v pq_decode(const uint32_t (&cw)[4], const _Float16 *cb16, int s, int u, int h) {
  auto byte = [&](int b) { return (cw[b >> 2] >> (8 * (b & 3))) & 0xFFu; };
  if constexpr (DSUB == 4) {  // dims 8h .. 8h+7 of the k-step: subspaces 4s + 2h, 4s + 2h + 1
    const uint32_t c0 = byte(2 * u), c1 = byte(2 * u + 1);
    const int m0 = 4 * s + 2 * h;
    const u2v lo = *reinterpret_cast<const u2v *>(cb16 + ((size_t)m0 * 256 + c0) * 4);
    const u2v hi = *reinterpret_cast<const u2v *>(cb16 + ((size_t)(m0 + 1) * 256 + c1) * 4);
    return __builtin_bit_cast(h8v, ((u4v){lo.x, lo.y, hi.x, hi.y}));
  } else if constexpr (DSUB == 8) {  // subspace 2s + h
    return *reinterpret_cast<const h8v *>(cb16 + ((size_t)(2 * s + h) * 256 + byte(u)) * 8);
  } else {  // 16, 32: subspace s / (DSUB / 16); dims (16 s + 8 h) mod DSUB of its sub-centroid
    constexpr int SPK = DSUB / 16;
    return *reinterpret_cast<const h8v *>(cb16 + ((size_t)(s / SPK) * 256 + byte(u)) * DSUB + 16 * (s % SPK) + 8 * h);
  }
}

__device__ __forceinline__ void split_word(const u4v v, uint32_t (&cw)[4]) {
  cw[0] = v.x;
  cw[1] = v.y;
  cw[2] = v.z;
  cw[3] = v.w;
}

// ---- work: per-XCD item queues (n_items[1 .. 9]: the queues' item bounds; work[0 .. 7]: their counters).
// A block takes items from the queue of its XCD group (blockIdx % 8: blocks b and b + 8 share an XCD),
// then from the others'.  Thread 0 only; qx / tried persist across the block's items.
__device__ __forceinline__ int pq_next_item(const StreamArgs &a, int &qx, int &tried) {
  const int32_t *qb = a.n_items + 1;
  while (tried < 8) {
    const int t = atomicAdd(a.work + qx, 1);
    if (qb[qx] + t < qb[qx + 1]) return qb[qx] + t;
    qx = (qx + 1) & 7;
    ++tried;
  }
  return -1;
}

// per-item LDS state shared by both tile loops
template <int QMAX>
struct PqItemLds {
  float2 qf[QMAX], qz[QMAX];  // {f, lowered T - cq} / {cq, query (main) or sample slot (SAMPLE)}
  int cnt_l[QMAX], base_l[QMAX];
  uint2 eb[PEB];
  int item, eb_n;
};

// prologue: the item's query operands into LDS (piece (j, s) = group j, k-step s at (j * kstride + s) KiB;
// lane (r, h) carries dims 16 s + 8 h .. +7 of query 32 j + r) and its per-query scalars
template <int QMAX, bool SAMPLE>
__device__ __forceinline__ void pq_item_prologue(const StreamArgs &a, const ScanItem &it, int KS, int kstride,
                                                 uint32_t bl_base, PqItemLds<QMAX> &L) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int qcnt = it.qcnt, ng = (qcnt + 31) >> 5;
  for (int p = w; p < ng * KS; p += PNW) {
    const int j = p / KS, s = p - j * KS;
    const int qi = min(32 * j + r, qcnt - 1);
    glds<16>(a.bq + (size_t)(it.qbeg + qi) * a.dim + 16 * s + 8 * h, bl_base + (uint32_t)((j * kstride + s) * 1024));
  }
  for (int i = tid; i < ng * 32; i += 64 * PNW) {
    float2 v = make_float2(0.0f, __builtin_nanf(""));
    float cqv = 0.0f;
    int o = -1;
    if (i < qcnt) {
      const int pos = it.qbeg + i;
      const int slot = a.qlist[pos];
      const float2 fc = a.qsc[pos];
      const int q = slot / a.nparts;
      const float T = (!SAMPLE && a.thr) ? a.thr[q] : -INFINITY;
      v = make_float2(fc.x, lower_thr(T, fc.y));
      cqv = fc.y;
      o = SAMPLE ? q * a.nprobe + (slot % a.nparts) / a.cmax : q;
    }
    L.qf[i] = v;
    L.qz[i] = make_float2(cqv, __int_as_float(o));
    L.cnt_l[i] = 0;
  }
  if (tid == 0) L.eb_n = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// the row terms of tile t: lane (r, h) holds rows rt + 8b + 4h + i (b < 4, i < 4), the 32x32 C layout
__device__ __forceinline__ void pq_row_terms(const StreamArgs &a, int rt, int rlim, int h, float (&mr)[16]) {
  const size_t mo = (size_t)rt + 4 * h;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const f4v m4 = *reinterpret_cast<const f4v *>(a.mub + mo + 8 * b);
#pragma unroll
    for (int i = 0; i < 4; ++i) mr[4 * b + i] = rt + 8 * b + 4 * h + i < rlim ? m4[i] : -INFINITY;
  }
}

// epilogue of group g against one tile (main pass): bounds -> emitted rows (LDS-staged, or straight to
// the query's buffer when the stage is full / the chunk too long for the packed row offset)
template <int QMAX>
__device__ __forceinline__ void pq_emit(const StreamArgs &a, f16v acc, int g, int r, int h, int rt, int r0, bool stage,
                                        const float (&mr)[16], PqItemLds<QMAX> &L) {
  const int qi = 32 * g + r;
  const float2 q = L.qf[qi];
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = fmaf(q.x, acc[v], mr[v]);
  float mx = max3f(acc[0], acc[1], acc[2]);
#pragma unroll
  for (int v = 3; v < 15; v += 2) mx = max3f(mx, acc[v], acc[v + 1]);
  mx = fmaxf(mx, acc[15]);
  if (__builtin_amdgcn_ballot_w64(mx >= q.y) == 0ull) return;
  const float cq = L.qz[qi].x;
  uint32_t base = ((uint32_t)qi << 23) | (uint32_t)(rt - r0 + 4 * h);
  asm volatile("" : "+v"(base));
  // 4-row blocks first (one ballot each), then the rows of a block that can emit (as scan.hip's emit_y)
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const float bm = fmaxf(max3f(acc[4 * b], acc[4 * b + 1], acc[4 * b + 2]), acc[4 * b + 3]);
    if (__builtin_amdgcn_ballot_w64(bm >= q.y) == 0ull) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = 4 * b + i;
      const bool p = acc[e] >= q.y;
      if (__builtin_amdgcn_ballot_w64(p) == 0ull) continue;
      if (p) {
        const float sc = acc[e] + cq;
        const uint32_t word = base + (uint32_t)(8 * (e >> 2) + (e & 3));
        const int at = stage ? atomicAdd(&L.eb_n, 1) : PEB;
        if (at < PEB) L.eb[at] = make_uint2(__float_as_uint(sc), word);
        else cand_put(a, __float_as_int(L.qz[qi].y), sc, a.key_base | (uint32_t)(r0 + (int)(word & 0x7FFFFFu)));
      }
    }
  }
}

__device__ __forceinline__ float pq_tile_max(const f16v &acc, float f, const float (&mr)[16]) {
  float y[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) y[v] = fmaf(f, acc[v], mr[v]);
  float mx = max3f(y[0], y[1], y[2]);
#pragma unroll
  for (int v = 3; v < 15; v += 2) mx = max3f(mx, y[v], y[v + 1]);
  return fmaxf(mx, y[15]);
}

// ---- tile loop 1 (KS <= 16): decoded A resident, every group against it ----
template <int KSP, int DSUB, bool SAMPLE>
__global__ __launch_bounds__(64 * PNW, 1) void pq_scan_res_kernel(StreamArgs a, const _Float16 *cb16, int lw) {
  constexpr int QG = KSP <= 8 ? 16 : 8;
  constexpr int QMAX = 32 * QG;
  constexpr int SPW = pq_steps_per_word<DSUB>();
  constexpr int NW = (KSP + SPW - 1) / SPW;  // code words covering KSP k-steps
  __shared__ __attribute__((aligned(16))) char bl[QG * KSP * 1024];
  __shared__ PqItemLds<QMAX> L;
  const uint32_t bl_base = (uint32_t)(size_t)(lds_void *)bl;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const uint8_t *cpk = reinterpret_cast<const uint8_t *>(a.h16);
  const int KS = a.dim >> 4;
  int qx = blockIdx.x & 7, tried = 0;

  for (;;) {
    if (tid == 0) L.item = pq_next_item(a, qx, tried);
    __syncthreads();
    const int item = L.item;
    __syncthreads();
    if (item < 0) return;
    const ScanItem it = a.items[item];
    if (SAMPLE && it.part != 0) continue;
    pq_item_prologue<QMAX, SAMPLE>(a, it, KS, KSP, bl_base, L);
    const int qcnt = it.qcnt, ng = (qcnt + 31) >> 5;
    const int r0 = it.row_begin;
    int nt = (it.row_end - r0 + 31) >> 5;
    if (SAMPLE) nt = min(nt, PSAMPLE_TILES);
    const int rlim = it.row_end;
    const bool stage = it.row_end - r0 < (1 << 23);
    float smx[SAMPLE ? QG : 1];
#pragma unroll
    for (int g = 0; g < (SAMPLE ? QG : 1); ++g) smx[g] = -INFINITY;
#pragma unroll 1
    for (int t = w; t < nt; t += PNW) {
      const int rt = r0 + 32 * t;
      h8v A[KSP];
      {
        const u4v *cp = reinterpret_cast<const u4v *>(cpk + ((size_t)(rt >> 5) * 64 + lane) * lw * 16);
#pragma unroll
        for (int wi = 0; wi < NW; ++wi) {
          uint32_t cw[4] = {0u, 0u, 0u, 0u};
          if (wi < lw) split_word(cp[wi], cw);
#pragma unroll
          for (int u = 0; u < SPW; ++u) {
            const int s = wi * SPW + u;
            if (s >= KSP) break;
            A[s] = s < KS ? pq_decode<DSUB>(cw, cb16, s, u, h) : (h8v){};
          }
        }
      }
      float mr[16];
      pq_row_terms(a, rt, rlim, h, mr);
      auto group = [&](int g) {
        f16v acc = {};
#pragma unroll
        for (int s = 0; s < KSP; ++s) {
          if (s >= KS) break;
          const h8v B = *reinterpret_cast<const h8v *>(bl + (g * KSP + s) * 1024 + lane * 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], B, acc, 0, 0, 0);
        }
        return acc;
      };
      if constexpr (SAMPLE) {
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          if (g >= ng) break;
          smx[g] = fmaxf(smx[g], pq_tile_max(group(g), L.qf[32 * g + r].x, mr));
        }
      } else {
#pragma unroll 1
        for (int g = 0; g < ng; ++g) pq_emit<QMAX>(a, group(g), g, r, h, rt, r0, stage, mr, L);
      }
    }
    if constexpr (SAMPLE) {
#pragma unroll
      for (int g = 0; g < QG; ++g) {
        const int qi = 32 * g + r;
        if (qi < qcnt) a.samp[(size_t)__float_as_int(L.qz[qi].y) * PSV + 2 * w + h] = smx[g] + L.qz[qi].x;
      }
      __syncthreads();
      continue;
    }
    __syncthreads();
    cand_flush<64 * PNW>(a, L.eb, min(L.eb_n, PEB), qcnt, r0, L.cnt_l, L.base_l,
                         [&](int i) { return __float_as_int(L.qz[i].y); });
  }
}

// ---- tile loop 2 (KS > 16): k-outer, each decoded k-step against PQG groups ----
template <int PQG, int DSUB, bool SAMPLE>
__global__ __launch_bounds__(64 * PNW, 1) void pq_scan_kout_kernel(StreamArgs a, const _Float16 *cb16, int lw) {
  constexpr int QMAX = 32 * PQG;
  constexpr int SPW = pq_steps_per_word<DSUB>();  // k-steps per code word
  __shared__ __attribute__((aligned(16))) char bl[144 * 1024];
  __shared__ PqItemLds<QMAX> L;
  const uint32_t bl_base = (uint32_t)(size_t)(lds_void *)bl;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const uint8_t *cpk = reinterpret_cast<const uint8_t *>(a.h16);
  const int KS = a.dim >> 4;
  int qx = blockIdx.x & 7, tried = 0;

  for (;;) {
    if (tid == 0) L.item = pq_next_item(a, qx, tried);
    __syncthreads();
    const int item = L.item;
    __syncthreads();
    if (item < 0) return;
    const ScanItem it = a.items[item];
    if (SAMPLE && it.part != 0) continue;
    pq_item_prologue<QMAX, SAMPLE>(a, it, KS, KS, bl_base, L);
    const int qcnt = it.qcnt, ng = (qcnt + 31) >> 5;
    const int r0 = it.row_begin;
    int nt = (it.row_end - r0 + 31) >> 5;
    if (SAMPLE) nt = min(nt, PSAMPLE_TILES);
    const int rlim = it.row_end;
    const bool stage = it.row_end - r0 < (1 << 23);
    float smx[PQG];
#pragma unroll
    for (int g = 0; g < PQG; ++g) smx[g] = -INFINITY;
#pragma unroll 1
    for (int t = w; t < nt; t += PNW) {
      const int rt = r0 + 32 * t;
      const u4v *cp = reinterpret_cast<const u4v *>(cpk + ((size_t)(rt >> 5) * 64 + lane) * lw * 16);
      f16v acc[PQG];
#pragma unroll
      for (int g = 0; g < PQG; ++g) acc[g] = (f16v){};
      u4v nxt = cp[0];  // the next word of the lane's code stream, loaded one word ahead
#pragma unroll 1
      for (int wi = 0; wi < lw; ++wi) {
        uint32_t cw[4];
        split_word(nxt, cw);
        if (wi + 1 < lw) nxt = cp[wi + 1];
#pragma unroll
        for (int u = 0; u < SPW; ++u) {
          const int s = wi * SPW + u;
          if (s >= KS) break;
          const h8v A = pq_decode<DSUB>(cw, cb16, s, u, h);
#pragma unroll
          for (int g = 0; g < PQG; ++g) {
            if (g >= ng) break;  // (wave-uniform) a short item skips the empty groups' MFMAs
            const h8v B = *reinterpret_cast<const h8v *>(bl + (g * KS + s) * 1024 + lane * 16);
            acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, B, acc[g], 0, 0, 0);
          }
        }
      }
      float mr[16];
      pq_row_terms(a, rt, rlim, h, mr);
#pragma unroll
      for (int g = 0; g < PQG; ++g) {
        if (g >= ng) break;
        if constexpr (SAMPLE) smx[g] = fmaxf(smx[g], pq_tile_max(acc[g], L.qf[32 * g + r].x, mr));
        else pq_emit<QMAX>(a, acc[g], g, r, h, rt, r0, stage, mr, L);
      }
    }
    if constexpr (SAMPLE) {
#pragma unroll
      for (int g = 0; g < PQG; ++g) {
        const int qi = 32 * g + r;
        if (qi < qcnt) a.samp[(size_t)__float_as_int(L.qz[qi].y) * PSV + 2 * w + h] = smx[g] + L.qz[qi].x;
      }
      __syncthreads();
      continue;
    }
    __syncthreads();
    cand_flush<64 * PNW>(a, L.eb, min(L.eb_n, PEB), qcnt, r0, L.cnt_l, L.base_l,
                         [&](int i) { return __float_as_int(L.qz[i].y); });
  }
}

// ---- refine: the reference's ADC sum of the merged candidates, top k, certificate ----
// One wave per query; lane l holds merged candidate l (bound ms, position mk: >= 0 a row, -2 a floor,
// -1 none).  A lane's exact score: resQuery of the row's list, then distSq += table[m][code_m] in m
// order (IvfPqVectorIndex.cs:182-194; table entries L2SquaredUnsafe, ProductQuantizer.cs:107-117).
struct Res {  // resQuery_m on the fly: q_i - c_i, the reference's fp32 subtraction
  const float *q, *c;
  __device__ float operator()(int i) const { return q[i] - c[i]; }
};
__global__ __launch_bounds__(256) void pq_refine_kernel(PqRefineArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nsel = a.nsel ? *a.nsel : a.nq;
  if (wq >= nsel) return;
  const int64_t q = a.qsel ? a.qsel[wq] : wq;
  const int K1 = a.k1;
  float sc = -INFINITY;
  int32_t key = lane < K1 ? a.mk[q * a.ld + lane] : -1;
  if (key >= 0) {
    int lo = 0, hi = a.nlist;  // the row's list: lb[lo] <= key < lb[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (a.lb[mid] <= key) lo = mid;
      else hi = mid;
    }
    const float *qv = a.queries + (size_t)q * a.dim;
    const float *cv = a.cents + (size_t)lo * a.dim;
    const uint8_t *tp = a.cpack + (size_t)(key >> 5) * 64 * a.lw * 16;  // the row's tile
    const int ds = a.dsub, r = key & 31;
    float dist = 0.0f;
    for (int m = 0; m < a.M; ++m) {
      // code m in the code stream of lane (r, h) (pq_pack_kernel): its k-step's byte
      const int h = ds == 8 ? (m & 1) : ds == 4 ? ((m >> 1) & 1) : 0;
      const int b = ds == 8 ? m >> 1 : ds == 16 ? m : ds == 32 ? 2 * m : 2 * (m >> 2) + (m & 1);
      const int c = tp[(size_t)(32 * h + r) * a.lw * 16 + b];
      dist = dist + em_l2sq_unsafe(Res{qv + m * ds, cv + m * ds}, Off{a.codebooks + ((size_t)m * a.ksub + c) * ds}, ds);
    }
    sc = -dist;
  }
  // rank (score desc, position asc) among the real candidates: each lane its rank by counting
  int rank = 0;
  for (int j = 0; j < 64; ++j) {
    const float sj = __shfl(sc, j);
    const int kj = __shfl(key, j);
    if (kj < 0 || key < 0) continue;
    if (sj > sc || (sj == sc && kj < key)) ++rank;
  }
  const int nreal = __popcll(__builtin_amdgcn_ballot_w64(key >= 0));
  // the k-th exact score and the K1-th bound (every row outside the first K1 is bounded by it)
  float kth = -INFINITY;
  for (int j = 0; j < 64; ++j) {
    const int rj = __shfl(rank, j);
    const int kj = __shfl(key, j);
    const float sj = __shfl(sc, j);
    if (kj >= 0 && rj == a.k - 1) kth = sj;
  }
  const float bound = a.ms[q * a.ld + K1 - 1];
  // fewer than K1 merged entries: no floor placeholder, so every visible row of the probed lists was
  // emitted and the candidates are all of them
  const bool full = a.mk[q * a.ld + K1 - 1] == -1;
  const bool ok = full || (nreal >= a.k && kth > bound);
  if (ok) {
    if (key >= 0 && rank < a.k) {
      a.out_s[q * a.k + rank] = sc;
      a.out_l[q * a.k + rank] = a.labels[key];
    }
    if (lane >= nreal && lane < a.k) {
      a.out_s[q * a.k + lane] = -INFINITY;
      a.out_l[q * a.k + lane] = -1;
    }
    if (a.out_c && lane == 0) a.out_c[q] = min(nreal, a.k);
  } else if (lane == 0) {
    a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
  }
}

// k > 60 (round 6): the merge + certified refine at depth K1 = 128 / 256 / 512 on the emitted
// rows (deeprank.h), one block per query.  A candidate's exact score is pq_refine_kernel's ADC sum: its 8-lane
// group computes the terms m = 8 i + l in parallel and every lane adds them in m order (distSq += table[m][code],
// IvfPqVectorIndex.cs:182-194), so the sum is bit-identical to the serial loop's.  Certified as refine_kernel's
// upper-bound branch (the K1 best rows, or every emitted row above the floor); a.qsel / a.nsel: only the queries a
// shallower pass failed (the grid is sized for all nq).  What fails re-runs on the LUT scan.
__global__ __launch_bounds__(256) void pq_deep_refine_kernel(CandMergeArgs m, PqRefineArgs a) {
  extern __shared__ uint64_t dk[];
  const int64_t nsel = a.nsel ? *a.nsel : a.nq;  // (a.qsel: the queries a shallower pass failed)
  if ((int64_t)blockIdx.x >= nsel) return;
  const int64_t q = a.qsel ? a.qsel[blockIdx.x] : (int64_t)blockIdx.x;
  const float *qv = a.queries + (size_t)q * a.dim;
  const int base = threadIdx.x & 56, ds = a.dsub;
  const DeepRank R = deep_select_rank(m, q, a.k1, dk, [&](uint32_t key, int l) {
    int lo = 0, hi = a.nlist;  // the row's list: lb[lo] <= key < lb[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (a.lb[mid] <= (int32_t)key) lo = mid;
      else hi = mid;
    }
    const float *cv = a.cents + (size_t)lo * a.dim;
    const uint8_t *tp = a.cpack + (size_t)(key >> 5) * 64 * a.lw * 16;  // the row's tile
    const int r = key & 31;
    float dist = 0.0f;
    for (int m0 = 0; m0 < a.M; m0 += 8) {
      const int mm = m0 + l;
      float t = 0.0f;
      if (mm < a.M) {  // code mm in the code stream of lane (r, h) (pq_pack_kernel): its k-step's byte
        const int h = ds == 8 ? (mm & 1) : ds == 4 ? ((mm >> 1) & 1) : 0;
        const int b = ds == 8 ? mm >> 1 : ds == 16 ? mm : ds == 32 ? 2 * mm : 2 * (mm >> 2) + (mm & 1);
        const int c = tp[(size_t)(32 * h + r) * a.lw * 16 + b];
        t = em_l2sq_unsafe(Res{qv + mm * ds, cv + mm * ds}, Off{a.codebooks + ((size_t)mm * a.ksub + c) * ds}, ds);
      }
      const int nm = min(8, a.M - m0);
      for (int u = 0; u < nm; ++u) dist = dist + __shfl(t, base + u);
    }
    return -dist;
  });
  const bool ok = (!R.excluded || (min(R.j, a.k) == a.k && deep_kth(R, a.k) > R.bound)) && !R.nan;
  deep_write(R, q, a.k, ok, a.labels, a.out_s, a.out_l, a.out_c, a.fail_list, a.fail_cnt);
}

template <class K>
void pq_launch(K kern, int grid, const StreamArgs &a, const _Float16 *cb16, int lw, hipStream_t st) {
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * PNW), 0, st, a, cb16, lw);
}
template <int DSUB>
void launch_scan_dsub(const StreamArgs &a, const _Float16 *cb16, const PqGeo &g, int grid, bool sample, hipStream_t st) {
  if (g.res) {
    if (sample) pq_launch(pq_scan_res_kernel<8, DSUB, true>, grid, a, cb16, g.lw, st);
    else pq_launch(pq_scan_res_kernel<8, DSUB, false>, grid, a, cb16, g.lw, st);
  } else if (g.kp == 4) {
    if (sample) pq_launch(pq_scan_kout_kernel<4, DSUB, true>, grid, a, cb16, g.lw, st);
    else pq_launch(pq_scan_kout_kernel<4, DSUB, false>, grid, a, cb16, g.lw, st);
  } else if (g.kp == 3) {
    if (sample) pq_launch(pq_scan_kout_kernel<3, DSUB, true>, grid, a, cb16, g.lw, st);
    else pq_launch(pq_scan_kout_kernel<3, DSUB, false>, grid, a, cb16, g.lw, st);
  } else {
    if (sample) pq_launch(pq_scan_kout_kernel<2, DSUB, true>, grid, a, cb16, g.lw, st);
    else pq_launch(pq_scan_kout_kernel<2, DSUB, false>, grid, a, cb16, g.lw, st);
  }
}

}  // namespace

bool pq32_supported(int dim, int M, int ksub, int k) {
  if (M <= 0 || dim <= 0 || dim % 16 != 0 || dim % M != 0) return false;
  const int dsub = dim / M;
  return (dsub == 4 || dsub == 8 || dsub == 16 || dsub == 32) && dim / 16 <= PQ_KS_MAX && ksub >= 1 && ksub <= 256 &&
         k >= 1 && k <= 256;  // k > 60: the deep refine (the engine checks its depth)
}
int pq32_qmax(int dim, int M) { return pq_geo(dim, M).qmax; }
int pq32_sample_values() { return PSV; }
int pq32_lane_words(int dim, int M) { return pq_geo(dim, M).lw; }

void launch_pq32_pack(const uint8_t *codes_rm, const int64_t *src, int64_t tot, int M, int dsub, const float *cb,
                      int ksub, uint8_t *cpack, float *nrm, hipStream_t st) {
  if (tot <= 0) return;
  const PqGeo g = pq_geo(M * dsub, M);
  hipLaunchKernelGGL(pq_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, codes_rm, src, tot, M,
                     g.ks, g.lw, dsub, cb, ksub, cpack, nrm);
}
void launch_pq32_cb16(const float *cb, int M, int ksub, int dsub, float sc, _Float16 *cb16, hipStream_t st) {
  const int64_t n = (int64_t)M * 256 * dsub;
  hipLaunchKernelGGL(pq_cb16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cb, M, ksub, dsub, sc,
                     cb16);
}
void launch_pq32_meta(const float *nrm, const uint8_t *live, int64_t tot, float *meta, hipStream_t st) {
  if (tot <= 0) return;
  hipLaunchKernelGGL(pq_meta_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, nrm, live, tot, meta);
}
void launch_pq32_prep(const StreamArgs &a, int64_t npos, hipStream_t st) {
  if (npos <= 0) return;
  hipLaunchKernelGGL(pq_prep_kernel, dim3((unsigned)((npos + 3) / 4)), dim3(256), 0, st, a, npos);
}
void launch_pq32_scan(const StreamArgs &a, const _Float16 *cb16, int M, int max_items, bool sample, hipStream_t st) {
  if (max_items <= 0) return;
  const PqGeo g = pq_geo(a.dim, M);
  if (a.dim % 16 != 0 || g.ks > PQ_KS_MAX) throw std::runtime_error("pq32: unsupported dimension");
  // one block per CU (launch_bounds 1 block): a multiple of the 8 XCDs keeps the queues' block counts equal
  const int grid = std::max(8, std::min((max_items + 7) / 8 * 8, device_cus()));
  switch (g.dsub) {
    case 4: launch_scan_dsub<4>(a, cb16, g, grid, sample, st); break;
    case 8: launch_scan_dsub<8>(a, cb16, g, grid, sample, st); break;
    case 16: launch_scan_dsub<16>(a, cb16, g, grid, sample, st); break;
    case 32: launch_scan_dsub<32>(a, cb16, g, grid, sample, st); break;
    default: throw std::runtime_error("pq32: unsupported subspace size");
  }
}
void launch_pq32_deep_refine(const CandMergeArgs &m, const PqRefineArgs &a, hipStream_t st) {
  if (a.nq <= 0) return;
  if (a.k1 > DEEP_MAX || a.k1 < a.k || a.k > 256) throw std::invalid_argument("pq32 deep refine: depth");
  constexpr int LDS_MAX = 144 * 1024;  // as launch_deep_refine's (filter.hip)
  const size_t lds = deep_refine_lds_bytes(m.cap, a.k1);
  if (lds > (size_t)LDS_MAX) throw std::invalid_argument("pq32 deep refine: candidate buffer too large");
  static std::atomic<uint64_t> done{0};
  allow_max_lds(reinterpret_cast<const void *>(&pq_deep_refine_kernel), done, LDS_MAX);
  hipLaunchKernelGGL(pq_deep_refine_kernel, dim3((unsigned)a.nq), dim3(256), lds, st, m, a);
}
void launch_pq32_refine(const PqRefineArgs &a, int64_t nq, hipStream_t st) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(pq_refine_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, st, a);
}

}  // namespace pyr
