// pq32.hip -- the IVF_PQ list scan on the matrix cores (gfx950, round 4).
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
// v_mfma_f32_32x32x16_f16: a 32-row tile is decoded on the fly, k-step s (16 dims = subspaces 2s, 2s+1,
// dsub = 8) of lane (r, h) being the fp16 sub-centroid C[2s + h][code] gathered from the fp16 codebook
// (393 KB at P1, L2-resident).  |x^|^2 is a per-row term fixed at build.  The approximate score plus the
// error bound of the fp16 filter (stream_ub_terms: the same terms as the IVF tiles' -- x^ plays x - c,
// X = |x^|) bounds the reference's fp32 ADC sum from above; rows whose bound reaches the query's sampled
// threshold are emitted, the best 64 per query merged (cand_merge_kernel), and pq_refine_kernel computes
// the reference's own table sum for them, in m order, and certifies the top k (k-th exact > the K1-th
// bound).  Queries that fail are re-run on the LUT path (engine.cpp).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

#define PYR_STREAM_EMIT
#include "f16util.h"

__device__ __forceinline__ size_t blk_off(int64_t r, int d, int D) {
  return ((size_t)(r >> 3) * (size_t)D + (size_t)d) * 8 + (size_t)(r & 7);
}
#include "vmath.h"

constexpr int PNW = 16;      // waves per scan block
constexpr int PQG = 3;       // 32-query groups per item (96 queries: 144 KiB of operands at D = 768)
constexpr int PQMAX = 32 * PQG;
constexpr int PSAMPLE_TILES = 2 * PNW;
constexpr int PSV = 2 * PNW;  // sample values per (query, probe): one per (wave, lane half)

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }

// ---- build: the tile layout of the codes, |x^|^2 per row, the fp16 codebook ----
// tile t (rows 32t .. 32t + 31 of the list-major positions), lane l = 32h + r: bytes s = 0 .. M/2 - 1 are
// code[row 32t + r][2s + h], at ((t * 64 + l) * MB + s)
__global__ void pq_pack_kernel(const uint8_t *codes_rm, const int64_t *src, int64_t tot, int M, int MB,
                               const float *cb, int ksub, uint8_t *cpack, float *nrm) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= tot) return;
  const int64_t sr = src[p];
  const int64_t t = p >> 5;
  const int r = (int)(p & 31);
  float n = 0.0f;
  for (int m = 0; m < M; ++m) {
    const int c = sr >= 0 ? codes_rm[(size_t)sr * M + m] : 0;
    cpack[((size_t)t * 64 + (m & 1) * 32 + r) * MB + (m >> 1)] = (uint8_t)c;
    if (sr >= 0) {
      const float *v = cb + ((size_t)m * ksub + c) * 8;
#pragma unroll
      for (int u = 0; u < 8; ++u) n += v[u] * v[u];
    }
  }
  nrm[p] = n;
}

__global__ void pq_cb16_kernel(const float *cb, int M, int ksub, float sc, _Float16 *cb16) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // [M][256][8]
  if (e >= (int64_t)M * 256 * 8) return;
  const int j = (int)((e >> 3) & 255), m = (int)(e >> 11), u = (int)(e & 7);
  cb16[e] = j < ksub ? (_Float16)(cb[((size_t)m * ksub + j) * 8 + u] * sc) : (_Float16)0.0f;
}

// meta of a position: -|x^|^2 for a visible row, -inf otherwise (a shadowed or padding position)
__global__ void pq_meta_kernel(const float *nrm, const uint8_t *live, int64_t tot, float *meta) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= tot) return;
  const float n = nrm[p];
  meta[p] = !live[p] || isnan(n) ? -INFINITY : isinf(n) ? INFINITY : -n;
}

// ---- the query operands per (list, query) pair: one wave per pair ----
// r = q - c(list) as the reference forms resQuery (:162-164), its scale, {f, -|r|^2 + E_pair}
template <int D>
__global__ __launch_bounds__(256) void pq_prep_kernel(StreamArgs a) {
  constexpr int PER = D / 64;  // dims per lane
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int item = unit / PQMAX, qi = unit - item * PQMAX;
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  if (it.part != 0 || qi >= it.qcnt) return;
  const int pos = it.qbeg + qi;
  const int q = a.qlist[pos] / a.nparts;
  float rv[PER], cq = 0.0f, amax = 0.0f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int d = lane + 64 * u;
    rv[u] = a.queries[(size_t)q * D + d] - a.cents[(size_t)it.list * D + d];
    cq += rv[u] * rv[u];
    amax = fmaxf(amax, fabsf(rv[u]));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    cq += __shfl_xor(cq, off);
    amax = fmaxf(amax, __shfl_xor(amax, off));
  }
  const float ep = a.kq * cq + a.kqa * sqrtf(cq);
  const float sq = pow2_scale(amax);
#pragma unroll
  for (int u = 0; u < PER; ++u) a.bq[(size_t)pos * D + lane + 64 * u] = (_Float16)(rv[u] * sq);
  if (lane == 0) a.qsc[pos] = make_float2(2.0f / (sq * a.sx), -cq + ep);
}

// ---- the scan (SAMPLE: the first PSAMPLE_TILES tiles of every list, maxima per (wave, lane half)) ----
// a.h16: the tile code layout (pq_pack_kernel); a.cents doubles as nothing; pq: the fp16 codebook
template <int D, bool SAMPLE, int AB = 0>
__global__ __launch_bounds__(64 * PNW, 1) void pq_scan_kernel(StreamArgs a, const _Float16 *cb16) {
  constexpr int KS = D / 16;                 // k-steps = subspace pairs
  constexpr int MB = (KS + 15) / 16 * 16;    // code bytes per lane per tile
  constexpr int PIECES = PQG * KS;
  __shared__ __attribute__((aligned(16))) char bl[PIECES * 1024];
  __shared__ float2 qf[PQMAX], qz[PQMAX];
  __shared__ int cnt_l[PQMAX];       // the item's staged rows per query slot (cand_flush)
  __shared__ int base_l[PQMAX];
  __shared__ int item_sh, eb_n;
  constexpr int EB = 768;
  __shared__ uint2 eb[EB];
  const uint32_t bl_base = (uint32_t)(size_t)(lds_void *)bl;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const uint8_t *cpk = reinterpret_cast<const uint8_t *>(a.h16);

  for (;;) {
    if (tid == 0) item_sh = atomicAdd(a.work, 1);
    __syncthreads();
    const int item = item_sh;
    __syncthreads();
    if (item >= *a.n_items) return;
    const ScanItem it = a.items[item];
    if (SAMPLE && it.part != 0) continue;
    const int qcnt = it.qcnt, ng = (qcnt + 31) >> 5;
    {
      for (int p = w; p < ng * KS; p += PNW) {
        const int j = p / KS, s = p - j * KS;
        const int qi = min(32 * j + r, qcnt - 1);
        glds<16>(a.bq + (size_t)(it.qbeg + qi) * D + 16 * s + 8 * h, bl_base + (uint32_t)(p * 1024));
      }
      for (int i = tid; i < PQMAX; i += 64 * PNW) {
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
        qf[i] = v;
        qz[i] = make_float2(cqv, __int_as_float(o));
        cnt_l[i] = 0;
      }
      if (tid == 0) eb_n = 0;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const int r0 = it.row_begin;
    int nt = (it.row_end - r0 + 31) >> 5;
    if (SAMPLE) nt = min(nt, PSAMPLE_TILES);
    const int rlim = it.row_end;
    const bool stage = it.row_end - r0 < (1 << 23);

    auto put = [&](int qi, float sc, int row) { cand_put(a, __float_as_int(qz[qi].y), sc, a.key_base | (uint32_t)row); };
    float smx[PQG];  // SAMPLE: this lane's best bound per query group
#pragma unroll
    for (int g = 0; g < PQG; ++g) smx[g] = -INFINITY;
#pragma unroll 1
    for (int t = w; t < nt; t += PNW) {
      const uint4 *cp = reinterpret_cast<const uint4 *>(cpk + ((size_t)(r0 / 32 + t) * 64 + lane) * MB);
      float mr[16];
      {
        const int rt = r0 + 32 * t;
        const size_t mo = (size_t)rt + 4 * h;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const f4v m4 = *reinterpret_cast<const f4v *>(a.mub + mo + 8 * b);
#pragma unroll
          for (int i = 0; i < 4; ++i) mr[4 * b + i] = rt + 8 * b + 4 * h + i < rlim ? m4[i] : -INFINITY;
        }
      }
      // k-outer: decode k-step s (one 16-B gather per lane) and run it against every group, 16 k-steps
      // (one 16-byte word of codes) at a time
      f16v acc[PQG];
#pragma unroll
      for (int g = 0; g < PQG; ++g) acc[g] = (f16v){};
      const char *cbb = reinterpret_cast<const char *>(cb16) + (size_t)h * 256 * 16;
#pragma unroll 1
      for (int i = 0; i < MB / 16; ++i) {
        const uint4 cv = cp[i];
        const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int s = 16 * i + u;
          if (s >= KS) break;
          const uint32_t c = (cw[u >> 2] >> (8 * (u & 3))) & 0xFFu;
          h8v A;
          if constexpr (AB == 2) A = (h8v){};  // measurement only: no decode gathers
          else A = *reinterpret_cast<const h8v *>(cbb + (size_t)(2 * s) * 256 * 16 + c * 16);
#pragma unroll
          for (int g = 0; g < PQG; ++g) {
            if (g >= ng) break;  // (wave-uniform) a short item skips the empty groups' MFMAs
            const h8v B = *reinterpret_cast<const h8v *>(bl + (g * KS + s) * 1024 + lane * 16);
            acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, B, acc[g], 0, 0, 0);
          }
        }
      }
      const int rt = r0 + 32 * t;
#pragma unroll
      for (int g = 0; g < PQG; ++g) {
        if (g >= ng) break;
        const int qi = 32 * g + r;
        const float2 q = qf[qi];
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[g][v] = fmaf(q.x, acc[g][v], mr[v]);
        float mx = max3f(acc[g][0], acc[g][1], acc[g][2]);
#pragma unroll
        for (int v = 3; v < 15; v += 2) mx = max3f(mx, acc[g][v], acc[g][v + 1]);
        mx = fmaxf(mx, acc[g][15]);
        if constexpr (SAMPLE) {
          smx[g] = fmaxf(smx[g], mx);
          continue;
        }
        if constexpr (AB == 1) {
          if (mx == 12345.0f) cnt_l[0] = 1;
          continue;
        }
        if (__builtin_amdgcn_ballot_w64(mx >= q.y) == 0ull) continue;
        const float cq = qz[qi].x;
        uint32_t base = ((uint32_t)qi << 23) | (uint32_t)(rt - r0 + 4 * h);
        asm volatile("" : "+v"(base));
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const bool p = acc[g][e] >= q.y;
          if (__builtin_amdgcn_ballot_w64(p) == 0ull) continue;
          if (p) {
            const float sc = acc[g][e] + cq;
            const uint32_t word = base + (uint32_t)(8 * (e >> 2) + (e & 3));
            const int at = stage ? atomicAdd(&eb_n, 1) : EB;
            if (at < EB) eb[at] = make_uint2(__float_as_uint(sc), word);
            else put(qi, sc, r0 + (int)(word & 0x7FFFFFu));
          }
        }
      }
    }
    if constexpr (SAMPLE) {
#pragma unroll
      for (int g = 0; g < PQG; ++g) {
        const int qi = 32 * g + r;
        if (qi < qcnt) a.samp[(size_t)__float_as_int(qz[qi].y) * PSV + 2 * w + h] = smx[g] + qz[qi].x;
      }
      __syncthreads();
      continue;
    }
    __syncthreads();
    cand_flush<64 * PNW>(a, eb, min(eb_n, EB), qcnt, r0, cnt_l, base_l, [&](int i) { return __float_as_int(qz[i].y); });
  }
}

// ---- refine: the reference's ADC sum of the merged candidates, top k, certificate ----
// One wave per query; lane l holds merged candidate l (bound ms, position mk: >= 0 a row, -2 a floor,
// -1 none).  A lane's exact score: resQuery of the row's list, then distSq += table[m][code_m] in m
// order (IvfPqVectorIndex.cs:182-194; table entries L2SquaredUnsafe, ProductQuantizer.cs:107-117).
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
    const uint8_t *cp = a.cpack + ((size_t)(key >> 5) * 64 + (key & 31)) * a.mb;
    float dist = 0.0f;
    for (int m = 0; m < a.M; ++m) {
      const int c = cp[(size_t)(m & 1) * 32 * a.mb + (m >> 1)];
      float rq[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) rq[u] = qv[8 * m + u] - cv[8 * m + u];
      dist = dist + em_l2sq_unsafe(Lin{rq}, Off{a.codebooks + ((size_t)m * a.ksub + c) * 8}, 8);
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

template <int D>
void launch_pq_scan_d(const StreamArgs &a, const _Float16 *cb16, int max_items, bool sample, hipStream_t st) {
  const int grid = std::max(1, std::min(max_items, device_cus()));
  if (sample) hipLaunchKernelGGL((pq_scan_kernel<D, true>), dim3(grid), dim3(64 * PNW), 0, st, a, cb16);
  else if (a.ablate & 64) hipLaunchKernelGGL((pq_scan_kernel<D, false, 1>), dim3(grid), dim3(64 * PNW), 0, st, a, cb16);
  else if (a.ablate & 128) hipLaunchKernelGGL((pq_scan_kernel<D, false, 2>), dim3(grid), dim3(64 * PNW), 0, st, a, cb16);
  else hipLaunchKernelGGL((pq_scan_kernel<D, false>), dim3(grid), dim3(64 * PNW), 0, st, a, cb16);
}

}  // namespace

bool pq32_supported(int dim, int M, int ksub, int k) {
  return dim == 768 && dim == 8 * M && ksub >= 1 && ksub <= 256 && k >= 1 && k + 4 <= STREAM_KO;
}
int pq32_qmax() { return PQMAX; }
int pq32_sample_values() { return PSV; }
int pq32_code_bytes(int dim) { return (dim / 16 + 15) / 16 * 16; }

void launch_pq32_pack(const uint8_t *codes_rm, const int64_t *src, int64_t tot, int M, const float *cb, int ksub,
                      uint8_t *cpack, float *nrm, hipStream_t st) {
  if (tot <= 0) return;
  hipLaunchKernelGGL(pq_pack_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, codes_rm, src, tot, M,
                     pq32_code_bytes(8 * M), cb, ksub, cpack, nrm);
}
void launch_pq32_cb16(const float *cb, int M, int ksub, float sc, _Float16 *cb16, hipStream_t st) {
  const int64_t n = (int64_t)M * 256 * 8;
  hipLaunchKernelGGL(pq_cb16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cb, M, ksub, sc, cb16);
}
void launch_pq32_meta(const float *nrm, const uint8_t *live, int64_t tot, float *meta, hipStream_t st) {
  if (tot <= 0) return;
  hipLaunchKernelGGL(pq_meta_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, nrm, live, tot, meta);
}
void launch_pq32_prep(const StreamArgs &a, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  hipLaunchKernelGGL(pq_prep_kernel<768>, dim3((unsigned)((int64_t)max_items * PQMAX / 4)), dim3(256), 0, st, a);
}
void launch_pq32_scan(const StreamArgs &a, const _Float16 *cb16, int max_items, bool sample, hipStream_t st) {
  if (max_items <= 0) return;
  launch_pq_scan_d<768>(a, cb16, max_items, sample, st);
}
void launch_pq32_refine(const PqRefineArgs &a, int64_t nq, hipStream_t st) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(pq_refine_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, st, a);
}

}  // namespace pyr
