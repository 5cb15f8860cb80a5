// kernels.hip -- gfx950 (CDNA4) kernels of the Pyrope ANN scan hot path.
//
// Parity contract: every score is computed with the SAME fp32 operation order
// as the reference C# SIMD engine (src/Pyrope.GarnetServer/Vector/VectorMath.cs),
// restated for x64 AVX2 RyuJIT: 8 fp32 lanes, mul and add rounded separately
// (no contraction: this file is compiled with -ffp-contract=off and the pragma
// below), horizontal sum ((v0+v1)+(v2+v3))+((v4+v5)+(v6+v7)).  Scores are
// therefore bit-identical to the CPU oracle (oracle/oracle.c), not just close.
//
// Row storage is "blocked": groups of 8 rows stored dim-major, element
// (row r, dim d) at ((r/8)*D + d)*8 + r%8.  One group of D=128 rows is 4 KiB
// contiguous, read by one wave instruction per 1 KiB.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "kernels.h"

namespace pyr {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));


__device__ __forceinline__ bool better(float s1, uint32_t k1, float s2, uint32_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}
__device__ __forceinline__ bool better64(float s1, int64_t k1, float s2, int64_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

__device__ __forceinline__ size_t blk_off(int64_t r, int d, int D) {
  return ((size_t)(r >> 3) * (size_t)D + (size_t)d) * 8 + (size_t)(r & 7);
}

#include "vmath.h"

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// insertion into a sorted (desc) top-k list: same semantics as oracle topk_push
__device__ __forceinline__ void list_insert(float *ls, uint32_t *lk, int &cnt, int k, float s, uint32_t key) {
  int n = cnt;
  if (n == k) n = k - 1;
  int j = n;
  while (j > 0 && better(s, key, ls[j - 1], lk[j - 1])) {
    ls[j] = ls[j - 1];
    lk[j] = lk[j - 1];
    j--;
  }
  ls[j] = s;
  lk[j] = key;
  cnt = n + 1;
}

// ---------------------------------------------------------------------------
// Fast scan: D in {32,64,96,128}, k <= 64.
// Workgroup = 256 threads = 32 "slots" x 8 lanes.  Slot s owns queries
// 4s..4s+3 of the item (held in registers, dims of two Vector blocks packed in
// one VGPR pair and broadcast with op_sel); lane l of a slot owns Vector<float>
// lane l, i.e. dims l, l+8, l+16, ...  Rows stream through LDS in stages of
// GPS 8-row groups (double buffered, one barrier per stage).  Per group each
// slot computes 4 x 8 pairs with packed fp32 math (v_pk_add/mul_f32: sub, mul,
// add per element, phase-ordered so no dependent pair is adjacent), then the 8
// lanes of a slot combine their partial sums with the reference's horizontal
// tree by a DPP transpose-reduce (quad_perm xor1, quad_perm xor2,
// row_half_mirror), leaving each lane with the 4 scores of one row.  Scores go
// to an LDS matrix; one owner thread per query filters them against its k-th
// best (branch-free) and keeps that query's sorted top-k in LDS.
// ---------------------------------------------------------------------------
// IVF = the launch has a qlist (list-major IVF items); a separate instantiation so the IVF
// list scan and the FLAT / k-means scans are distinct kernel symbols in rocprof.
template <int GPS>
constexpr int score_stride() {  // floats per query row of the score matrix: conflict-free ds_write_b32
  return GPS * 8 + 4;
}

// QS = queries per slot: 2 -> 512 threads (register tile small enough for 5-6 waves per
// SIMD); 4 -> 256 threads (~140 VGPRs, 3 waves per SIMD: VALU issue ~47%, profiles/).
template <int D, int V, int MET, int GPS, bool IVF, int QS, int W>
__global__ __launch_bounds__(8 * QCHUNK / QS, W) void scan_fast(ScanArgs a) {
  constexpr int NT = 8 * QCHUNK / QS;   // threads
  constexpr int QPW = 8 * QS;           // queries per wave
  constexpr int T = D / 8;              // Vector<float> blocks per row
  constexpr int GF = D * 8;             // floats per 8-row group
  constexpr int RS = score_stride<GPS>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if ((int)blockIdx.x >= *a.n_items) return;
  const ScanItem it = a.items[blockIdx.x];
  const int k = a.k;
  float *tile = smem;                            // [2][GPS*GF]
  float *sc = smem + 2 * GPS * GF;               // [2][QCHUNK][RS]  (query-major scores)
  float *tks = sc + 2 * QCHUNK * RS;             // [QCHUNK][k]
  uint32_t *tkk = reinterpret_cast<uint32_t *>(tks + QCHUNK * k);

  const int tid = threadIdx.x;
  const int l = tid & 7, s = tid >> 3;
  const int c1 = (l ^ (l >> 2)) & 1, c2 = ((l >> 1) ^ (l >> 2)) & 1, c3 = (l >> 2) & 1;
  const int myj = c1 | (c2 << 1) | (c3 << 2);
  const bool wave_active = (tid >> 6) * QPW < it.qcnt;

  // queries arrive lane-major (transpose_queries): lane l's dims l, l+8, ... are
  // contiguous and load as float4; kept as plain scalars (packed FP32 has no extra
  // rate on gfx950 and its op_sel broadcast would double the register footprint).
  float q[QS][T];
  float qn[QS];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    const int i = s * QS + u;
    qn[u] = 0.0f;
    if (i < it.qcnt) {
      const int qi = IVF ? a.qlist[it.qbeg + i] / a.nparts : it.qbeg + i;
      const float4 *qp = reinterpret_cast<const float4 *>(a.queries_t + (size_t)qi * D + l * T);
#pragma unroll
      for (int p = 0; p < T / 4; ++p) {
        const float4 v = qp[p];
        q[u][4 * p] = v.x;
        q[u][4 * p + 1] = v.y;
        q[u][4 * p + 2] = v.z;
        q[u][4 * p + 3] = v.w;
      }
      if (MET == COS) qn[u] = a.qnorm[qi];
    } else {
#pragma unroll
      for (int t = 0; t < T; ++t) q[u][t] = 0.0f;
    }
  }

  const bool owner = tid < it.qcnt;
  int oslot = 0, qown = 0;
  uint32_t lim = 0xFFFFFFFFu;
  float gs = -INFINITY;  // shared per-query bound (ScanArgs::gthr): rows strictly below it are skipped
  uint32_t published = 0;
  if (owner) {
    oslot = IVF ? a.qlist[it.qbeg + tid] + it.part : (it.qbeg + tid) * a.nparts + it.part;
    qown = IVF ? a.qlist[it.qbeg + tid] / a.nparts : it.qbeg + tid;
    if (a.limits) lim = a.limits[oslot];
    if (a.gthr) gs = key_score(__hip_atomic_load(a.gthr + qown, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  int cnt = 0;
  float thr_s = -INFINITY;  // (-inf, NONE) lets every real candidate pass until the list is full
  uint32_t thr_k = KEY_NONE;
  float *ls = tks + tid * k;
  uint32_t *lk = tkk + tid * k;

  const int g0 = it.row_begin >> 3;
  const int ng = ((it.row_end + 7) >> 3) - g0;
  const int nst = (ng + GPS - 1) / GPS;
  // Register staging of the next stage: the loads are issued at the top of stage st
  // (pinned there by sched_barrier so the scheduler cannot sink them behind the
  // compute) and written to the other LDS buffer after the compute, so their HBM
  // latency hides under a whole stage of VALU work.
  constexpr int NV = GPS * D * 2;  // float4 per stage
  constexpr int LOADS = (NV + NT - 1) / NT;
  const float4 *src = reinterpret_cast<const float4 *>(a.rows);
  float4 pf[LOADS];
#define PYR_LOAD_STAGE(STG)                                                                     \
  _Pragma("unroll") for (int i = 0; i < LOADS; ++i) {                                          \
    const int v = min(tid + NT * i, NV - 1);                                                    \
    const int gg = min((STG) * GPS + v / (2 * D), ng - 1); /* clamp: rows past the end unused */ \
    pf[i] = src[(size_t)(g0 + gg) * (2 * D) + v % (2 * D)];                                     \
  }
#define PYR_STORE_STAGE(BUF)                                                                    \
  _Pragma("unroll") for (int i = 0; i < LOADS; ++i) {                                          \
    const int v = tid + NT * i;                                                                 \
    if (v < NV) reinterpret_cast<float4 *>(tile + (BUF) * GPS * GF)[v] = pf[i];                 \
  }
  float xn_next[GPS], xn_cur[GPS];  // cosine row norms, prefetched one stage ahead
#pragma unroll
  for (int g = 0; g < GPS; ++g) xn_next[g] = xn_cur[g] = 0.0f;
  if (nst > 0) {
    if (MET == COS) {
#pragma unroll
      for (int g = 0; g < GPS; ++g) xn_next[g] = a.rnorm[(size_t)(g0 + min(g, ng - 1)) * 8 + myj];
    }
    PYR_LOAD_STAGE(0)
    PYR_STORE_STAGE(0)
  }
  __syncthreads();

  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (MET == COS) {
#pragma unroll
      for (int g = 0; g < GPS; ++g) {
        xn_cur[g] = xn_next[g];  // retired by the previous barrier
        xn_next[g] = a.rnorm[(size_t)(g0 + min((st + 1) * GPS + g, ng - 1)) * 8 + myj];
      }
    }
    {
      const int nxt = more ? st + 1 : st;
      PYR_LOAD_STAGE(nxt)
    }
    __builtin_amdgcn_sched_barrier(0);

    if (wave_active) {
#pragma unroll
      for (int g = 0; g < GPS; ++g) {
        if (st * GPS + g >= ng) break;
        const float *tp = tile + cur * GPS * GF + g * GF + l * 8;
        float fin[QS][8];
        if constexpr (V == 1) {
          // QS queries x 8 rows per slot, one accumulator per (query, row) for lane l of
          // the single Vector accumulator (VectorMath.cs:52-58).  LDS reads are
          // software-pipelined one t-step ahead.
          float acc[QS][8];
#pragma unroll
          for (int u = 0; u < QS; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[u][j] = 0.0f;
          float4 xa = *reinterpret_cast<const float4 *>(tp);
          float4 xb = *reinterpret_cast<const float4 *>(tp + 4);
#pragma unroll
          for (int t = 0; t < T; ++t) {
            float4 na = xa, nb = xb;
            if (t + 1 < T) {
              na = *reinterpret_cast<const float4 *>(tp + (t + 1) * 64);
              nb = *reinterpret_cast<const float4 *>(tp + (t + 1) * 64 + 4);
            }
            const float xs[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
            for (int u = 0; u < QS; ++u) {
              float d[8];
              if constexpr (MET == L2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) d[j] = q[u][t] - xs[j];
#pragma unroll
                for (int j = 0; j < 8; ++j) d[j] = d[j] * d[j];
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) d[j] = q[u][t] * xs[j];
              }
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[u][j] = acc[u][j] + d[j];
            }
            xa = na;
            xb = nb;
          }
#pragma unroll
          for (int u = 0; u < QS; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) fin[u][j] = acc[u][j];
        } else {
          // four Vector accumulators: acc[v] sums dims 32s + 8v + l (VectorMath.cs:197-221),
          // rows in two halves of 4 to bound the register tile
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float acc[4][QS][4];
#pragma unroll
            for (int v = 0; v < 4; ++v)
#pragma unroll
              for (int u = 0; u < QS; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[v][u][j] = 0.0f;
            float4 xa = *reinterpret_cast<const float4 *>(tp + 4 * h);
#pragma unroll
            for (int t = 0; t < T; ++t) {
              const int v = t & 3;
              float4 na = xa;
              if (t + 1 < T) na = *reinterpret_cast<const float4 *>(tp + (t + 1) * 64 + 4 * h);
              const float xs[4] = {xa.x, xa.y, xa.z, xa.w};
#pragma unroll
              for (int u = 0; u < QS; ++u) {
                float d[4];
                if constexpr (MET == L2) {
#pragma unroll
                  for (int j = 0; j < 4; ++j) d[j] = q[u][t] - xs[j];
#pragma unroll
                  for (int j = 0; j < 4; ++j) d[j] = d[j] * d[j];
                } else {
#pragma unroll
                  for (int j = 0; j < 4; ++j) d[j] = q[u][t] * xs[j];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[v][u][j] = acc[v][u][j] + d[j];
              }
              xa = na;
            }
#pragma unroll
            for (int u = 0; u < QS; ++u)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                fin[u][4 * h + j] = ((acc[0][u][j] + acc[1][u][j]) + acc[2][u][j]) + acc[3][u][j];  // :224
          }
        }
        // transpose-reduce = Vector.Dot(acc, One) tree, one row per lane at the end
        float r1[QS][4], r2[QS][2], r3[QS];
#pragma unroll
        for (int u = 0; u < QS; ++u)
#pragma unroll
          for (int jp = 0; jp < 4; ++jp) {
            const float x0 = fin[u][2 * jp], x1 = fin[u][2 * jp + 1];
            const float keep = c1 ? x1 : x0, send = c1 ? x0 : x1;
            r1[u][jp] = keep + dpp<0xB1>(send);
          }
#pragma unroll
        for (int u = 0; u < QS; ++u)
#pragma unroll
          for (int jq = 0; jq < 2; ++jq) {
            const float x0 = r1[u][2 * jq], x1 = r1[u][2 * jq + 1];
            const float keep = c2 ? x1 : x0, send = c2 ? x0 : x1;
            r2[u][jq] = keep + dpp<0x4E>(send);
          }
#pragma unroll
        for (int u = 0; u < QS; ++u) {
          const float x0 = r2[u][0], x1 = r2[u][1];
          const float keep = c3 ? x1 : x0, send = c3 ? x0 : x1;
          r3[u] = keep + dpp<0x141>(send);
        }
        const float xn = xn_cur[g];
#pragma unroll
        for (int u = 0; u < QS; ++u) {
          const float sum = 0.0f + r3[u];  // `sum += Vector.Dot(...)` with sum = 0f
          float sv;
          if (MET == L2) sv = -sum;
          else if (MET == IP) sv = sum;
          else sv = (qn[u] < 1e-6f || xn < 1e-6f) ? 0.0f : sum / (qn[u] * xn);
          sc[(cur * QCHUNK + s * QS + u) * RS + g * 8 + myj] = sv;
        }
      }
    }
    PYR_STORE_STAGE(cur ^ 1)  // after the last stage this fills an unused buffer
    __syncthreads();

    if (owner) {
#pragma unroll
      for (int g = 0; g < GPS; ++g) {
        if (st * GPS + g >= ng) break;
        const float *scp = sc + (cur * QCHUNK + tid) * RS + g * 8;
        const int rb = (g0 + st * GPS + g) * 8;
        float v[8];
        unsigned pass = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = scp[j];
          const int r = rb + j;
          if (r < it.row_end && v[j] >= gs && better(v[j], a.key_base | (uint32_t)r, thr_s, thr_k))
            pass |= 1u << j;
        }
        if (pass) {  // rare once the list is full
          for (int j = 0; j < 8; ++j) {
            if (!((pass >> j) & 1)) continue;
            const int r = rb + j;
            const uint32_t key = a.key_base | (uint32_t)r;
            const float vj = scp[j];
            if (!better(vj, key, thr_s, thr_k) || (uint32_t)r >= lim || !a.live[r]) continue;
            list_insert(ls, lk, cnt, k, vj, key);
            if (cnt == k) {
              thr_s = ls[k - 1];
              thr_k = lk[k - 1];
            }
          }
        }
      }
      if (a.gthr && (st & 7) == 7) {  // every 8 stages: publish this list's k-th best, refresh the bound
        if (cnt == k && score_key(thr_s) > published) {
          published = score_key(thr_s);
          atomicMax(a.gthr + qown, published);
        }
        gs = fmaxf(gs, key_score(__hip_atomic_load(a.gthr + qown, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
      }
    }
  }
  if (owner) {
    if (a.gthr && cnt == k && score_key(thr_s) > published) atomicMax(a.gthr + qown, score_key(thr_s));
    float *ps = a.part_s + (size_t)oslot * k;
    uint32_t *pk = a.part_k + (size_t)oslot * k;
    for (int j = 0; j < k; ++j) {
      ps[j] = j < cnt ? ls[j] : -INFINITY;
      pk[j] = j < cnt ? lk[j] : KEY_NONE;
    }
  }
#undef PYR_LOAD_STAGE
#undef PYR_STORE_STAGE
}

// ---------------------------------------------------------------------------
// Generic scan: any D, k <= KMAX.  One thread per query, exact restatement.
// ---------------------------------------------------------------------------
template <int V, int MET>
__global__ __launch_bounds__(64) void scan_generic(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if ((int)blockIdx.x >= *a.n_items) return;
  const ScanItem it = a.items[blockIdx.x];
  const int tid = threadIdx.x, k = a.k, D = a.dim;
  if (tid >= it.qcnt) return;
  float *ls = smem + tid * k;
  uint32_t *lk = reinterpret_cast<uint32_t *>(smem + 64 * k) + tid * k;
  const int qi = a.qlist ? a.qlist[it.qbeg + tid] / a.nparts : it.qbeg + tid;
  const int slot = a.qlist ? a.qlist[it.qbeg + tid] + it.part : qi * a.nparts + it.part;
  const uint32_t lim = a.limits ? a.limits[slot] : 0xFFFFFFFFu;
  const Lin qa{a.queries + (size_t)qi * D};
  const float qn = MET == COS ? a.qnorm[qi] : 0.0f;
  int cnt = 0;
  for (int r = it.row_begin; r < it.row_end; ++r) {
    if ((uint32_t)r >= lim) break;
    if (!a.live[r]) continue;
    const Blk xa{a.rows, D, r};
    const float xn = MET == COS ? a.rnorm[r] : 0.0f;
    const float v = em_score<V, MET>(qa, xa, D, qn, xn);
    const uint32_t key = a.key_base | (uint32_t)r;
    if (cnt == k && !better(v, key, ls[k - 1], lk[k - 1])) continue;
    list_insert(ls, lk, cnt, k, v, key);
  }
  float *ps = a.part_s + (size_t)slot * k;
  uint32_t *pk = a.part_k + (size_t)slot * k;
  for (int j = 0; j < k; ++j) {
    ps[j] = j < cnt ? ls[j] : -INFINITY;
    pk[j] = j < cnt ? lk[j] : KEY_NONE;
  }
}

__global__ void flat_items_kernel(ScanItem *items, int32_t *n_items, int nchunks, int nqc, int chunk_rows,
                                  int64_t nrows, int64_t nq, int part_off, int qchunk) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id == 0) *n_items = nchunks * nqc;
  if (id >= nchunks * nqc) return;
  const int c = id / nqc, qc = id % nqc;
  ScanItem it;
  it.row_begin = c * chunk_rows;
  const int64_t e = (int64_t)(c + 1) * chunk_rows;
  it.row_end = (int)(e < nrows ? e : nrows);
  it.qbeg = qc * qchunk;
  const int64_t qe = (int64_t)(qc + 1) * qchunk;
  it.qcnt = (int)((qe < nq ? qe : nq) - it.qbeg);
  it.part = part_off + c;
  it.list = 0;
  items[id] = it;
}

// queries row-major -> lane-major: qt[q][l][t] = q[q][8t + l] (fast-scan register layout)
__global__ void transpose_queries_kernel(const float *q, int64_t nq, int D, float *qt) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int r = (int)(e % D);
    const int T = D / 8, l = r / T, t = r % T;
    qt[e] = q[(size_t)i * D + 8 * t + l];
  }
}

__global__ void norms_kernel(const float *x, int64_t n, int dim, int blocked, float *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = blocked ? em_norm(Blk{x, dim, i}, dim) : em_norm(Lin{x + (size_t)i * dim}, dim);
}

// ---------------------------------------------------------------------------
// Merge of sorted partial lists: one wave per query, k rounds of wave argmax.
// ---------------------------------------------------------------------------
// MERGE_U: parts per lane, a compile-time bound (1..16) chosen from nparts at launch, so that
// the per-round scan over a lane's heads touches only the slots that can exist
template <int MERGE_U>
__global__ __launch_bounds__(256) void merge_keys_kernel(const float *ps, const uint32_t *pk, int64_t nq, int nparts,
                                                         int k, const int64_t *row_labels, const int64_t *buf_labels,
                                                         float *out_s, int64_t *out_l, int32_t *out_keys,
                                                         int32_t *out_cnt, MergeIvf iv) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  int h[MERGE_U];
  float cs[MERGE_U];
  uint32_t ck[MERGE_U];
  const size_t base = (size_t)q * nparts * k;
  const int ivf_parts = iv.probes ? iv.nprobe * iv.ch.cmax : 0;
#pragma unroll
  for (int u = 0; u < MERGE_U; ++u) {
    const int p = lane + 64 * u;
    h[u] = 0;
    bool valid = p < nparts;
    if (valid && p < ivf_parts) {  // chunk slot p = probe * cmax + c exists iff c < chunks of that list
      const int lst = iv.probes[q * iv.nprobe + p / iv.ch.cmax];
      valid = p % iv.ch.cmax < ivf_list_chunks(iv.le[lst] - iv.lb[lst], iv.ch);
    }
    if (valid) {
      cs[u] = ps[base + (size_t)p * k];
      ck[u] = pk[base + (size_t)p * k];
    } else {
      cs[u] = -INFINITY;
      ck[u] = KEY_NONE;
    }
  }
  int produced = 0;
  for (int r = 0; r < k; ++r) {
    float bs = -INFINITY;
    uint32_t bk = KEY_NONE;
#pragma unroll
    for (int u = 0; u < MERGE_U; ++u)
      if (ck[u] != KEY_NONE && (bk == KEY_NONE || better(cs[u], ck[u], bs, bk))) {
        bs = cs[u];
        bk = ck[u];
      }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float os = __shfl_xor(bs, off);
      const uint32_t ok = __shfl_xor(bk, off);
      if (ok != KEY_NONE && (bk == KEY_NONE || better(os, ok, bs, bk))) {
        bs = os;
        bk = ok;
      }
    }
    if (bk == KEY_NONE) break;
    if (lane == 0) {
      const size_t o = (size_t)q * k + r;
      if (out_s) out_s[o] = bs;
      if (out_keys) out_keys[o] = (int32_t)bk;
      if (out_l) {
        int64_t lab;
        if (bk == KEY_FLOOR) lab = -1;  // a region's floor placeholder (stream scans): no row
        else if (bk & KEY_BUF) lab = buf_labels ? buf_labels[bk & ~KEY_BUF] : (int64_t)(bk & ~KEY_BUF);
        else lab = row_labels ? row_labels[bk] : (int64_t)bk;
        out_l[o] = lab;
      }
    }
#pragma unroll
    for (int u = 0; u < MERGE_U; ++u)
      if (ck[u] == bk) {  // keys are unique: exactly one lane/u advances
        const int p = lane + 64 * u;
        h[u]++;
        if (h[u] < k) {  // a valid slot's list is KEY_NONE-terminated, so reads stay in written slots
          cs[u] = ps[base + (size_t)p * k + h[u]];
          ck[u] = pk[base + (size_t)p * k + h[u]];
        } else {
          cs[u] = -INFINITY;
          ck[u] = KEY_NONE;
        }
      }
    produced++;
  }
  if (lane == 0) {
    for (int r = produced; r < k; ++r) {
      const size_t o = (size_t)q * k + r;
      if (out_s) out_s[o] = -INFINITY;
      if (out_keys) out_keys[o] = -1;
      if (out_l) out_l[o] = -1;
    }
    if (out_cnt) out_cnt[q] = produced;
  }
}

constexpr int MERGE_LU = MAX_PARTS / 64;  // parts per lane (merge_labels_kernel)

// element (q, part, j) of the partial lists at q * sq + part * sp + j: query-major [nq][nparts][k]
// (sq = nparts k, sp = k) or part-major [nparts][nq][k] as an all_gather leaves it (sq = k, sp = nq k)
__global__ __launch_bounds__(256) void merge_labels_kernel(const float *ps, const int64_t *pl, int64_t nq, int nparts,
                                                           int k, int64_t sq, int64_t sp, float *out_s, int64_t *out_l) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  int h[MERGE_LU];
  float cs[MERGE_LU];
  int64_t cl[MERGE_LU];
  const size_t base = (size_t)q * sq;
#pragma unroll
  for (int u = 0; u < MERGE_LU; ++u) {
    const int p = lane + 64 * u;
    h[u] = 0;
    cs[u] = p < nparts ? ps[base + (size_t)p * sp] : -INFINITY;
    cl[u] = p < nparts ? pl[base + (size_t)p * sp] : -1;
  }
  int produced = 0;
  for (int r = 0; r < k; ++r) {
    float bs = -INFINITY;
    int64_t bl = -1;
#pragma unroll
    for (int u = 0; u < MERGE_LU; ++u)
      if (cl[u] >= 0 && (bl < 0 || better64(cs[u], cl[u], bs, bl))) {
        bs = cs[u];
        bl = cl[u];
      }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float os = __shfl_xor(bs, off);
      const int64_t ol = __shfl_xor(bl, off);
      if (ol >= 0 && (bl < 0 || better64(os, ol, bs, bl))) {
        bs = os;
        bl = ol;
      }
    }
    if (bl < 0) break;
    if (lane == 0) {
      out_s[(size_t)q * k + r] = bs;
      out_l[(size_t)q * k + r] = bl;
    }
#pragma unroll
    for (int u = 0; u < MERGE_LU; ++u)
      if (cl[u] == bl && cs[u] == bs) {
        const int p = lane + 64 * u;
        h[u]++;
        cs[u] = h[u] < k ? ps[base + (size_t)p * sp + h[u]] : -INFINITY;
        cl[u] = h[u] < k ? pl[base + (size_t)p * sp + h[u]] : -1;
      }
    produced++;
  }
  if (lane == 0)
    for (int r = produced; r < k; ++r) {
      out_s[(size_t)q * k + r] = -INFINITY;
      out_l[(size_t)q * k + r] = -1;
    }
}

// Two sorted result sets of one query merged into its top k: a (the lists') before b (the buffer's) on equal
// score keys -- the order launch_merge_keys gives list keys (< KEY_BUF) against KEY_BUF | slot -- each set
// already in its own (score desc, storage slot asc) order; ca / cb their real entries.  One thread per query.
__global__ void merge_two_kernel(const float *as, const int64_t *al, const int32_t *ca, const float *bs,
                                 const int64_t *bl, const int32_t *cb, int64_t nq, int k, float *out_s,
                                 int64_t *out_l, int32_t *out_c) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const float *a = as + q * k, *b = bs + q * k;
  const int64_t *la = al + q * k, *lb = bl + q * k;
  const int na = min(ca[q], k), nb = min(cb[q], k);
  int i = 0, j = 0, o = 0;
  // (the outputs are neither input: written in place, any k)
  for (; o < k && (i < na || j < nb); ++o) {
    const bool ta = i < na && (j >= nb || score_key(a[i]) >= score_key(b[j]));
    out_s[q * k + o] = ta ? a[i] : b[j];
    out_l[q * k + o] = ta ? la[i] : lb[j];
    if (ta) ++i;
    else ++j;
  }
  const int n = o;
  for (; o < k; ++o) {
    out_s[q * k + o] = -INFINITY;
    out_l[q * k + o] = -1;
  }
  if (out_c) out_c[q] = n;
}

// ---------------------------------------------------------------------------
// IVF list-major work lists
// ---------------------------------------------------------------------------
// probes [nq][nprobe]; only probe ranks [pb, pe) of every query take part
// skip: the lists a rank does not hold (IvfChunking::skip_empty; list_taken) take no (query, probe) entry
__device__ __forceinline__ bool list_taken(const int32_t *lb, const int32_t *le, int l) {
  return !lb || le[l] > lb[l];
}
__global__ void ivf_count_kernel(const int32_t *probes, int64_t nq, int nprobe, int pb, int pe, int32_t *cnt,
                                 const int32_t *lb, const int32_t *le) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int np = pe - pb;
  if (i >= nq * np) return;
  const int l = probes[(i / np) * nprobe + pb + i % np];
  if (list_taken(lb, le, l)) atomicAdd(&cnt[l], 1);
}

// The same two passes with block-local LDS histograms (nlist <= IVF_LDS_BINS): a block takes
// IVF_EPB consecutive (query, probe) entries, counts them per list in LDS and adds each non-empty
// bin to the global count once; the fill pass reserves one range per (block, list) with one global
// atomic and places entries by their LDS rank.  320k entries into 1,024 lists: ~80k global atomics
// instead of 320k on 1,024 addresses.  (Entry order inside a list differs from the one-atomic-per-
// entry pass; it is arbitrary in both, and results do not depend on it.)
// EPT entries per thread: 4 (EPT 16 left 79 blocks at I1), 16 from 2M entries on (a list-sharded rank's N x
// batch: 2.56M entries at the N = 8 shape, most of them dropped, where 4 per thread spent the launch clearing
// and scanning 2,500 blocks' histograms)
constexpr int IVF_LDS_BINS = 16384;
inline int ivf_ept(int64_t n) { return n >= (int64_t)2 << 20 ? 16 : 4; }

template <int IVF_EPT>
__global__ __launch_bounds__(256) void ivf_count_lds_kernel(const int32_t *probes, int64_t nq, int nprobe, int pb,
                                                            int pe, int nlist, int32_t *cnt, const int32_t *lb,
                                                            const int32_t *le) {
  extern __shared__ int hist[];
  constexpr int IVF_EPB = 256 * IVF_EPT;
  const int np = pe - pb;
  const int64_t n = nq * np, e0 = (int64_t)blockIdx.x * IVF_EPB;
  for (int i = threadIdx.x; i < nlist; i += 256) hist[i] = 0;
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < IVF_EPT; ++j) {
    const int64_t i = e0 + j * 256 + threadIdx.x;
    if (i < n) {
      const int l = probes[(i / np) * nprobe + pb + i % np];
      if (list_taken(lb, le, l)) atomicAdd(&hist[l], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nlist; i += 256)
    if (hist[i]) atomicAdd(&cnt[i], hist[i]);
}

template <int IVF_EPT>
__global__ __launch_bounds__(256) void ivf_fill_lds_kernel(const int32_t *probes, int64_t nq, int nprobe, int pb,
                                                           int pe, int nparts, int cmax, int nlist,
                                                           const int32_t *qoff, int32_t *fill, int32_t *qlist,
                                                           int32_t *qpos, const int32_t *lb, const int32_t *le) {
  extern __shared__ int hist[];
  constexpr int IVF_EPB = 256 * IVF_EPT;
  const int np = pe - pb;
  const int64_t n = nq * np, e0 = (int64_t)blockIdx.x * IVF_EPB;
  for (int i = threadIdx.x; i < nlist; i += 256) hist[i] = 0;
  __syncthreads();
  int lst[IVF_EPT], rank[IVF_EPT];
#pragma unroll
  for (int j = 0; j < IVF_EPT; ++j) {
    const int64_t i = e0 + j * 256 + threadIdx.x;
    lst[j] = i < n ? probes[(i / np) * nprobe + pb + i % np] : -1;
    if (lst[j] >= 0 && !list_taken(lb, le, lst[j])) {
      lst[j] = -1;
      if (qpos) qpos[(i / np) * nprobe + pb + i % np] = -1;  // (a dropped entry has no position)
    }
    rank[j] = lst[j] >= 0 ? atomicAdd(&hist[lst[j]], 1) : 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nlist; i += 256)  // the block's range of each list
    if (hist[i]) hist[i] = qoff[i] + atomicAdd(&fill[i], hist[i]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IVF_EPT; ++j) {
    if (lst[j] < 0) continue;
    const int64_t i = e0 + j * 256 + threadIdx.x;
    const int64_t q = i / np;
    const int p = pb + (int)(i % np);
    qlist[hist[lst[j]] + rank[j]] = (int32_t)(q * nparts + p * cmax);  // chunk c adds c (ScanItem.part)
    if (qpos) qpos[q * nprobe + p] = hist[lst[j]] + rank[j];
  }
}

// chunks of list `lst` that launch phase `phase` scans (IvfChunking, kernels.h)
__device__ __forceinline__ int phase_chunks(const int32_t *lb, const int32_t *le, int lst, IvfChunking ch, int phase) {
  const int n = ivf_list_chunks(le[lst] - lb[lst], ch);
  if (ch.warm <= 0) return n;
  return phase == 0 ? 1 : n - 1;
}

// IvfChunking::xcd: the list at position i of the queue-major order (queue x = lists l with l % 8 == x,
// a + (x < b) of them for nlist = 8a + b), and whether i starts queue x
__device__ __forceinline__ int xcd_order_list(int i, int nlist, int *x, bool *first) {
  const int a = nlist >> 3, b = nlist & 7, head = b * (a + 1);
  int j;
  if (i < head) {
    *x = i / (a + 1);
    j = i - *x * (a + 1);
  } else {
    *x = b + (i - head) / a;
    j = (i - head) - (*x - b) * a;
  }
  *first = j == 0;
  return *x + 8 * j;
}

// the items of list `lst` (rows [lb0, lb0 + len)) in launch phase `phase` (c probing queries from qoff_l,
// items from o): for each of its row chunks, for each block of <= qchunk probing queries
__device__ __forceinline__ void ivf_list_items(int lst, int c, int qoff_l, int o, int lb0, int len, int qchunk,
                                               IvfChunking chk, int phase, int balance, ScanItem *items) {
  const int c0 = (chk.warm > 0 && phase == 1) ? 1 : 0;
  const int nch = ivf_list_chunks(len, chk);
  const int c1 = c0 + (chk.warm <= 0 ? nch : (phase == 0 ? 1 : nch - 1));
  // balance: the list's ceil(c / qchunk) groups get equal shares rounded up to 16 queries (whole
  // 16-query MFMA groups) instead of full groups plus a remainder
  const int ng = (c + qchunk - 1) / qchunk;
  const int sz = balance && ng > 0 ? ((c + ng - 1) / ng + 15) / 16 * 16 : qchunk;
  for (int ch = c0; ch < c1; ++ch) {
    int rb, re;
    ivf_chunk_rows(len, ch, chk, &rb, &re);
    for (int gi = 0; gi < ng; ++gi, ++o) {
      const int b = gi * sz;
      ScanItem it;
      it.row_begin = lb0 + rb;
      it.row_end = lb0 + re;
      it.qbeg = qoff_l + min(b, c);
      it.qcnt = max(0, min(sz, c - b));
      it.part = ch;
      it.list = lst;
      items[o] = it;
    }
  }
}

// single workgroup: qoff = exclusive scan of cnt, ioff = exclusive scan of ceil(cnt/qchunk) * chunks
// (over the lists in XCD queue order when chk.xcd; n_items[1 + x] = the first item of queue x), and each
// list's items (ivf_list_items; round 4 wrote them in a launch of their own)
__global__ __launch_bounds__(1024) void ivf_scan_kernel(const int32_t *cnt, int nlist, int qchunk, const int32_t *lb,
                                                        const int32_t *le, IvfChunking chk, int phase, int32_t *qoff,
                                                        int32_t *ioff, int32_t *n_items, int balance, ScanItem *items) {
  __shared__ int sq[1024], si[1024];
  const int tid = threadIdx.x;
  const int per = (nlist + 1023) / 1024;
  const int b = tid * per, e = min(nlist, b + per);
  auto at = [&](int i) {
    if (!chk.xcd) return i;
    int x;
    bool f;
    return xcd_order_list(i, nlist, &x, &f);
  };
  // (4 lists at a time with their loads issued together: at nlist = 8,192 a thread owns 8 lists, and one
  // dependent load chain per list made this single block a 50 us launch)
  int lq = 0, li = 0;
  for (int i0 = b; i0 < e; i0 += 4) {
    int c4[4], n4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int l = i0 + u < e ? at(i0 + u) : 0;
      c4[u] = i0 + u < e ? cnt[l] : 0;
      n4[u] = i0 + u < e ? phase_chunks(lb, le, l, chk, phase) : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      lq += c4[u];
      li += (c4[u] + qchunk - 1) / qchunk * n4[u];
    }
  }
  sq[tid] = lq;
  si[tid] = li;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int vq = tid >= off ? sq[tid - off] : 0;
    const int vi = tid >= off ? si[tid - off] : 0;
    __syncthreads();
    sq[tid] += vq;
    si[tid] += vi;
    __syncthreads();
  }
  int rq = sq[tid] - lq, ri = si[tid] - li;
  for (int i0 = b; i0 < e; i0 += 4) {
    int l4[4], c4[4], b4[4], n4[4], x4[4];
    bool f4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u;
      x4[u] = 0;
      f4[u] = false;
      l4[u] = i < e ? (chk.xcd ? xcd_order_list(i, nlist, &x4[u], &f4[u]) : i) : -1;
      const int l = max(l4[u], 0);
      c4[u] = l4[u] >= 0 ? cnt[l] : 0;
      b4[u] = l4[u] >= 0 ? lb[l] : 0;
      n4[u] = l4[u] >= 0 ? le[l] - b4[u] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (l4[u] < 0) continue;
      const int l = l4[u];
      if (chk.xcd && f4[u]) n_items[1 + x4[u]] = ri;
      qoff[l] = rq;
      ioff[l] = ri;
      ivf_list_items(l, c4[u], rq, ri, b4[u], n4[u], qchunk, chk, phase, balance, items);
      const int nch = ivf_list_chunks(n4[u], chk);
      rq += c4[u];
      ri += (c4[u] + qchunk - 1) / qchunk * (chk.warm <= 0 ? nch : (phase == 0 ? 1 : nch - 1));
    }
  }
  if (tid == 1023) {
    qoff[nlist] = sq[1023];
    ioff[nlist] = si[1023];
    *n_items = si[1023];
    if (chk.xcd)  // the end bound, and the bounds of queues with no list (nlist < 8)
      for (int x = min(nlist, 8); x <= 8; ++x) n_items[1 + x] = si[1023];
    else  // one queue holding every item (a queue-taking kernel steals it from the others' empty ones)
      for (int x = 0; x <= 8; ++x) n_items[1 + x] = x == 0 ? 0 : si[1023];
  }
}

__global__ void ivf_fill_kernel(const int32_t *probes, int64_t nq, int nprobe, int pb, int pe, int nparts, int cmax,
                                const int32_t *qoff, int32_t *fill, int32_t *qlist, int32_t *qpos, const int32_t *lb,
                                const int32_t *le) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int np = pe - pb;
  if (i >= nq * np) return;
  const int64_t q = i / np;
  const int p = pb + (int)(i % np);
  const int lst = probes[q * nprobe + p];
  if (!list_taken(lb, le, lst)) {
    if (qpos) qpos[q * nprobe + p] = -1;  // (a dropped entry has no position)
    return;
  }
  const int pos = atomicAdd(&fill[lst], 1);
  qlist[qoff[lst] + pos] = (int32_t)(q * nparts + p * cmax);  // chunk c adds c (ScanItem.part)
  if (qpos) qpos[q * nprobe + p] = qoff[lst] + pos;
}

// One wave per query: the probed lists in probe order, each taking min(its live rows, what is left); the list
// where the budget runs out is bounded at its (rem + 1)-th live row (rows before it hold exactly rem live
// ones), found 64 rows at a time (ballot + prefix popcount) -- a tombstone-free list directly at lb + rem.
// (Round 4 walked that list row by row in one thread: 2.5 ms at I1 with MaxScans 5,000.)
// prem != null (a list-sharded rank): the home rank already ran the budget down the probe order over every
// rank's lists (shard_budget_kernel); prem[q * rstride + p] is what was left when pair p's list was reached.
__global__ __launch_bounds__(256) void ivf_limits_kernel(const int32_t *probes, int64_t nq, int nprobe, int nparts,
                                                         int cmax, int64_t remaining, const int32_t *lb,
                                                         const int32_t *le, const int32_t *llive, const uint8_t *live,
                                                         uint32_t *limits, const int32_t *prem, int rstride) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  int64_t rem = remaining;
  for (int p = 0; p < nprobe; ++p) {
    if (prem) rem = prem[(size_t)q * rstride + p];
    const int lst = probes[q * nprobe + p];
    const int b = lb[lst], e = le[lst], n = llive[lst];
    uint32_t lim;
    if (rem <= 0) {
      lim = (uint32_t)b;
    } else if (rem >= n) {
      lim = (uint32_t)e;
      rem -= n;
    } else if (n == e - b) {
      lim = (uint32_t)(b + rem);
      rem = 0;
    } else {
      int64_t c = 0;  // live rows before r0
      lim = (uint32_t)e;
      for (int r0 = b; r0 < e; r0 += 64) {
        const int r = r0 + lane;
        const bool lv = r < e && live[r] != 0;
        const uint64_t m = __builtin_amdgcn_ballot_w64(lv);
        const int cnt = (int)__builtin_popcountll(m);
        if (c + cnt > rem) {  // the (rem - c)-th live row of this block (0-based) is the bound
          const int pre = (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
          const uint64_t hit = __builtin_amdgcn_ballot_w64(lv && pre == (int)(rem - c));
          lim = (uint32_t)(r0 + (int)__builtin_ctzll(hit));
          break;
        }
        c += cnt;
      }
      rem = 0;
    }
    for (int c = lane; c < cmax; c += 64) limits[(size_t)q * nparts + p * cmax + c] = lim;  // bound is absolute
  }
}

__global__ void pos_limits_kernel(const int32_t *qpos, const uint32_t *limits, int64_t n, uint32_t *plim) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t pos = qpos[i];
  if (pos >= 0) plim[pos] = limits[i];
}

// ---------------------------------------------------------------------------
// IVF-PQ: per (query, probed list) LUT in LDS + ADC scan over blocked codes.
// Codes: lists padded to 64-row blocks; block b holds [ceil(M/16)][64 rows][16 B].
// ---------------------------------------------------------------------------
__device__ __forceinline__ size_t pq_code_off(int64_t r, int chunk, int nch) {
  return (((size_t)(r >> 6) * nch + chunk) * 64 + (size_t)(r & 63)) * 16;
}

__global__ __launch_bounds__(256) void pq_scan_kernel(PqArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if ((int)blockIdx.x >= *a.n_items) return;
  const ScanItem it = a.items[blockIdx.x];
  const int D = a.dim, M = a.M, ksub = a.ksub, k = a.k, sub = D / M;
  const int nch = (M + 15) / 16;
  const int Dp = (D + 3) & ~3;
  float *res = smem;
  float *lut = res + Dp;
  float *tks = lut + M * ksub;
  uint32_t *tkk = reinterpret_cast<uint32_t *>(tks + k);
  float *qs = reinterpret_cast<float *>(tkk + k);
  uint32_t *qk = reinterpret_cast<uint32_t *>(qs + 256);
  int *misc = reinterpret_cast<int *>(qk + 256);
  const int tid = threadIdx.x;
  const int lst = it.list;
  const float *cent = a.cents + (size_t)lst * D;

  for (int i = 0; i < it.qcnt; ++i) {
    const int slot = a.qlist[it.qbeg + i] + it.part;
    const int qi = slot / a.nparts;
    const float *qp = a.queries + (size_t)qi * D;
    for (int d = tid; d < D; d += 256) res[d] = qp[d] - cent[d];  // IvfPqVectorIndex.cs:163
    if (tid == 0) {
      misc[0] = 0;
      misc[1] = 0;
    }
    __syncthreads();
    for (int e = tid; e < M * ksub; e += 256) {  // ProductQuantizer.cs:112-117
      const int m = e / ksub, j = e - m * ksub;
      lut[e] = em_l2sq_unsafe(Off{res + m * sub}, Off{a.codebooks + ((size_t)m * ksub + j) * sub}, sub);
    }
    __syncthreads();
    for (int base = it.row_begin; base < it.row_end; base += 256) {
      const int r = base + tid;
      bool valid = r < it.row_end && a.live[r];
      float score = 0.0f;
      if (valid) {
        float dist = 0.0f;  // IvfPqVectorIndex.cs:182-186, m order
        for (int c = 0; c < nch; ++c) {
          const uint4 w = *reinterpret_cast<const uint4 *>(a.codes + pq_code_off(r, c, nch));
          const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int b = 0; b < 16; ++b) {
            const int m = c * 16 + b;
            if (m < M) dist = dist + lut[m * ksub + ((ws[b >> 2] >> (8 * (b & 3))) & 0xFF)];
          }
        }
        score = -dist;  // :194
      }
      const int cnt = misc[1];
      const uint32_t key = (uint32_t)r;
      if (valid && (cnt < k || better(score, key, tks[k - 1], tkk[k - 1]))) {
        const int idx = atomicAdd(&misc[0], 1);
        qs[idx] = score;
        qk[idx] = key;
      }
      __syncthreads();
      if (tid == 0) {
        int c2 = misc[1];
        const int nqd = misc[0];
        for (int j = 0; j < nqd; ++j) {
          if (c2 == k && !better(qs[j], qk[j], tks[k - 1], tkk[k - 1])) continue;
          list_insert(tks, tkk, c2, k, qs[j], qk[j]);
        }
        misc[1] = c2;
        misc[0] = 0;
      }
      __syncthreads();
    }
    const int cnt = misc[1];
    for (int j = tid; j < k; j += 256) {
      a.part_s[(size_t)slot * k + j] = j < cnt ? tks[j] : -INFINITY;
      a.part_k[(size_t)slot * k + j] = j < cnt ? tkk[j] : KEY_NONE;
    }
    __syncthreads();
  }
}

// Top-k of a wave spread over lanes 0..k-1 (lane j = j-th best): candidates beating the wave's k-th
// (and the query's shared bound) are found with one ballot and inserted with a shuffle, so the common
// no-candidate case costs two compares.  (Rounds 1-3 also had pq_adc, one query per pass; pq_adc4
// superseded it.)

// wave-wide insertion of the candidates flagged in `cand` into the lane-distributed list
__device__ __forceinline__ void wave_list_insert(bool cand, float sc, uint32_t key, float &ls, uint32_t &lk, float &kth,
                                                 uint32_t &kthk, int k, int lane) {
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

// k > 64: the same list in R registers per lane (entry i = 64 r + lane, i < k <= 64 R); an insertion at pos
// shifts the entries past it up by one, across the registers (lane 63 of register r - 1 -> lane 0 of r)
template <int R>
__device__ __forceinline__ void wave_list_insert_r(bool cand, float sc, uint32_t key, float (&ls)[R],
                                                   uint32_t (&lk)[R], float &kth, uint32_t &kthk, int k, int lane) {
  if constexpr (R == 1) {
    wave_list_insert(cand, sc, key, ls[0], lk[0], kth, kthk, k, lane);
  } else {
    const int kr = (k - 1) >> 6, kl = (k - 1) & 63;
    uint64_t m = __ballot(cand);
    while (m) {
      const int j = __ffsll((unsigned long long)m) - 1;
      const float s = __shfl(sc, j);
      const uint32_t kk = __shfl(key, j);
      int pos = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) pos += __popcll(__ballot(64 * r + lane < k && better(ls[r], lk[r], s, kk)));
      float us[R];
      uint32_t uk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        us[r] = __shfl_up(ls[r], 1);
        uk[r] = __shfl_up(lk[r], 1);
        if (r > 0) {
          const float cs = __shfl(ls[r - 1], 63);
          const uint32_t ck = __shfl(lk[r - 1], 63);
          if (lane == 0) {
            us[r] = cs;
            uk[r] = ck;
          }
        }
      }
      float ts = 0.0f;
      uint32_t tk = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int i = 64 * r + lane;
        if (i > pos && i < k) {
          ls[r] = us[r];
          lk[r] = uk[r];
        }
        if (i == pos) {
          ls[r] = s;
          lk[r] = kk;
        }
        if (r == kr) {  // (no dynamic register index)
          ts = ls[r];
          tk = lk[r];
        }
      }
      kth = __shfl(ts, kl);
      kthk = __shfl(tk, kl);
      m &= m - 1;
      m &= __ballot(cand && better(sc, key, kth, kthk));
    }
  }
}

// ---------------------------------------------------------------------------
// pq_adc4: four queries per pass over the rows.  The LUT entries of the 4 queries for one
// (subspace, code) form one float4, so a single ds_read_b128 serves a row's lookup for all
// four: a random-bank LDS gather costs about the same per instruction at 4 B or 16 B per
// lane (MI355X_MICROARCH.md LDS table: b32 = 2 x 32-lane groups over 32 banks, b128 = 4 x
// 16-lane groups over 16 slots), so lookups per LDS cycle rise ~2x, and the codes and the
// codebook are read once per 4 queries.  The LUT is built PQ4_SC subspaces at a time into a
// double buffer (building pass p+1 overlaps the ADC of pass p; LDS holds 2 x PQ4_SC x ksub
// x 16 B, not M x ksub x 4 B per query).  Each lane keeps its rows' 4 running sums in
// registers across the passes, adding subspaces in m order (IvfPqVectorIndex.cs:182-186),
// so the scores are bit-identical to pq_scan_kernel's.  Rows per item <= PQ4_ROWS (longer
// lists are split into row chunks with their own partial slots, IvfChunking).
// ---------------------------------------------------------------------------
constexpr int PQ4_ROWS = 8192, PQ4_SC = 8, PQ4_MAX_NW = 16;

template <int SUB>
struct CbRow {  // one codebook centroid held in registers
  float v[SUB];
  __device__ float operator()(int i) const { return v[i]; }
};

template <int SUB, bool K256, int NT, int R>
__global__ __launch_bounds__(NT) void pq_adc4_kernel(PqArgs a) {
  constexpr int PQ4_NT = NT, PQ4_NW = NT / 64, PQ4_G = PQ4_ROWS / NT;  // row groups per wave
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nit = *a.n_items;
  const int per = (nit + 7) >> 3;  // XCD-major item mapping: the items of one list run on one XCD
  if ((int)(blockIdx.x >> 3) >= per) return;
  const int item = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
  if (item >= nit) return;
  const ScanItem it = a.items[item];
  const int D = a.dim, M = a.M, ksub = K256 ? 256 : a.ksub, k = a.k;
  const int sub = SUB > 0 ? SUB : D / M;
  const int npass = (M + PQ4_SC - 1) / PQ4_SC, nch = (M + 15) / 16;
  float4 *lut = reinterpret_cast<float4 *>(smem);  // [2][PQ4_SC][ksub] x 4 queries
  float *res = smem + 2 * PQ4_SC * ksub * 4;       // [4][D] residuals
  float *mrs = res + 4 * D;                        // [4][PQ4_NW][k] wave lists
  uint32_t *mrk = reinterpret_cast<uint32_t *>(mrs + 4 * PQ4_NW * k);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const float *cent = a.cents + (size_t)it.list * D;
  const int rb = it.row_begin, re = it.row_end;  // rb: multiple of 64
  const int ngrp = (re - rb + 63) >> 6;          // <= PQ4_NW * PQ4_G
  const uint2 *codes = reinterpret_cast<const uint2 *>(a.codes);

  // LUT entries of subspaces [p*SC, p*SC + SC) for the 4 residuals (ProductQuantizer.cs:112-117)
  auto build = [&](int p, int buf) {
#pragma unroll 1
    for (int e = tid; e < PQ4_SC * ksub; e += PQ4_NT) {
      const int j = e / ksub, c = e - j * ksub, m = p * PQ4_SC + j;
      if (m >= M) continue;
      const float *cb = a.codebooks + ((size_t)m * ksub + c) * sub;
      float4 o;
      if constexpr (SUB > 0) {
        CbRow<SUB> r;
#pragma unroll
        for (int t = 0; t < SUB; ++t) r.v[t] = cb[t];
        o.x = em_l2sq_unsafe(Off{res + m * SUB}, r, SUB);
        o.y = em_l2sq_unsafe(Off{res + D + m * SUB}, r, SUB);
        o.z = em_l2sq_unsafe(Off{res + 2 * D + m * SUB}, r, SUB);
        o.w = em_l2sq_unsafe(Off{res + 3 * D + m * SUB}, r, SUB);
      } else {
        o.x = em_l2sq_unsafe(Off{res + m * sub}, Off{cb}, sub);
        o.y = em_l2sq_unsafe(Off{res + D + m * sub}, Off{cb}, sub);
        o.z = em_l2sq_unsafe(Off{res + 2 * D + m * sub}, Off{cb}, sub);
        o.w = em_l2sq_unsafe(Off{res + 3 * D + m * sub}, Off{cb}, sub);
      }
      lut[buf * PQ4_SC * ksub + e] = o;
    }
  };

  for (int qb = 0; qb < it.qcnt; qb += 4) {
    for (int e = tid; e < 4 * D; e += PQ4_NT) {  // IvfPqVectorIndex.cs:161-163
      const int t = e / D, d = e - t * D, i = qb + t;
      float v = 0.0f;
      if (i < it.qcnt) v = a.queries[(size_t)(a.qlist[it.qbeg + i] / a.nparts) * D + d] - cent[d];
      res[e] = v;
    }
    __syncthreads();
    build(0, 0);
    __syncthreads();
    float acc[PQ4_G][4];
#pragma unroll
    for (int gi = 0; gi < PQ4_G; ++gi) acc[gi][0] = acc[gi][1] = acc[gi][2] = acc[gi][3] = 0.0f;
    for (int p = 0; p < npass; ++p) {
      const float4 *L = lut + (p & 1) * PQ4_SC * ksub;
      if (p + 1 < npass) build(p + 1, (p + 1) & 1);
#pragma unroll
      for (int gi = 0; gi < PQ4_G; ++gi) {
        const int g = w + gi * PQ4_NW;
        if (g < ngrp) {
          const int r = rb + g * 64 + lane;  // rows past `re` read the 64-row block padding
          const uint2 cw = codes[(((size_t)(r >> 6) * nch + (p >> 1)) * 64 + (r & 63)) * 2 + (p & 1)];
#pragma unroll
          for (int j = 0; j < PQ4_SC; ++j) {
            if (p * PQ4_SC + j < M) {
              const uint32_t word = j < 4 ? cw.x : cw.y;
              const float4 e = L[j * ksub + ((word >> (8 * (j & 3))) & 0xFF)];
              acc[gi][0] = acc[gi][0] + e.x;
              acc[gi][1] = acc[gi][1] + e.y;
              acc[gi][2] = acc[gi][2] + e.z;
              acc[gi][3] = acc[gi][3] + e.w;
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep one group's gathers in flight at a time (VGPRs)
      }
      __syncthreads();
    }
    // per-wave top-k of each query (lane-distributed lists), then wave t merges query t
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (qb + t >= it.qcnt) break;
      const int qi = a.qlist[it.qbeg + qb + t] / a.nparts;
      const float gs = a.gthr ? key_score(__hip_atomic_load(a.gthr + qi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : -INFINITY;
      float ls[R], kth = -INFINITY;
      uint32_t lk[R], kthk = KEY_NONE;
#pragma unroll
      for (int u = 0; u < R; ++u) {
        ls[u] = -INFINITY;
        lk[u] = KEY_NONE;
      }
#pragma unroll
      for (int gi = 0; gi < PQ4_G; ++gi) {
        const int g = w + gi * PQ4_NW;
        if (g < ngrp) {
          const int r = rb + g * 64 + lane;
          const bool valid = r < re && a.live[r];
          const float score = -acc[gi][t];  // :194
          const bool cand = valid && score >= gs && better(score, (uint32_t)r, kth, kthk);
          wave_list_insert_r<R>(cand, score, (uint32_t)r, ls, lk, kth, kthk, k, lane);
        }
      }
#pragma unroll
      for (int u = 0; u < R; ++u)
        if (64 * u + lane < k) {
          mrs[(t * PQ4_NW + w) * k + 64 * u + lane] = ls[u];
          mrk[(t * PQ4_NW + w) * k + 64 * u + lane] = lk[u];
        }
    }
    __syncthreads();
    if (w < 4 && qb + w < it.qcnt) {
      const int slot = a.qlist[it.qbeg + qb + w] + it.part;
      const int qi = slot / a.nparts;
      float ls[R], kth = -INFINITY;
      uint32_t lk[R], kthk = KEY_NONE;
#pragma unroll
      for (int u = 0; u < R; ++u) {
        ls[u] = -INFINITY;
        lk[u] = KEY_NONE;
      }
      for (int e0 = 0; e0 < PQ4_NW * k; e0 += 64) {
        const int e = e0 + lane;
        const float s = e < PQ4_NW * k ? mrs[w * PQ4_NW * k + e] : -INFINITY;
        const uint32_t kk = e < PQ4_NW * k ? mrk[w * PQ4_NW * k + e] : KEY_NONE;
        const bool cand = kk != KEY_NONE && better(s, kk, kth, kthk);
        wave_list_insert_r<R>(cand, s, kk, ls, lk, kth, kthk, k, lane);
      }
#pragma unroll
      for (int u = 0; u < R; ++u)
        if (64 * u + lane < k) {
          a.part_s[(size_t)slot * k + 64 * u + lane] = ls[u];
          a.part_k[(size_t)slot * k + 64 * u + lane] = lk[u];
        }
      if (lane == 0 && a.gthr && kthk != KEY_NONE) atomicMax(a.gthr + qi, score_key(kth));
    }
    // waves 0-3 finish reading mrs / mrk before the barrier after the next quad's residuals
  }
}

__global__ void pq_encode_kernel(const float *x, const int32_t *assign, const float *cents, int64_t n, int D, int M,
                                 int ksub, const float *cb, uint8_t *codes) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * M;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / M;
    const int m = (int)(e % M);
    const int sub = D / M;
    const float *xs = x + (size_t)i * D + (size_t)m * sub;
    const float *cs = cents + (size_t)assign[i] * D + (size_t)m * sub;
    struct R {
      const float *x, *c;
      __device__ float operator()(int d) const { return x[d] - c[d]; }
    };
    float mind = FLT_MAX;
    int best = 0;
    for (int j = 0; j < ksub; ++j) {  // ProductQuantizer.cs:124-134
      const float d = em_l2sq_unsafe(R{xs, cs}, Off{cb + ((size_t)m * ksub + j) * sub}, sub);
      if (d < mind) {
        mind = d;
        best = j;
      }
    }
    codes[i * M + m] = (uint8_t)best;
  }
}

__global__ void residuals_kernel(const float *x, const int32_t *assign, const float *cents, int64_t n, int D,
                                 float *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    out[e] = x[e] - cents[(size_t)assign[i] * D + d];
  }
}

__global__ void extract_sub_kernel(const float *x, int64_t n, int D, int off, int sub, float *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * sub;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / sub;
    const int d = (int)(e % sub);
    out[e] = x[(size_t)i * D + off + d];
  }
}

__global__ void pack_codes_kernel(const uint8_t *codes, const int64_t *src, int64_t ndst, int M, uint8_t *out) {
  const int nch = (M + 15) / 16;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ndst * nch * 16;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t r = e / (nch * 16);
    const int m = (int)(e % (nch * 16));
    const int64_t s = src[r];
    const uint8_t v = (s >= 0 && m < M) ? codes[(size_t)s * M + m] : 0;
    out[pq_code_off(r, m >> 4, nch) + (m & 15)] = v;
  }
}

// ---------------------------------------------------------------------------
// layout helpers
// ---------------------------------------------------------------------------
__global__ void to_blocked_kernel(const float *src, const int64_t *sidx, int64_t n, int D, float *dst, int64_t r0) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    const int64_t s = sidx ? sidx[i] : i;
    dst[blk_off(r0 + i, d, D)] = s >= 0 ? src[(size_t)s * D + d] : 0.0f;
  }
}
__global__ void scatter_blocked_kernel(const float *src, const int64_t *slots, int64_t n, int D, float *dst) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    dst[blk_off(slots[i], d, D)] = src[e];
  }
}
// row-major copies (RowStore::rrm, the refine's rows): dst row i = src row sidx[i] (0 when < 0), or the
// rows scattered to their slots
__global__ void to_rowmajor_kernel(const float *src, const int64_t *sidx, int64_t n, int D, float *dst) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    const int64_t s = sidx ? sidx[i] : i;
    dst[e] = s >= 0 ? src[(size_t)s * D + d] : 0.0f;
  }
}
__global__ void scatter_rowmajor_kernel(const float *src, const int64_t *slots, int64_t n, int D, float *dst) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    dst[(size_t)slots[i] * D + d] = src[e];
  }
}
__global__ void gather_blocked_kernel(const float *src, const int64_t *slots, int64_t n, int D, float *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    out[e] = src[blk_off(slots[i], d, D)];
  }
}
__global__ void gather2_kernel(const float *A, const float *B, const int64_t *idx, int64_t n, int D, float *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    const int64_t s = idx[i];
    out[e] = s >= 0 ? A[blk_off(s, d, D)] : B[blk_off(-s - 1, d, D)];
  }
}
template <class T>
__global__ void gather_rows_kernel(const T *src, const int32_t *idx, int64_t n, int D, T *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    const int d = (int)(e % D);
    out[e] = src[(size_t)idx[i] * D + d];
  }
}

// ---------------------------------------------------------------------------
// k-means (KMeansUtils.cs:40-62)
// ---------------------------------------------------------------------------
__global__ void keys_to_assign_kernel(const uint32_t *keys, int64_t n, int32_t *assign) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) assign[i] = (int32_t)keys[i];
}

// one thread per (cluster, dim): members summed in data order, then / Count.
__global__ void kmeans_sum_kernel(const float *data, const int32_t *members, const int32_t *coff, int k, int D,
                                  const float *cents, float *tmp, int32_t *flags) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (d >= D || c >= k) return;
  const int b = coff[c], e = coff[c + 1];
  if (b == e) return;  // :48 empty cluster keeps its centroid
  float s = 0.0f;
  int i = b;
  for (; i + 4 <= e; i += 4) {
    const float v0 = data[(size_t)members[i] * D + d];
    const float v1 = data[(size_t)members[i + 1] * D + d];
    const float v2 = data[(size_t)members[i + 2] * D + d];
    const float v3 = data[(size_t)members[i + 3] * D + d];
    s = s + v0;
    s = s + v1;
    s = s + v2;
    s = s + v3;
  }
  for (; i < e; ++i) s = s + data[(size_t)members[i] * D + d];
  const float nc = s / (float)(e - b);  // :55 newC[d] /= Count
  tmp[(size_t)c * D + d] = nc;
  if ((double)fabsf(cents[(size_t)c * D + d] - nc) > 1e-6) flags[c] = 1;  // ArraysEqual :95-101
}
__global__ void kmeans_commit_kernel(float *cents, const float *tmp, const int32_t *flags, int k, int D,
                                     int32_t *changed) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)k * D) return;
  const int c = (int)(e / D);
  if (flags[c]) {
    cents[e] = tmp[e];
    if (e % D == 0) atomicOr(changed, 1);
  }
}

// up to WordFill::MAXR ranges of 32-bit words set to their value in one grid-stride launch (the
// per-search counter resets: no hipMemsetAsync on a search path, see launch_fill_words)
__global__ void fill_words_kernel(WordFill f) {
  int64_t tot = 0;
  for (int r = 0; r < f.cnt; ++r) tot += f.n[r];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = e;
    int r = 0;
    while (o >= f.n[r]) o -= f.n[r++];
    f.p[r][o] = f.v[r];
  }
}

__global__ void list_ids_kernel(const int32_t *lb, const int32_t *le, int32_t *out) {
  const int l = blockIdx.x;
  for (int r = lb[l] + threadIdx.x; r < le[l]; r += blockDim.x) out[r] = l;
}

__global__ void copy_words_kernel(uint32_t *dst, const uint32_t *src, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    dst[e] = src[e];
}

__global__ void fill_u8_kernel(uint8_t *p, uint8_t v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void scatter_i64_kernel(int64_t *dst, const int64_t *idx, const int64_t *vals, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = vals[i];
}
__global__ void scatter_u8_kernel(uint8_t *dst, const int64_t *idx, uint8_t v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = v;
}
__global__ void norms_slots_kernel(const float *rows, const int64_t *slots, int64_t n, int dim, float *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots[i];
  out[r] = em_norm(Blk{rows, dim, r}, dim);
}
__global__ void labels_to_i32_kernel(const int64_t *in, int64_t n, int32_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)in[i];
}

__global__ void fill_results_kernel(float *s, int64_t *l, int32_t *c, int64_t nq, int k) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nq * k) {
    if (s) s[i] = -INFINITY;
    if (l) l[i] = -1;
  }
  if (c && i < nq) c[i] = 0;
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

template <int D, int V, int MET, int GPS, bool IVF, int QS, int W>
void launch_fast_i(const ScanArgs &a, int max_items, hipStream_t st) {
  const size_t lds =
      (size_t)(2 * GPS * D * 8 + 2 * QCHUNK * score_stride<GPS>() + QCHUNK * a.k * 2) * sizeof(float);
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&scan_fast<D, V, MET, GPS, IVF, QS, W>), attr);
  hipLaunchKernelGGL((scan_fast<D, V, MET, GPS, IVF, QS, W>), dim3(max_items), dim3(8 * QCHUNK / QS), lds, st, a);
}

// Register-tile variant of the fast scan: QS = 2 (512 threads); the safe form (V = 1) with a register
// cap for 6 waves per SIMD (80 VGPRs, a small spill), the *Unsafe form (V = 4) at 4 waves (~98 VGPRs).
// (Round 2 also measured QS = 4 / 256 threads: slower at both.)
template <int D, int V, int MET, int GPS, bool IVF>
void launch_fast_var(const ScanArgs &a, int max_items, hipStream_t st) {
  if constexpr (V == 1) launch_fast_i<D, V, MET, GPS, IVF, 2, 6>(a, max_items, st);
  else launch_fast_i<D, V, MET, GPS, IVF, 2, 1>(a, max_items, st);
}

template <int D, int V, int MET>
void launch_fast_t(const ScanArgs &a, int max_items, hipStream_t st) {
  if constexpr (V == 1) {  // IVF list scans use the safe (1-accumulator) VectorMath form
    if (a.qlist) {
      launch_fast_var<D, V, MET, 1, true>(a, max_items, st);
      return;
    }
  }
  launch_fast_var<D, V, MET, 1, false>(a, max_items, st);
}

template <int V, int MET>
void launch_generic_t(const ScanArgs &a, int max_items, hipStream_t st) {
  const size_t lds = (size_t)64 * a.k * 8;
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&scan_generic<V, MET>), attr);
  hipLaunchKernelGGL((scan_generic<V, MET>), dim3(max_items), dim3(64), lds, st, a);
}

template <int D, int V>
void launch_fast_m(const ScanArgs &a, int metric, int max_items, hipStream_t st) {
  if (metric == L2) launch_fast_t<D, V, L2>(a, max_items, st);
  else if (metric == IP) launch_fast_t<D, V, IP>(a, max_items, st);
  else launch_fast_t<D, V, COS>(a, max_items, st);
}
template <int D>
void launch_fast_v(const ScanArgs &a, int metric, int V, int max_items, hipStream_t st) {
  if (V == 4) launch_fast_m<D, 4>(a, metric, max_items, st);
  else launch_fast_m<D, 1>(a, metric, max_items, st);
}


// ---- exact IVF re-run of certificate failures, device-driven (IvfRerunArgs, kernels.h) ----
__device__ __forceinline__ uint64_t rr_shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rr_shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rr_sort64_desc(uint64_t v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j >= 1; j >>= 1) {
      const uint64_t o = rr_shfl_xor64(v, j);
      const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == desc) ? (v > o ? v : o) : (v < o ? v : o);
    }
  return v;
}
__device__ __forceinline__ uint64_t rr_merge64_desc(uint64_t v, int lane) {  // bitonic -> sorted desc
#pragma unroll
  for (int j = 32; j >= 1; j >>= 1) {
    const uint64_t o = rr_shfl_xor64(v, j);
    v = (lane & j) == 0 ? (v > o ? v : o) : (v < o ? v : o);
  }
  return v;
}
// rank key: score desc, then storage slot asc (~slot); 0 = no entry
__device__ __forceinline__ uint64_t rr_key(float s, uint32_t slot) { return ((uint64_t)score_key(s) << 32) | (uint32_t)~slot; }

// Work units are (failing query i, probe p, chunk c): every probed list is cut into nc near-equal
// chunks of whole 64-row groups, nc = min(a.nchunk, ceil(RR_UNITS / (nfail * nprobe))) -- a few
// failures spread over every CU, many keep one unit per (query, probe).  One block per unit: the
// exact scores of the chunk's live rows, its top k (<= 64) to part[u * k ..] as rank keys (score
// desc, slot asc; 0 = none).
constexpr int64_t RR_UNITS = 8192;
__device__ __forceinline__ int rr_nchunks(int64_t pairs, int nchunk) {
  if (pairs <= 0) return 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(nchunk, (RR_UNITS + pairs - 1) / pairs));
}
// em_score<1, MET> (the safe L2Squared / DotProduct) of blocked row r for a compile-time D, the row
// read 32 dims at a time (the sums keep the reference order: acc[l] over i ascending, then hsum8)
template <int MET, int DT>
__device__ __forceinline__ float rr_score(const float *qs, const float *rows, int64_t r) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
  for (int i0 = 0; i0 < DT; i0 += 32) {
    float x[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) x[d] = rows[blk_off(r, i0 + d, DT)];
#pragma unroll
    for (int i = 0; i < 32; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        if (MET == L2) {
          const float d = qs[i0 + i + l] - x[i + l];
          acc[l] = acc[l] + d * d;
        } else {
          acc[l] = acc[l] + qs[i0 + i + l] * x[i + l];
        }
      }
  }
  const float sum = 0.0f + hsum8(acc);
  return MET == L2 ? -sum : sum;
}

__device__ void rerun_merge_one(IvfRerunArgs a, const uint64_t *part, int64_t i, int lane);
template <int MET, int DT, int V = 1>
__global__ __launch_bounds__(256) void ivf_rerun_scan_kernel(IvfRerunArgs a, uint64_t *part) {
  __shared__ uint64_t wl[4][64];
  __shared__ float qsh[DT > 0 ? DT : 1];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int D = DT > 0 ? DT : a.dim, k = a.k;
  const int64_t pairs = (int64_t)(*a.nfail) * a.nprobe;
  const int nc = rr_nchunks(pairs, a.nchunk);
  const int64_t units = pairs * nc;
  for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    const int64_t pi = u / nc;
    const int c = (int)(u - pi * nc);
    const int64_t i = pi / a.nprobe;
    const int p = (int)(pi - i * a.nprobe);
    const int64_t q = a.fail[i];
    const float *qp = a.queries + (size_t)q * D;
    if constexpr (DT > 0) {
      if (threadIdx.x < DT) qsh[threadIdx.x] = qp[threadIdx.x];
      __syncthreads();
    }
    const int lst = a.probes[(size_t)q * (a.pstride > 0 ? a.pstride : a.nprobe) + p];
    uint64_t cur = 0ull;  // lane j: the wave's j-th best so far
    if (lst >= 0) {
      const int b = a.lb[lst];
      const int e = a.qlim ? (int)min((uint32_t)a.le[lst], max((uint32_t)b, a.qlim[(size_t)q * a.nprobe + p]))
                           : a.le[lst];  // MaxScans: the rows before the bound (:202-212)
      const int cl = (((e - b) + nc - 1) / nc + 63) & ~63;
      const int cb = b + c * cl, ce = min(e, cb + cl);
      for (int r0 = cb + 64 * w; r0 < ce; r0 += 256) {
        const int r = r0 + lane;
        uint64_t key = 0ull;
        if (r < ce && a.live[r]) {
          float sc;
          if constexpr (MET == COS) {  // VectorMath.Cosine (:102-109) with the cached norms
            const float qn = a.qnorm[q], xn = a.rnorm[r];
            float dot;
            if constexpr (V == 4) dot = em_score<4, IP>(Lin{qp}, Blk{a.rows, D, r}, D, 0.0f, 0.0f);  // FLAT (:354)
            else if constexpr (DT > 0) dot = rr_score<IP, DT>(qsh, a.rows, r);
            else dot = em_score<1, IP>(Lin{qp}, Blk{a.rows, D, r}, D, 0.0f, 0.0f);
            sc = (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
          } else if constexpr (V == 4) {  // FLAT (BruteForceVectorIndex.cs:350-356): the *Unsafe forms
            sc = em_score<4, MET>(Lin{qp}, Blk{a.rows, D, r}, D, 0.0f, 0.0f);
          } else if constexpr (DT > 0) {
            sc = rr_score<MET, DT>(qsh, a.rows, r);
          } else {
            sc = em_score<1, MET>(Lin{qp}, Blk{a.rows, D, r}, D, 0.0f, 0.0f);
          }
          if (!isnan(sc)) key = rr_key(sc, (uint32_t)r);  // NaN never ranks (as better() in the scans)
        }
        const uint64_t kth = rr_shfl64(cur, k - 1);
        if (!__builtin_amdgcn_ballot_w64(key > kth)) continue;
        key = rr_sort64_desc(key, lane);
        const uint64_t rv = rr_shfl64(key, 63 - lane);
        cur = rr_merge64_desc(cur > rv ? cur : rv, lane);
      }
    }
    wl[w][lane] = cur;
    __syncthreads();
    if (w == 0) {
      for (int o = 1; o < 4; ++o) {
        const uint64_t rv = wl[o][63 - lane];
        cur = rr_merge64_desc(cur > rv ? cur : rv, lane);
      }
      if (lane < k) part[u * k + lane] = cur;
      if (a.done) {  // the query's last unit merges it (its units' parts are visible after the fences)
        __threadfence();
        int last = 0;
        if (lane == 0) last = atomicAdd(a.done + i, 1) == a.nprobe * nc - 1;
        if (__shfl(last, 0)) {
          __threadfence();
          rerun_merge_one(a, part, i, lane);
          if (lane == 0) a.done[i] = 0;
        }
      }
    }
    __syncthreads();
  }
}

// one wave per failing query: its nprobe x nc partial lists merged, the top k written at the query's row
__global__ __launch_bounds__(256) void ivf_rerun_merge_kernel(IvfRerunArgs a, const uint64_t *part) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nfail = *a.nfail;
  // grid-stride over the failing queries (a small grid: it exits at once when nothing failed)
  for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < nfail; i += (int64_t)gridDim.x * 4) rerun_merge_one(a, part, i, lane);
}
__device__ void rerun_merge_one(IvfRerunArgs a, const uint64_t *part, int64_t i, int lane) {
  const int64_t nfail = *a.nfail;
  const int k = a.k;
  const int64_t q = a.fail[i];
  const int nc = rr_nchunks(nfail * a.nprobe, a.nchunk);
  const uint64_t *pp = part + (size_t)i * a.nprobe * nc * k;
  const int n = a.nprobe * nc * k;
  uint64_t cur = 0ull;
  // 8 rows of 64 keys loaded at once (independent loads: one L2 round trip per 512 keys, not per 64)
  for (int b0 = 0; b0 < n; b0 += 512) {
    uint64_t vv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vv[j] = b0 + 64 * j + lane < n ? pp[b0 + 64 * j + lane] : 0ull;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t v = vv[j];
      const uint64_t kth = rr_shfl64(cur, k - 1);
      if (!__builtin_amdgcn_ballot_w64(v > kth)) continue;
      v = rr_sort64_desc(v, lane);
      const uint64_t rv = rr_shfl64(v, 63 - lane);
      cur = rr_merge64_desc(cur > rv ? cur : rv, lane);
    }
  }
  const uint64_t real = __builtin_amdgcn_ballot_w64(lane < k && cur != 0ull);
  if (a.rec) {  // list-sharded re-run (shard.hip): the exact local top-k as record rec_pos[i], bound -inf
    uint8_t *rp = static_cast<uint8_t *>(a.rec) + (size_t)a.rec_pos[i] * shard_record_bytes(k);
    if (lane < k) {
      ShardEntry e;
      e.label = -1;
      e.score = -INFINITY;
      e.list = 0x7FFFFFFF;
      if (cur != 0ull) {
        const uint32_t slot = ~(uint32_t)cur;
        e.label = a.labels[slot];
        e.score = key_score((uint32_t)(cur >> 32));
        e.list = shard_list_of(a.rec_lb, a.rec_nlist, slot);
      }
      reinterpret_cast<ShardEntry *>(rp)[lane] = e;
    }
    if (lane == 0) {
      ShardTrailer t;
      t.bound = -INFINITY;
      t.n = (int32_t)__builtin_popcountll(real);
      t.pad = 0;
      *reinterpret_cast<ShardTrailer *>(rp + 16 * (size_t)k) = t;
    }
    return;
  }
  if (lane < k) {
    float s = -INFINITY;
    int64_t lab = -1;
    if (cur != 0ull) {
      s = key_score((uint32_t)(cur >> 32));
      lab = a.labels[~(uint32_t)cur];
    }
    a.out_s[(size_t)q * k + lane] = s;
    a.out_l[(size_t)q * k + lane] = lab;
  }
  if (lane == 0 && a.out_c) a.out_c[q] = (int32_t)__builtin_popcountll(real);
}
}  // namespace

bool fast_path(int dim, int k) { return k <= KMAX_FAST && (dim == 32 || dim == 64 || dim == 96 || dim == 128); }

void launch_scan(const ScanArgs &a, int metric, int V, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  if (fast_path(a.dim, a.k) && a.queries_t) {
    switch (a.dim) {
      case 32: launch_fast_v<32>(a, metric, V, max_items, st); return;
      case 64: launch_fast_v<64>(a, metric, V, max_items, st); return;
      case 96: launch_fast_v<96>(a, metric, V, max_items, st); return;
      default: launch_fast_v<128>(a, metric, V, max_items, st); return;
    }
  }
  if (V == 4) {
    if (metric == L2) launch_generic_t<4, L2>(a, max_items, st);
    else if (metric == IP) launch_generic_t<4, IP>(a, max_items, st);
    else launch_generic_t<4, COS>(a, max_items, st);
  } else {
    if (metric == L2) launch_generic_t<1, L2>(a, max_items, st);
    else if (metric == IP) launch_generic_t<1, IP>(a, max_items, st);
    else launch_generic_t<1, COS>(a, max_items, st);
  }
}

int make_flat_items(ScanItem *d_items, int32_t *d_nitems, int64_t nrows, int32_t chunk_rows, int64_t nq,
                    int32_t part_off, int32_t qchunk, hipStream_t st) {
  const int nchunks = (int)((nrows + chunk_rows - 1) / chunk_rows);
  const int nqc = (int)((nq + qchunk - 1) / qchunk);
  const int n = nchunks * nqc;
  hipLaunchKernelGGL(flat_items_kernel, dim3(nblk(n > 0 ? n : 1, 256)), dim3(256), 0, st, d_items, d_nitems, nchunks,
                     nqc, chunk_rows, nrows, nq, part_off, qchunk);
  return n;
}

void launch_transpose_queries(const float *q, int64_t nq, int32_t dim, float *qt, hipStream_t st) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(transpose_queries_kernel, dim3(gblk(nq * dim)), dim3(256), 0, st, q, nq, dim, qt);
}

void launch_norms(const float *x, int64_t n, int32_t dim, int blocked, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(norms_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, x, n, dim, blocked, out);
}

void launch_merge_keys(const float *ps, const uint32_t *pk, int64_t nq, int32_t nparts, int32_t k,
                       const int64_t *row_labels, const int64_t *buf_labels, float *out_s, int64_t *out_l,
                       int32_t *out_keys, int32_t *out_cnt, hipStream_t st, const MergeIvf *ivf) {
  if (nq <= 0) return;
  const MergeIvf iv = ivf ? *ivf : MergeIvf{};
  const dim3 g(nblk(nq, 4)), b(256);
  if (nparts <= 64)
    hipLaunchKernelGGL(merge_keys_kernel<1>, g, b, 0, st, ps, pk, nq, nparts, k, row_labels, buf_labels, out_s, out_l,
                       out_keys, out_cnt, iv);
  else if (nparts <= 128)
    hipLaunchKernelGGL(merge_keys_kernel<2>, g, b, 0, st, ps, pk, nq, nparts, k, row_labels, buf_labels, out_s, out_l,
                       out_keys, out_cnt, iv);
  else if (nparts <= 256)
    hipLaunchKernelGGL(merge_keys_kernel<4>, g, b, 0, st, ps, pk, nq, nparts, k, row_labels, buf_labels, out_s, out_l,
                       out_keys, out_cnt, iv);
  else
    hipLaunchKernelGGL(merge_keys_kernel<MAX_PARTS / 64>, g, b, 0, st, ps, pk, nq, nparts, k, row_labels, buf_labels,
                       out_s, out_l, out_keys, out_cnt, iv);
}

void launch_labels_to_i32(const int64_t *in, int64_t n, int32_t *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(labels_to_i32_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, in, n, out);
}

void launch_merge_labels(const float *ps, const int64_t *pl, int64_t nq, int32_t nparts, int32_t k, float *out_s,
                         int64_t *out_l, hipStream_t st, bool part_major) {
  if (nq <= 0) return;
  const int64_t sq = part_major ? k : (int64_t)nparts * k, sp = part_major ? nq * k : k;
  hipLaunchKernelGGL(merge_labels_kernel, dim3(nblk(nq, 4)), dim3(256), 0, st, ps, pl, nq, nparts, k, sq, sp, out_s,
                     out_l);
}

int64_t ivf_max_items(int64_t nq, int32_t nprobe, int32_t nlist, int32_t qchunk, IvfChunking ch, int phase) {
  // sum_l ceil(cnt_l / qchunk) * chunks_l <= chunks_max * (ceil(nq * nprobe / qchunk) + nlist)
  const int64_t cm = ch.warm > 0 ? (phase == 0 ? 1 : std::max(1, ch.cmax - 1)) : ch.cmax;
  return cm * ((nq * nprobe + qchunk - 1) / qchunk + nlist);
}

void launch_ivf_items(const int32_t *probes, int64_t nq, int32_t nprobe, int32_t nparts, int32_t nlist,
                      const int32_t *list_begin, const int32_t *list_end, int32_t qchunk, IvfChunking ch,
                      int phase, IvfItemWs &ws, hipStream_t st, int32_t pb, int32_t pe, bool balance, bool zeroed) {
  if (pe < 0) pe = nprobe;
  const int64_t n = nq * (pe - pb);
  const bool lds = nlist <= IVF_LDS_BINS && !knob("PYR_IVF_GLOBAL_HIST");  // (knob: measurement only)
  const size_t hb = sizeof(int) * (size_t)nlist;
  // skip_empty (a list-sharded rank): the (query, probe) entries of the lists it does not hold take no slot
  const int32_t *skb = ch.skip_empty ? list_begin : nullptr, *ske = ch.skip_empty ? list_end : nullptr;
  if (phase == 0) {
    if (!zeroed) {
      WordFill z;
      z.add(ws.cnt, nlist, 0);
      z.add(ws.fill, nlist, 0);
      launch_fill_words(z, st);
    }
    if (n > 0 && lds && ivf_ept(n) == 16)
      hipLaunchKernelGGL(ivf_count_lds_kernel<16>, dim3(nblk(n, 256 * 16)), dim3(256), hb, st, probes, nq, nprobe, pb,
                         pe, nlist, ws.cnt, skb, ske);
    else if (n > 0 && lds)
      hipLaunchKernelGGL(ivf_count_lds_kernel<4>, dim3(nblk(n, 256 * 4)), dim3(256), hb, st, probes, nq, nprobe, pb, pe,
                         nlist, ws.cnt, skb, ske);
    else if (n > 0)
      hipLaunchKernelGGL(ivf_count_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, probes, nq, nprobe, pb, pe, ws.cnt, skb,
                         ske);
  }
  hipLaunchKernelGGL(ivf_scan_kernel, dim3(1), dim3(1024), 0, st, ws.cnt, nlist, qchunk, list_begin, list_end, ch,
                     phase, ws.qoff, ws.ioff, ws.n_items, balance ? 1 : 0, ws.items);
  if (phase == 0 && n > 0 && lds && ivf_ept(n) == 16)
    hipLaunchKernelGGL(ivf_fill_lds_kernel<16>, dim3(nblk(n, 256 * 16)), dim3(256), hb, st, probes, nq, nprobe, pb, pe,
                       nparts, ch.cmax, nlist, ws.qoff, ws.fill, ws.qlist, pb == 0 && pe == nprobe ? ws.qpos : nullptr,
                       skb, ske);
  else if (phase == 0 && n > 0 && lds)
    hipLaunchKernelGGL(ivf_fill_lds_kernel<4>, dim3(nblk(n, 256 * 4)), dim3(256), hb, st, probes, nq, nprobe, pb, pe,
                       nparts, ch.cmax, nlist, ws.qoff, ws.fill, ws.qlist, pb == 0 && pe == nprobe ? ws.qpos : nullptr,
                       skb, ske);
  else if (phase == 0 && n > 0)
    hipLaunchKernelGGL(ivf_fill_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, probes, nq, nprobe, pb, pe, nparts,
                       ch.cmax, ws.qoff, ws.fill, ws.qlist, pb == 0 && pe == nprobe ? ws.qpos : nullptr, skb, ske);
}

void launch_ivf_limits(const int32_t *probes, int64_t nq, int32_t nprobe, int32_t nparts, int64_t remaining,
                       const int32_t *list_begin, const int32_t *list_end, const int32_t *list_live,
                       const uint8_t *live, IvfChunking ch, uint32_t *limits, hipStream_t st, const int32_t *prem,
                       int rstride) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(ivf_limits_kernel, dim3(nblk(nq, 4)), dim3(256), 0, st, probes, nq, nprobe, nparts, ch.cmax,
                     remaining, list_begin, list_end, list_live, live, limits, prem, rstride);
}

void launch_pos_limits(const int32_t *qpos, const uint32_t *limits, int64_t n, uint32_t *plim, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(pos_limits_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, qpos, limits, n, plim);
}

size_t pq_scan_lds_bytes(int dim, int M, int ksub, int k) {
  return (size_t)(((dim + 3) & ~3) + M * ksub + 2 * k + 2 * 256 + 4) * 4;
}

// k <= 64: 1024-thread blocks (measured 1.5x faster than 512), one list register; k <= 256: 512 threads (the
// 8 waves' lists of k entries per query fit the LDS beside the LUT), four list registers
constexpr int PQ4_DEEP_NT = 512, PQ4_KMAX = 256;
size_t pq_adc4_lds_bytes(int dim, int ksub, int k) {  // sized for the largest block
  const int nw = k > 64 ? PQ4_DEEP_NT / 64 : PQ4_MAX_NW;
  return (size_t)(2 * PQ4_SC * ksub * 4 + 4 * dim + 2 * 4 * nw * k) * 4;
}
int pq_adc4_rows() { return PQ4_ROWS; }
bool pq_adc4_supported(int dim, int M, int ksub, int k) {
  return k >= 1 && k <= PQ4_KMAX && ksub <= 256 && M >= 1 && pq_adc4_lds_bytes(dim, ksub, k) <= 160 * 1024;
}
template <int SUB, bool K256, int NT, int R>
static void launch_pq_adc4_nt(const PqArgs &a, int max_items, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&pq_adc4_kernel<SUB, K256, NT, R>), attr);
  const int grid = (max_items + 7) / 8 * 8;
  hipLaunchKernelGGL((pq_adc4_kernel<SUB, K256, NT, R>), dim3(grid), dim3(NT), pq_adc4_lds_bytes(a.dim, a.ksub, a.k),
                     st, a);
}
template <int SUB, bool K256>
static void launch_pq_adc4_t(const PqArgs &a, int max_items, hipStream_t st) {
  if (a.k <= 64) launch_pq_adc4_nt<SUB, K256, 1024, 1>(a, max_items, st);
  else launch_pq_adc4_nt<SUB, K256, PQ4_DEEP_NT, PQ4_KMAX / 64>(a, max_items, st);
}
void launch_pq_adc4(const PqArgs &a, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  if (!pq_adc4_supported(a.dim, a.M, a.ksub, a.k)) throw std::invalid_argument("pq_adc4: unsupported shape");
  const int sub = a.dim / a.M;
  const bool k256 = a.ksub == 256;
  if (sub == 8) {
    if (k256) launch_pq_adc4_t<8, true>(a, max_items, st);
    else launch_pq_adc4_t<8, false>(a, max_items, st);
  } else if (sub == 4) {
    if (k256) launch_pq_adc4_t<4, true>(a, max_items, st);
    else launch_pq_adc4_t<4, false>(a, max_items, st);
  } else if (sub == 16) {
    if (k256) launch_pq_adc4_t<16, true>(a, max_items, st);
    else launch_pq_adc4_t<16, false>(a, max_items, st);
  } else {
    if (k256) launch_pq_adc4_t<0, true>(a, max_items, st);
    else launch_pq_adc4_t<0, false>(a, max_items, st);
  }
}

void launch_pq_scan(const PqArgs &a, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&pq_scan_kernel), attr);
  hipLaunchKernelGGL(pq_scan_kernel, dim3(max_items), dim3(256), pq_scan_lds_bytes(a.dim, a.M, a.ksub, a.k), st, a);
}

void launch_pq_encode(const float *x, const int32_t *assign, const float *cents, int64_t n, int32_t dim, int32_t M,
                      int32_t ksub, const float *codebooks, uint8_t *codes, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(pq_encode_kernel, dim3(gblk(n * M)), dim3(256), 0, st, x, assign, cents, n, dim, M, ksub,
                     codebooks, codes);
}
void launch_residuals(const float *x, const int32_t *assign, const float *cents, int64_t n, int32_t dim, float *out,
                      hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(residuals_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, x, assign, cents, n, dim, out);
}
void launch_extract_sub(const float *x, int64_t n, int32_t dim, int32_t off, int32_t sub, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(extract_sub_kernel, dim3(gblk(n * sub)), dim3(256), 0, st, x, n, dim, off, sub, out);
}
void launch_pack_codes(const uint8_t *codes, const int64_t *src_of_dst, int64_t ndst, int32_t M, uint8_t *out,
                       hipStream_t st) {
  if (ndst <= 0) return;
  const int nch = (M + 15) / 16;
  hipLaunchKernelGGL(pack_codes_kernel, dim3(gblk(ndst * nch * 16)), dim3(256), 0, st, codes, src_of_dst, ndst,
                     M, out);
}

void launch_to_blocked(const float *src, const int64_t *src_idx, int64_t n, int32_t dim, float *dst, int64_t dst_row0,
                       hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(to_blocked_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, src, src_idx, n, dim, dst,
                     dst_row0);
}
void launch_scatter_blocked(const float *src, const int64_t *dst_slots, int64_t n, int32_t dim, float *dst,
                            hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_blocked_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, src, dst_slots, n, dim, dst);
}
void launch_to_rowmajor(const float *src, const int64_t *src_idx, int64_t n, int32_t dim, float *dst, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(to_rowmajor_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, src, src_idx, n, dim, dst);
}
void launch_scatter_rowmajor(const float *src, const int64_t *dst_slots, int64_t n, int32_t dim, float *dst,
                             hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_rowmajor_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, src, dst_slots, n, dim, dst);
}
void launch_gather_blocked(const float *src, const int64_t *src_slots, int64_t n, int32_t dim, float *out,
                           hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_blocked_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, src, src_slots, n, dim, out);
}
void launch_gather2(const float *A, const float *B, const int64_t *idx, int64_t n, int32_t dim, float *out,
                    hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather2_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, A, B, idx, n, dim, out);
}
void launch_gather_rows(const float *src, const int32_t *idx, int64_t n, int32_t dim, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(gblk(n * dim)), dim3(256), 0, st, src, idx, n, dim, out);
}

void launch_gather_rows_i32(const int32_t *src, const int32_t *idx, int64_t n, int32_t width, int32_t *out,
                            hipStream_t st) {
  if (n <= 0 || width <= 0) return;
  hipLaunchKernelGGL(gather_rows_kernel<int32_t>, dim3(gblk(n * width)), dim3(256), 0, st, src, idx, n, width,
                     out);
}

void launch_keys_to_assign(const uint32_t *keys, int64_t n, int32_t *assign, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(keys_to_assign_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, keys, n, assign);
}

void launch_kmeans_update(const float *data, const int32_t *members, const int32_t *coff, int32_t k, int32_t dim,
                          float *cents, float *tmp, int32_t *flags, int32_t *changed, hipStream_t st) {
  (void)hipMemsetAsync(flags, 0, sizeof(int32_t) * k, st);
  (void)hipMemsetAsync(changed, 0, sizeof(int32_t), st);
  const int bx = dim < 64 ? dim : 64;
  hipLaunchKernelGGL(kmeans_sum_kernel, dim3((dim + bx - 1) / bx, k), dim3(bx), 0, st, data, members, coff, k, dim,
                     cents, tmp, flags);
  hipLaunchKernelGGL(kmeans_commit_kernel, dim3(nblk((int64_t)k * dim, 256)), dim3(256), 0, st, cents, tmp, flags, k,
                     dim, changed);
}

void launch_scatter_i64(int64_t *dst, const int64_t *idx, const int64_t *vals, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_i64_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, dst, idx, vals, n);
}
void launch_scatter_u8(uint8_t *dst, const int64_t *idx, uint8_t v, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scatter_u8_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, dst, idx, v, n);
}
namespace {
__global__ __launch_bounds__(64) void write_small_kernel(SmallWriteArgs a, SmallWriteRows inl) {
  // the row comes from host-coherent memory (kernel arguments or a mapped host slot): one coalesced read of
  // it into LDS, every later pass reads LDS (a lane's sequential loop over host memory took ~20 us)
  __shared__ float xsh[SMALL_WRITE_MAX_DIM];
  const int i = blockIdx.x, lane = threadIdx.x, D = a.dim;
  const int64_t r = a.x ? a.slots[i] : inl.slot[i];
  const float *xg = a.x ? a.x + (size_t)i * D : inl.x + (size_t)i * D;
  for (int d = lane; d < D; d += 64) {
    const float v = xg[d];
    xsh[d] = v;
    a.rows[blk_off(r, d, D)] = v;
    if (a.rrm) a.rrm[(size_t)r * D + d] = v;
  }
  __syncthreads();
  const float *xs = xsh;
  float s = 0.0f, s16 = 0.0f;
  if (lane == 0) {
    for (int d = 0; d < D; ++d) s = s + xs[d] * xs[d];  // sqnorms_kernel's order (filter.hip)
    a.rsq[r] = s;
    if (isfinite(s)) atomicMax(a.rmax, score_key(s));
    else a.rmax[1] = 1u;
    if (a.norms) a.norms[r] = em_norm(Lin{xs}, D);  // norms_slots_kernel: the reference ComputeNorm
    if (a.h16 && a.center) {  // resid_sq_kernel (tiles16.hip)
      for (int d = 0; d < D; ++d) {
        const float v = xs[d] - a.center[d];
        s16 += v * v;
      }
      a.rsq16[r] = s16;
      if (isfinite(s16)) atomicMax(a.rmax_r, score_key(s16));
    }
    a.labels[r] = a.x ? a.labs[i] : inl.lab[i];
    a.live[r] = 1;
    if (a.q8ok) a.q8ok[r] = 0;
  }
  if (!a.h16) return;
  // encode16_kernel + meta16_kernel (tiles16.hip) for this row
  const float rn = __shfl(a.center ? s16 : s, 0);
  const bool special = !isfinite(rn);
  const int G = a.dp / 8;
  for (int g = lane; g < G; g += 64) {
    _Float16 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * g + j;
      v[j] = special || d >= D ? (_Float16)0.0f : (_Float16)((a.center ? xs[d] - a.center[d] : xs[d]) * a.sx);
    }
    const size_t off = (((size_t)(r >> 5) * (a.dp / 16) + (g >> 1)) * 2 + (g & 1)) * 32 + (r & 31);
    _Float16 *o = a.h16 + off * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j];
  }
  if (lane == 0) {
    const float mt = isnan(rn) ? -INFINITY : isinf(rn) ? INFINITY : (a.met16 == L2 ? -rn : 0.0f);
    a.meta[r] = mt;
    if (a.mub) {  // row_terms_kernel (sample16.hip) for this row
      float v = fmaf(a.mkr, rn, mt);
      if (a.mmet == IP) v = fmaf(a.mkx, s, v);
      a.mub[r] = v;
    }
  }
}

__global__ __launch_bounds__(256) void live_sums_kernel(const float *rows, const uint8_t *live, int64_t n, int D,
                                                        double *sums, unsigned long long *count) {
  // block b: rows [b * 256, b * 256 + 256); thread d < D sums dimension d over the block's live rows
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int64_t r1 = min(n, r0 + 256);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    double acc = 0.0;
    for (int64_t r = r0; r < r1; ++r)
      if (live[r]) {
        const float v = rows[blk_off(r, d, D)];
        if (isfinite(v)) acc += (double)v;
      }
    if (acc != 0.0) atomicAdd(sums + d, acc);
  }
  if (threadIdx.x == 0) {
    unsigned long long c = 0;
    for (int64_t r = r0; r < r1; ++r) c += live[r] ? 1ull : 0ull;
    if (c) atomicAdd(count, c);
  }
}
}  // namespace

void launch_write_small(const SmallWriteArgs &a, hipStream_t st, const SmallWriteRows *rows) {
  if (a.cnt <= 0) return;
  static const SmallWriteRows none{};
  hipLaunchKernelGGL(write_small_kernel, dim3((unsigned)a.cnt), dim3(64), 0, st, a, rows ? *rows : none);
}
void launch_live_sums(const float *rows, const uint8_t *live, int64_t n, int32_t dim, double *sums,
                      unsigned long long *count, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(live_sums_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, live, n, dim, sums, count);
}

void launch_norms_slots(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(norms_slots_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, slots, n, dim, out);
}
void launch_fill_results(float *s, int64_t *l, int32_t *c, int64_t nq, int32_t k, hipStream_t st) {
  const int64_t n = nq * (k > 1 ? k : 1) > nq ? nq * (k > 1 ? k : 1) : nq;
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_results_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, s, l, c, nq, k);
}

void WordFill::add(void *ptr, int64_t words, uint32_t value) {
  if (!ptr || words <= 0) return;
  if (cnt == MAXR) throw std::invalid_argument("WordFill: more than 8 ranges");
  p[cnt] = static_cast<uint32_t *>(ptr);
  n[cnt] = words;
  v[cnt] = value;
  ++cnt;
}

void launch_fill_words(const WordFill &f, hipStream_t st) {
  int64_t tot = 0;
  for (int r = 0; r < f.cnt; ++r) tot += f.n[r];
  if (tot <= 0) return;
  hipLaunchKernelGGL(fill_words_kernel, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 1024)), dim3(256), 0, st,
                     f);
}

void launch_merge_two(const float *as, const int64_t *al, const int32_t *ca, const float *bs, const int64_t *bl,
                      const int32_t *cb, int64_t nq, int k, float *out_s, int64_t *out_l, int32_t *out_c,
                      hipStream_t st) {
  if (nq <= 0 || k <= 0) return;
  if (k > 256) throw std::invalid_argument("merge_two: k > 256");
  hipLaunchKernelGGL(merge_two_kernel, dim3(nblk(nq, 128)), dim3(128), 0, st, as, al, ca, bs, bl, cb, nq, k, out_s,
                     out_l, out_c);
}

void launch_list_ids(const int32_t *lb, const int32_t *le, int nlist, int32_t *out, hipStream_t st) {
  if (nlist <= 0) return;
  hipLaunchKernelGGL(list_ids_kernel, dim3((unsigned)nlist), dim3(256), 0, st, lb, le, out);
}

void launch_copy_words(void *dst, const void *src, int64_t words, hipStream_t st) {
  if (words <= 0) return;
  hipLaunchKernelGGL(copy_words_kernel, dim3((unsigned)std::min<int64_t>((words + 255) / 256, 4096)), dim3(256), 0, st,
                     static_cast<uint32_t *>(dst), static_cast<const uint32_t *>(src), words);
}

void fill_u8(uint8_t *p, uint8_t v, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_u8_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, p, v, n);
}

int64_t ivf_rerun_part_keys(int64_t max_fail, int nprobe, int k) {
  return (int64_t)k * std::max<int64_t>(max_fail * nprobe, 2 * RR_UNITS);
}

void launch_ivf_exact_rerun(const IvfRerunArgs &a, int metric, int64_t max_fail, uint64_t *part, hipStream_t st) {
  if (max_fail <= 0 || a.k <= 0 || a.k > 64 || a.nprobe <= 0 || a.nchunk <= 0) return;
  const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(max_fail * a.nprobe, 2 * RR_UNITS), 2048);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, a, part); };
  auto by_dim = [&](auto k32, auto k64, auto k128, auto k0) {
    switch (a.dim) {
      case 32: go(k32); break;
      case 64: go(k64); break;
      case 128: go(k128); break;
      default: go(k0); break;
    }
  };
  if (a.v4 && metric == L2)
    go(ivf_rerun_scan_kernel<L2, 0, 4>);
  else if (a.v4 && metric == IP)
    go(ivf_rerun_scan_kernel<IP, 0, 4>);
  else if (a.v4 && metric == COS)
    go(ivf_rerun_scan_kernel<COS, 0, 4>);
  else if (metric == L2)
    by_dim(ivf_rerun_scan_kernel<L2, 32>, ivf_rerun_scan_kernel<L2, 64>, ivf_rerun_scan_kernel<L2, 128>,
           ivf_rerun_scan_kernel<L2, 0>);
  else if (metric == IP)
    by_dim(ivf_rerun_scan_kernel<IP, 32>, ivf_rerun_scan_kernel<IP, 64>, ivf_rerun_scan_kernel<IP, 128>,
           ivf_rerun_scan_kernel<IP, 0>);
  else
    by_dim(ivf_rerun_scan_kernel<COS, 32>, ivf_rerun_scan_kernel<COS, 64>, ivf_rerun_scan_kernel<COS, 128>,
           ivf_rerun_scan_kernel<COS, 0>);
  if (!a.done)
    hipLaunchKernelGGL(ivf_rerun_merge_kernel, dim3((unsigned)std::min<int64_t>((max_fail + 3) / 4, 256)), dim3(256),
                       0, st, a, part);
}

}  // namespace pyr
