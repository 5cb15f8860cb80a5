// scan.hip -- the IVF list scan of round 4: stream-and-emit over fp16 residual tiles on
// v_mfma_f32_32x32x16_f16 (gfx950).
//
// Contract of stream16.hip (approximate scores over the lists' fp16 residual tiles -> every row whose
// bound reaches the query's sampled threshold T_q is emitted -> certified exact refine, filter.hip
// refine_kernel), with three changes measured on the I1 configuration:
//
//  1. sample_kernel: ONE wave per (list, 32-query group).  It prepares the group's query operands
//     itself (q - c or q, a power-of-two scale, fp16; {f, cq + E_pair}), writes them for the main pass,
//     and scores the list's first SAMPLE_TILES tiles with them from registers -- no LDS, no barrier, no
//     per-item query staging.  It replaces sprep_kernel + the sampling launch of the list scan.
//  2. scan_kernel: the MFMA shape 32x32x16.  A 32-row tile is ONE A operand per 16-dim k-step (lane
//     (r, h) holds row r, dims 16s + 8h .. +7: the tile layout is lane-linear for it as it stands), a
//     query group is 32 queries, and the 32 x 32 result leaves lane (r, h) query r's scores of rows
//     8b + 4h + i (b, i < 4): per (tile, group) 8 MFMAs against 8 ds_read_b128 and a 16-value epilogue.
//     16 waves per block (4 per SIMD, <= 128 VGPRs): no prefetch of a wave's next tile (the other 15
//     waves' work hides its load; an L2 prefetch by LDS-DMA measured slower), and tiles are taken from
//     an LDS counter so the waves reach the item's end together.
//  3. Emitted rows are staged in LDS and written to their queries' candidate buffers by the whole block
//     at the item's end: one global atomic per (item, query) reserves the query's run (cand_flush).
//
// Row terms (meta + the row's share of the error bound) come precomputed per store
// (RowStore::row_terms, StreamArgs::mub).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace pyr {
namespace {

#define PYR_STREAM_EMIT
#include "f16util.h"

constexpr int SAMPLE_TILES = 16;       // tiles of a list the sample scores (stream16.hip: 2 x 8 waves)
constexpr int SV = 2 * SAMPLE_TILES;   // sample values per (query, probe): one per (tile, lane half)

// Tile dimensions (scan_tile_dim): dims up to 128 rounded up to 32; 256, 512, 768.  Per tile dimension
// the queries per item (the item's fp16 query operands fill <= 128 KB of LDS) and the waves per block
// (16 while a tile's A operands and a group's B operands fit 128 VGPRs, else 8).
constexpr int tile_dim_of(int dim) {
  return dim <= 0 ? 0 : dim <= 128 ? (dim + 31) / 32 * 32 : dim <= 256 ? 256 : dim <= 512 ? 512 : dim <= 768 ? 768 : 0;
}
constexpr int qmax_of(int D) { return D <= 128 ? 512 : D == 256 ? 256 : D == 512 ? 128 : 64; }
constexpr int nw_of(int D) { return D <= 128 ? 16 : 8; }

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(a, fmaxf(b, c)); }

// dims d0 .. d0 + 7 of a row of `dim` floats; PAD: the row is shorter than the tile dimension, dims past
// it read as zero (the zero-padded tiles' counterpart)
template <bool PAD>
__device__ __forceinline__ void load8(const float *row, int d0, int dim, float (&v)[8]) {
  if constexpr (!PAD) {
    const float4 x = *reinterpret_cast<const float4 *>(row + d0), y = *reinterpret_cast<const float4 *>(row + d0 + 4);
    v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w, v[4] = y.x, v[5] = y.y, v[6] = y.z, v[7] = y.w;
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = d0 + u < dim ? row[d0 + u] : 0.0f;
  }
}

// ---- 1. query operands + sample ----
// Wave (item, g): the item's queries 32g .. 32g + 31 (lane (r, h): query 32g + r, dims 16s + 8h .. +7).
// Sample value (t, h) of a query = the best bound of rows 8b + 4h + i of tile t (distinct rows per value).
// D <= 128: the query's residual stays in registers; larger D: a first pass takes the norms, the operands
// are rebuilt per k-step (no per-lane array of D / 2 values).
template <int D, int MET, bool PAD>
__global__ __launch_bounds__(256) void sample_kernel(StreamArgs a) {
  constexpr int KS = D / 16, TB = 64 * D, QG = qmax_of(D) / 32;
  constexpr bool REG = KS <= 8;
  constexpr int UN = REG ? KS : 2;  // k-step loops: unrolled in the register form, lean otherwise
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int item = unit / QG, g = unit - item * QG;
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  if (it.part != 0 || 32 * g >= it.qcnt) return;  // chunk-0 items cover every (list, query) pair once
  const int qi = min(32 * g + r, it.qcnt - 1);
  const bool own = 32 * g + r < it.qcnt;
  const int pos = it.qbeg + qi;
  const int slot = a.qlist[pos];
  const int q = slot / a.nparts;
  const int dim = a.dim;
  const float *qrow = a.queries + (size_t)q * dim, *crow = a.cents + (size_t)it.list * dim;
  // the residual q - c (L2) or q (IP) of dims 16s + 8h .. +7
  auto resid8 = [&](int s, float (&v)[8]) {
    float qv[8], cv[8];
    load8<PAD>(qrow, 16 * s + 8 * h, dim, qv);
    if (MET == L2) {
      load8<PAD>(crow, 16 * s + 8 * h, dim, cv);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = qv[u] - cv[u];
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = qv[u];
    }
  };
  // its norm terms and max |.|
  float rv[REG ? KS : 1][8];
  float cq = 0.0f, amax = 0.0f, q2 = 0.0f, c2 = 0.0f;
#pragma unroll UN
  for (int s = 0; s < KS; ++s) {
    float v[8];
    resid8(s, v);
    if (MET == IP) {
      float cv[8];
      load8<PAD>(crow, 16 * s + 8 * h, dim, cv);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        cq += v[u] * cv[u];
        q2 += v[u] * v[u];
        c2 += cv[u] * cv[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) cq += v[u] * v[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      amax = fmaxf(amax, fabsf(v[u]));
      if constexpr (REG) rv[s][u] = v[u];
    }
  }
  cq += __shfl_xor(cq, 32);
  amax = fmaxf(amax, __shfl_xor(amax, 32));
  if (MET == IP) {
    q2 += __shfl_xor(q2, 32);
    c2 += __shfl_xor(c2, 32);
  }
  // the pair's share of the error bound (stream_ub_terms), rounded up by the 1e-3 in its constants
  float ep;
  if (MET == L2) {
    ep = a.kq * cq + a.kqa * sqrtf(cq);
  } else {
    const float qn = sqrtf(q2);
    ep = a.kq * q2 + a.kqa * qn + a.kqc * qn * sqrtf(c2);
  }
  const float sq = pow2_scale(amax);
  const float f = (MET == L2 ? 2.0f : 1.0f) / (sq * a.sx);
  const float cqe = (MET == L2 ? -cq : cq) + ep;
  // the fp16 operand of k-step s (exact scaling: a power of two)
  auto operand = [&](int s) -> h8v {
    h8v b;
    if constexpr (REG) {
#pragma unroll
      for (int u = 0; u < 8; ++u) b[u] = (_Float16)(rv[s][u] * sq);
    } else {
      float v[8];
      resid8(s, v);
#pragma unroll
      for (int u = 0; u < 8; ++u) b[u] = (_Float16)(v[u] * sq);
    }
    return b;
  };
  h8v B[REG ? KS : 1];
#pragma unroll UN
  for (int s = 0; s < KS; ++s) {
    const h8v b = operand(s);
    if constexpr (REG) B[s] = b;
    if (own) *reinterpret_cast<h8v *>(a.bq + (size_t)pos * D + 16 * s + 8 * h) = b;
  }
  if (own && h == 0) a.qsc[pos] = make_float2(f, cqe);
  // score the first SAMPLE_TILES tiles of the list with the group (rows as A, the queries as B)
  const int r0 = it.row_begin;
  const int nt = min((it.row_end - r0 + 31) >> 5, SAMPLE_TILES);
  const char *hsrc = reinterpret_cast<const char *>(a.h16);
  float mx[SAMPLE_TILES];
#pragma unroll
  for (int t = 0; t < SAMPLE_TILES; ++t) {
    mx[t] = -INFINITY;
    if (t < nt) {
      const char *tb = hsrc + (size_t)(r0 / 32 + t) * TB + lane * 16;
      const size_t mo = (size_t)(r0 + 32 * t) + 4 * h;
      f4v M[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) M[b] = *reinterpret_cast<const f4v *>(a.mub + mo + 8 * b);
      f16v acc = {};
      if constexpr (REG) {
        h8v A[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) A[s] = *reinterpret_cast<const h8v *>(tb + s * 1024);
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], B[s], acc, 0, 0, 0);
      } else {
#pragma unroll 2
        for (int s = 0; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*reinterpret_cast<const h8v *>(tb + s * 1024), operand(s), acc,
                                                       0, 0, 0);
      }
      const int rt = r0 + 32 * t, rlim = it.row_end;
      float m = -INFINITY;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float y = fmaf(f, acc[4 * b + i], M[b][i]);
          m = rt + 8 * b + 4 * h + i < rlim ? fmaxf(m, y) : m;
        }
      mx[t] = m;
    }
  }
  if (own) {
    float *sp = a.samp + (size_t)(q * a.nprobe + (slot % a.nparts) / a.cmax) * SV + h;
#pragma unroll
    for (int t = 0; t < SAMPLE_TILES; ++t) sp[2 * t] = mx[t] + cqe;
  }
}

// ---- 2. the list scan ----
// AB (measurement only, PYR_FILTER_ABLATE; separate instantiations at D = 128, none of them in the shipped
// kernel): 1 (64) = no emission, 2 (128) = tile stream only (no MFMA), 3 (256) = no emission and every tile
// read from the item's first one (compute without HBM), 4 (1024) = round 4's B schedule, 5 (512) = an L2
// prefetch of the wave's next tile (4-byte LDS-DMA per line; measured slower: 0.94 vs 0.90 ms and FETCH 1.83x
// vs 1.09x the stored bytes at I1, profiles/r4_scan), 7 (2048) = the emission without the 4-row block tests,
// 8 (PYR_STREAM_TIMING) = per-wave cycle buckets into a.tdbg, 9 (4096) = issue priority 1 for half the waves, 11 (8192) =
// round 5's emission staging (one LDS atomic per emitting row position on a block-wide counter)
// SMP: the sample pass on the same kernel (round 5): chunk-0 items only, wave w scores tile w of the list
// (SAMPLE_TILES = 16 = the waves of a block at D <= 128) against every query group, and writes per (query,
// probe) the 2 x 16 values max(f acc + row term) + cq over its lane half's rows -- each the bound of distinct
// rows, as sample16_kernel's -- into samp; no emission.
// LIM: a MaxScans search (a.plim): a row at or past its (query, list) pair's bound is neither sampled nor
// emitted (its own instantiation: the check in the default kernel's emission path cost 4 % of the I1 step,
// 1.175 vs 1.125 ms, profiles/r5_late/maxscans_ab.log)
// cand_flush over per-wave staging regions: wave v's rows are eb[v R, v R + nw[v])
template <int NT, int R, class QID>
__device__ __forceinline__ void cand_flush_waves(const StreamArgs &a, const uint2 *eb, const int *nw, int waves,
                                                 int qcnt, int r0, int *cnt, int *base, QID qid) {
  const int tid = threadIdx.x, tot = waves * R;
  for (int i = tid; i < tot; i += NT)
    if (i % R < nw[i / R]) atomicAdd(&cnt[eb[i].y >> 23], 1);
  __syncthreads();
  for (int i = tid; i < qcnt; i += NT) {
    const int c = cnt[i];
    base[i] = c > 0 ? atomicAdd(a.cand_n + qid(i), c) : 0;
    cnt[i] = 0;
  }
  __syncthreads();
  for (int i = tid; i < tot; i += NT) {
    if (i % R >= nw[i / R]) continue;
    const uint2 e = eb[i];
    const int qi = (int)(e.y >> 23);
    const int slot = base[qi] + atomicAdd(&cnt[qi], 1);
    const int q = qid(qi);
    if (slot < a.cap) a.cand[(size_t)q * a.cap + slot] = make_uint2(e.x, a.key_base | (uint32_t)(r0 + (int)(e.y & 0x7FFFFFu)));
    else atomicMax(a.cand_f + q, score_key(__uint_as_float(e.x)));
  }
}

template <int D, int MET, int AB = 0, bool SMP = false, bool LIM = false>
__global__ __launch_bounds__(64 * nw_of(D), 1) void scan_kernel(StreamArgs a) {
  constexpr int NW = nw_of(D);       // waves per block
  constexpr int KS = D / 16;         // 32x32x16 k-steps
  constexpr int KC = KS < 16 ? KS : 16;  // k-steps of A held in registers at a time (D > 256: chunks)
  constexpr int NC = KS / KC;
  constexpr int TB = 64 * D;         // h16 bytes per 32-row tile
  constexpr int QMAX = qmax_of(D);   // queries per item
  constexpr int NG = QMAX / 32;      // query groups per item
  constexpr int PIECES = NG * KS;
  static_assert(KS % KC == 0 && QMAX <= 512, "tile dimension");
  __shared__ __attribute__((aligned(16))) char bl[PIECES * 1024];
  __shared__ float2 qf[QMAX];        // per query slot: {f, threshold in y = f acc + row term space}
  __shared__ float2 qz[QMAX];        // {cq (score = y + cq), the query as int bits}
  __shared__ int cnt_l[QMAX];        // the item's staged rows per query slot (cand_flush)
  __shared__ int base_l[QMAX];       // and their run in the query's buffer
  __shared__ int eb_n, tnext;
  // the block's items, double-buffered: thread 0 writes the NEXT one (slot par ^ 1) while the block still works on
  // slot par, so no thread can ever read a half-replaced item (or re-read the current one after the switch)
  __shared__ int item_buf[2];
  __shared__ ScanItem it_buf[2];
  __shared__ int ebw_n[NW];          // each wave's staged rows (WP)
  __shared__ uint32_t pf_sink[64];   // the L2 prefetch's LDS-DMA target (never read)
  // the item's emitted rows, staged in the LDS left over: (score bits, query slot << 23 | row offset)
  constexpr int EB = (163840 - (int)sizeof(bl) - QMAX * 24 - 512) / 8;
  __shared__ uint2 eb[EB];
  const uint32_t bl_base = (uint32_t)(size_t)(lds_void *)bl;
  const uint32_t sink = (uint32_t)(size_t)(lds_void *)pf_sink;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const char *hsrc = reinterpret_cast<const char *>(a.h16);
  constexpr bool WP = AB != 11;  // wave-private emission staging (AB 11: the block-wide counter, A/B only)

  // measurement only (AB 8, a.tdbg): per wave, cycles in the prologue, its tiles, the end-of-item barrier and
  // the flush; items taken
  uint64_t tb[5] = {0, 0, 0, 0, 0};
  uint64_t tq = 0;
  auto stamp = [&](int b) {
    if constexpr (AB == 8) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (b >= 0) tb[b] += now - tq;
      tq = now;
    }
  };

  // AB 9 (measurement only): the second half of each SIMD's waves at issue priority 1 (MI355X_MICROARCH.md,
  // two waves per SIMD, item 4)
  if constexpr (AB == 9)
    if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // Thread 0 takes the block's next item (the atomic and the item's load) while the other waves finish their
  // tiles, so the round trips sit inside the end-of-item barrier instead of before each prologue (round 6).
  // The sample pass (a.lioff) takes LISTS from its counter and walks each list's chunk-0 items
  // (lioff[l] .. + ceil(lcnt[l] / lqchunk)), instead of drawing and skipping the other chunks' items.
  const int nit = *a.n_items;
  int sm_l = 0, sm_g = 0, sm_ng = 0;  // (thread 0: the sample pass's current list)
  int par = 0;  // (block-uniform) the current item's slot
  auto fetch = [&](int slot) {
    int nx;
    if (SMP && a.lioff) {
      if (sm_g < sm_ng) {
        nx = a.lioff[sm_l] + sm_g++;
      } else {
        nx = nit;
        for (;;) {
          const int l = atomicAdd(a.work, 1);
          if (l >= a.nlist) break;
          const int c = a.lcnt[l];
          if (c > 0) {
            sm_l = l;
            sm_ng = (c + a.lqchunk - 1) / a.lqchunk;
            sm_g = 1;
            nx = a.lioff[l];
            break;
          }
        }
      }
    } else {
      nx = atomicAdd(a.work, 1);
    }
    item_buf[slot] = nx;
    if (nx < nit) it_buf[slot] = a.items[nx];
  };
  if (tid == 0) fetch(0);
  __syncthreads();
  for (;;) {
    const int item = item_buf[par];
    if (item >= nit) {
      if constexpr (AB == 8)
        if (lane == 0)
          for (int b = 0; b < 5; ++b) atomicAdd(a.tdbg + b, (unsigned long long)tb[b]);
      return;
    }
    // (the compiler may re-read these fields from it_buf[par] at any later point of the item, the flush included:
    // slot par is not rewritten before the NEXT item's fetch -- with one buffer, rewritten by the fetch ahead of the
    // end barrier, such re-reads picked up the next item's rows and misplaced the flushed candidates)
    const ScanItem it = it_buf[par];
    if (SMP && it.part != 0) {  // (block-uniform) chunk-0 items cover every (list, query) pair once
      if (tid == 0) fetch(par ^ 1);
      par ^= 1;
      __syncthreads();
      continue;
    }
    stamp(-1);
    if constexpr (AB == 8) tb[4] += 1;
    const int qcnt = it.qcnt, ng = (qcnt + 31) >> 5;

    // prologue: piece (j, s) = dims 16s + 8h .. +7 of query 32j + r in lane (r, h) (the B layout);
    // an unused slot's threshold is NaN, so no row is ever emitted for it
    {
      const int npc = ng * KS;
      for (int p = w; p < npc; p += NW) {
        const int j = p / KS, s = p - j * KS;
        const int qi = min(32 * j + r, qcnt - 1);
        glds<16>(a.bq + (size_t)(it.qbeg + qi) * D + 16 * s + 8 * h, bl_base + (uint32_t)(p * 1024));
      }
      for (int i = tid; i < ng * 32; i += 64 * NW) {
        float2 v = make_float2(0.0f, __builtin_nanf(""));
        float cqv = 0.0f;
        int o = -1;
        if (i < qcnt) {
          const int pos = it.qbeg + i;
          const int slot = a.qlist[pos];
          const float2 fc = a.qsc[pos];
          const float T = (!SMP && a.thr) ? a.thr[slot / a.nparts] + a.thr_bias : -INFINITY;
          v = make_float2(fc.x, lower_thr(T, fc.y));
          // MaxScans: a pair whose bound is at or before the item's rows has none of them scanned -- its rows never
          // reach the emission test (a low T_q from a small budget would otherwise send most of every other
          // list's tiles down the emission path, to be dropped there)
          if constexpr (LIM && !SMP)
            if (a.plim[pos] <= (uint32_t)it.row_begin) v.y = __builtin_nanf("");
          cqv = fc.y;
          o = SMP ? (slot / a.nparts) * a.nprobe + (slot % a.nparts) / a.cmax : slot / a.nparts;
        }
        qf[i] = v;
        qz[i] = make_float2(cqv, __int_as_float(o));
        cnt_l[i] = 0;
      }
      if (tid == 0) {
        eb_n = 0;
        tnext = NW;  // the waves' first tiles are taken in order
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces landed
      __syncthreads();
      stamp(0);
    }

    const int r0 = it.row_begin;  // multiple of 32
    const int nt = SMP ? min((it.row_end - r0 + 31) >> 5, SAMPLE_TILES) : (it.row_end - r0 + 31) >> 5;
    const int rlim = (int)min((int64_t)it.row_end, (int64_t)a.row_limit);
    const bool stage = it.row_end - r0 < (1 << 23);  // row offsets fit the staged word
    // wave-private staging (round 6): wave w writes rows [w EBW, (w + 1) EBW) of eb, counted in a wave-uniform
    // register -- no LDS atomic and its round trip per emitting row position (scan 0.775 vs 0.80 ms at I1,
    // profiles/r6_scan_ab/scan_ab_2.log); a wave whose region is full writes straight to the query's buffer
    constexpr int EBW = EB / NW;
    int ebc = 0;

    // tile t for lane (r, h): the A fragments and the row terms of rows 8b + 4h .. +3
    auto load = [&](int t, h8v (&A)[KC], f4v (&M)[4]) {
      if constexpr (AB == 3) t = 0;
      const char *tp = hsrc + (size_t)(r0 / 32 + t) * TB + lane * 16;
      if constexpr (NC == 1) {
#pragma unroll
        for (int s = 0; s < KS; ++s) A[s] = *reinterpret_cast<const h8v *>(tp + s * 1024);
      }
      const size_t mo = (size_t)(r0 + 32 * t) + 4 * h;
#pragma unroll
      for (int b = 0; b < 4; ++b) M[b] = *reinterpret_cast<const f4v *>(a.mub + mo + 8 * b);
    };
    auto row_terms = [&](const f4v (&M)[4], int t, float (&mr)[16]) {
      const int rt = r0 + 32 * t;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) mr[4 * b + i] = rt + 8 * b + 4 * h + i < rlim ? M[b][i] : -INFINITY;
    };
    auto read_b = [&](int j, h8v (&B)[KS]) {
      const char *bp = bl + j * KS * 1024 + lane * 16;
#pragma unroll
      for (int s = 0; s < KS; ++s) B[s] = *reinterpret_cast<const h8v *>(bp + s * 1024);
    };
    // a row straight to query slot qi's buffer (staging full, or an item of 2^23+ rows)
    auto put = [&](int qi, float sc, int row) { cand_put(a, __float_as_int(qz[qi].y), sc, a.key_base | (uint32_t)row); };
    // the rare emit branch: per row position e a wave-uniform test (one compare, a scalar branch)
    auto emit_y = [&](const f16v &y, float thr, int qi, int rt) {
      const float cq = qz[qi].x;
      // the staged word of row position e is base + 8 (e >> 2) + (e & 3); the empty asm keeps the compiler
      // from hoisting 16 per-position words out of the group loop (they spilled)
      uint32_t base = ((uint32_t)qi << 23) | (uint32_t)(rt - r0 + 4 * h);
      asm volatile("" : "+v"(base));
      // 4-row blocks first (a block's max, one ballot): an emitting (tile, group) usually holds one row
      // above the threshold, so 4 block tests + 4 row tests instead of 16 row tests
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if constexpr (AB != 7) {  // (AB 7: every row tested, round 4's loop; A/B only)
          const float bm = fmaxf(max3f(y[4 * b], y[4 * b + 1], y[4 * b + 2]), y[4 * b + 3]);
          if (__builtin_amdgcn_ballot_w64(bm >= thr) == 0ull) continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * b + i;
          if constexpr (WP) {
            const bool p = y[e] >= thr &&
                           (!LIM || (uint32_t)(rt + 4 * h + 8 * (e >> 2) + (e & 3)) < a.plim[it.qbeg + qi]);
            const uint64_t m = __builtin_amdgcn_ballot_w64(p);
            if (m == 0ull) continue;
            const int at = ebc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            ebc += (int)__builtin_popcountll(m);
            if (p) {
              const float sc = y[e] + cq;
              const uint32_t word = base + (uint32_t)(8 * (e >> 2) + (e & 3));
              if (stage && at < EBW) eb[w * EBW + at] = make_uint2(__float_as_uint(sc), word);
              else put(qi, sc, r0 + (int)(word & 0x7FFFFFu));
            }
            continue;
          }
          const bool p = y[e] >= thr;
          if (__builtin_amdgcn_ballot_w64(p) == 0ull) continue;
          if (p) {
            // MaxScans: a row at or past the pair's bound is not scanned (the bound read only here, per row)
            if (LIM && (uint32_t)(rt + 4 * h + 8 * (e >> 2) + (e & 3)) >= a.plim[it.qbeg + qi]) continue;
            const float sc = y[e] + cq;
            const uint32_t word = base + (uint32_t)(8 * (e >> 2) + (e & 3));
            const int at = stage ? atomicAdd(&eb_n, 1) : EB;
            if (at < EB) eb[at] = make_uint2(__float_as_uint(sc), word);
            else put(qi, sc, r0 + (int)(word & 0x7FFFFFu));
          }
        }
      }
    };
    // group j's scores y = f acc + row term, in place, and whether any can reach its query's threshold
    auto epi_test = [&](f16v &acc, const float (&mr)[16], const float2 q) -> bool {
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[v] = fmaf(q.x, acc[v], mr[v]);
      float mx = max3f(acc[0], acc[1], acc[2]);
      mx = max3f(mx, acc[3], acc[4]);
      mx = max3f(mx, acc[5], acc[6]);
      mx = max3f(mx, acc[7], acc[8]);
      mx = max3f(mx, acc[9], acc[10]);
      mx = max3f(mx, acc[11], acc[12]);
      mx = max3f(mx, acc[13], acc[14]);
      mx = fmaxf(mx, acc[15]);
      if constexpr (AB == 1 || AB == 3) {
        if (mx == 12345.0f) cnt_l[0] = 1;  // keep the scores live
        return false;
      }
      return __builtin_amdgcn_ballot_w64(mx >= q.y) != 0ull;
    };
    // the wave's next tile and its row terms into L2 (one 4-byte LDS-DMA per 128-byte line)
    auto prefetch = [&](int tpf) {
      const char *tp = hsrc + (size_t)(r0 / 32 + tpf) * TB;
#pragma unroll
      for (int o = 0; o < TB; o += 64 * 128) glds<4>(tp + min(o + lane * 128, TB - 128), sink);
      glds<4>(a.mub + r0 + 32 * tpf + (lane & 31), sink);
    };
    // D > 256: the tile's A operands in chunks of KC k-steps, every group's accumulator live meanwhile
    // (NG <= 4); the chunk's loads are waited for once, the next tile is pulled into L2 after the first
    auto tile_chunked = [&](const float (&mr)[16], int t, int tpf) {
      const int rt = r0 + 32 * t;
      const char *tp = hsrc + (size_t)(r0 / 32 + (AB == 3 ? 0 : t)) * TB + lane * 16;
      f16v acc[NG];
#pragma unroll
      for (int j = 0; j < NG; ++j) acc[j] = (f16v){};
#pragma unroll 1
      for (int c = 0; c < NC; ++c) {
        h8v A[KC];
#pragma unroll
        for (int s = 0; s < KC; ++s) A[s] = *reinterpret_cast<const h8v *>(tp + (c * KC + s) * 1024);
#pragma unroll
        for (int j = 0; j < NG; ++j) {
          if (j < ng) {
            const char *bp = bl + (j * KS + c * KC) * 1024 + lane * 16;
#pragma unroll
            for (int s = 0; s < KC; ++s)
              acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], *reinterpret_cast<const h8v *>(bp + s * 1024),
                                                              acc[j], 0, 0, 0);
          }
        }
        if constexpr (AB == 5)
          if (c == 0 && tpf >= 0) prefetch(tpf);
      }
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        if (j < ng) {
          const float2 q = qf[32 * j + r];
          const bool e = epi_test(acc[j], mr, q);
          if (__builtin_expect(e, 0)) emit_y(acc[j], q.y, 32 * j + r, rt);
        }
      }
    };
    // one tile against every group; tpf >= 0: the wave's next tile, pulled into L2 meanwhile
    auto tile = [&](const h8v (&A)[KC], const float (&mr)[16], int t, int tpf) {
      const int rt = r0 + 32 * t;
      if constexpr (AB == 2) {  // consume the tile without scoring it
        float v = mr[0];
#pragma unroll
        for (int s = 0; s < KS; ++s) v += (float)A[s][0];
        if (v == 12345.0f) cnt_l[0] = 1;
        return;
      }
      for (int j = 0; j < ng; ++j) {
        const float2 q = qf[32 * j + r];
        if constexpr (LIM)  // MaxScans: a group none of whose pairs reaches these rows is not scored
          if (__builtin_amdgcn_ballot_w64(!__builtin_isnan(q.y)) == 0ull) continue;
        h8v bj[KS];
        read_b(j, bj);
        f16v acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], bj[0], (f16v){}, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], bj[s], acc, 0, 0, 0);
        const bool e = epi_test(acc, mr, q);
        if constexpr (AB == 4) {  // round 4 (A/B only, PYR_FILTER_ABLATE=1024): every B read before the chain
          __builtin_amdgcn_sched_group_barrier(0x100, KS + 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
        } else {
          // staged: 4 B reads (+ the group's scalars), then 2 MFMAs per 2 further reads -- at most 4 B
          // operands live (16 VGPRs, not 32): with all 8 live the kernel spilled 11 VGPRs, reloaded
          // (serially) on every emitting (tile, group)
          constexpr int P0 = KS < 4 ? KS : 4, NS = (KS - P0 + 1) / 2;
          __builtin_amdgcn_sched_group_barrier(0x100, P0 + 1, 0);
#pragma unroll
          for (int i = 0; i < NS; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, KS - 2 * NS, 0);
        }
        if constexpr (AB == 5)
          if (j == 0 && tpf >= 0) prefetch(tpf);  // the tile's own loads were waited for: warm L2
        if (__builtin_expect(e, 0)) emit_y(acc, q.y, 32 * j + r, rt);
      }
    };

    if constexpr (SMP) {
      static_assert(NW == SAMPLE_TILES && NC == 1, "the sample mode: one tile per wave, tiles in registers");
      float smx[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) smx[g] = -INFINITY;
      if (w < nt) {  // tile w of the list (nt: the item's tiles; the first SAMPLE_TILES of them)
        h8v A[KC];
        f4v M[4];
        float mr[16];
        load(w, A, M);
        row_terms(M, w, mr);
#pragma unroll
        for (int j = 0; j < NG; ++j) {
          if (j >= ng) break;  // (wave-uniform)
          const float2 q = qf[32 * j + r];
          h8v bj[KS];
          read_b(j, bj);
          f16v acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], bj[0], (f16v){}, 0, 0, 0);
#pragma unroll
          for (int s = 1; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], bj[s], acc, 0, 0, 0);
          float mx = fmaf(q.x, acc[0], mr[0]);
#pragma unroll
          for (int v = 1; v < 16; ++v) mx = fmaxf(mx, fmaf(q.x, acc[v], mr[v]));
          if constexpr (LIM) {  // MaxScans: only the rows before the pair's bound are sampled
            const uint32_t lim = a.plim[it.qbeg + min(32 * j + r, qcnt - 1)];
            const int rt = r0 + 32 * w + 4 * h;
            mx = -INFINITY;
#pragma unroll
            for (int v = 0; v < 16; ++v)
              if ((uint32_t)(rt + 8 * (v >> 2) + (v & 3)) < lim) mx = fmaxf(mx, fmaf(q.x, acc[v], mr[v]));
          }
          smx[j] = mx;
        }
      }
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        if (j >= ng) break;
        const int qi = 32 * j + r;
        if (qi < qcnt) a.samp[(size_t)__float_as_int(qz[qi].y) * SV + 2 * w + h] = smx[j] + qz[qi].x;
      }
      if (tid == 0) fetch(par ^ 1);
      par ^= 1;
      __syncthreads();  // every wave is done with the item's LDS before the next prologue
      continue;
    }
    int t = w;
    while (t < nt) {
      h8v A[KC];
      f4v M[4];
      float mr[16];
      load(t, A, M);
      int tn = 0;
      if (lane == 0) tn = atomicAdd(&tnext, 1);
      tn = __builtin_amdgcn_readfirstlane(tn);
      row_terms(M, t, mr);
      if constexpr (NC == 1) tile(A, mr, t, tn < nt ? tn : -1);
      else tile_chunked(mr, t, tn < nt ? tn : -1);
      t = tn;
    }
    stamp(1);
    if constexpr (WP)
      if (lane == 0) ebw_n[w] = stage ? min(ebc, EBW) : 0;
    if (tid == 0) fetch(par ^ 1);  // the next item, inside the end barrier's wait
    par ^= 1;
    __syncthreads();
    stamp(2);
    if constexpr (WP) {
      cand_flush_waves<64 * NW, EBW>(a, eb, ebw_n, NW, qcnt, r0, cnt_l, base_l,
                                     [&](int i) { return __float_as_int(qz[i].y); });
    } else {
      cand_flush<64 * NW>(a, eb, min(eb_n, EB), qcnt, r0, cnt_l, base_l, [&](int i) { return __float_as_int(qz[i].y); });
    }
    // every wave has placed its rows (the flush reads qz / cnt_l / base_l of this item) before any wave's next
    // prologue rewrites them: with the next item fetched ahead of the end barrier, the loop top no longer holds the
    // barrier that used to separate the two (a wave that ran ahead misplaced a slower wave's rows)
    __syncthreads();
    stamp(3);
  }
}

template <int D, int MET>
void launch_scan_dm(const StreamArgs &a, int max_items, hipStream_t st) {
  const int grid = std::max(1, std::min(max_items, device_cus()));
  const dim3 b(64 * nw_of(D));
  if constexpr (D == 128) {  // the ablations (measurement only) at the I1 dimension
    if (a.ablate & 64) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 1>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 128) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 2>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 256) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 3>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 1024) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 4>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 2048) {  // A/B: the emit loop tests every row (no 4-row block test)
      hipLaunchKernelGGL((scan_kernel<D, MET, 7>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 512) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 5>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.tdbg) {
      hipLaunchKernelGGL((scan_kernel<D, MET, 8>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 8192) {  // A/B: round 5's block-wide emission counter
      hipLaunchKernelGGL((scan_kernel<D, MET, 11>), dim3(grid), b, 0, st, a);
      return;
    }
    if (a.ablate & 4096) {  // A/B: issue priority 1 for waves NW/2 .. NW-1
      hipLaunchKernelGGL((scan_kernel<D, MET, 9>), dim3(grid), b, 0, st, a);
      return;
    }
  }
  if (a.plim) hipLaunchKernelGGL((scan_kernel<D, MET, 0, false, true>), dim3(grid), b, 0, st, a);  // MaxScans
  else hipLaunchKernelGGL((scan_kernel<D, MET>), dim3(grid), b, 0, st, a);
}

template <int D, int MET>
void launch_scan_sample_dm(const StreamArgs &a, int max_items, hipStream_t st) {
  if constexpr (nw_of(D) == SAMPLE_TILES && D / 16 <= 16) {
    const int grid = std::max(1, std::min(max_items, device_cus()));
    if (a.plim) hipLaunchKernelGGL((scan_kernel<D, MET, 0, true, true>), dim3(grid), dim3(64 * nw_of(D)), 0, st, a);
    else hipLaunchKernelGGL((scan_kernel<D, MET, 0, true>), dim3(grid), dim3(64 * nw_of(D)), 0, st, a);
  }
}

template <int D, int MET>
void launch_sample_dm(const StreamArgs &a, int max_items, hipStream_t st) {
  const dim3 grid((unsigned)(((int64_t)max_items * (qmax_of(D) / 32) + 3) / 4));  // 4 waves per block
  if (a.dim == D) hipLaunchKernelGGL((sample_kernel<D, MET, false>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((sample_kernel<D, MET, true>), grid, dim3(256), 0, st, a);
}

// every tile dimension, both metrics
#define PYR_SCAN_BY_DIM(fn)                                                                 \
  switch (dt) {                                                                             \
    case 32: return metric == L2 ? fn<32, L2>(a, max_items, st) : fn<32, IP>(a, max_items, st);    \
    case 64: return metric == L2 ? fn<64, L2>(a, max_items, st) : fn<64, IP>(a, max_items, st);    \
    case 96: return metric == L2 ? fn<96, L2>(a, max_items, st) : fn<96, IP>(a, max_items, st);    \
    case 128: return metric == L2 ? fn<128, L2>(a, max_items, st) : fn<128, IP>(a, max_items, st); \
    case 256: return metric == L2 ? fn<256, L2>(a, max_items, st) : fn<256, IP>(a, max_items, st); \
    case 512: return metric == L2 ? fn<512, L2>(a, max_items, st) : fn<512, IP>(a, max_items, st); \
    case 768: return metric == L2 ? fn<768, L2>(a, max_items, st) : fn<768, IP>(a, max_items, st); \
    default: throw_unsupported(dt);                                                         \
  }

[[noreturn]] void throw_unsupported(int dt) {
  throw std::invalid_argument("stream scan: no tile dimension " + std::to_string(dt));
}

__global__ void chunk_lists_kernel(int32_t *lb, int32_t *le, int nch, int64_t crow, int64_t cutoff, const float *center,
                                   int dim, float *cents) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)nch * dim) return;
  const int c = (int)(e / dim), d = (int)(e - (int64_t)c * dim);
  cents[e] = center ? center[d] : 0.0f;
  if (d == 0) {
    lb[c] = (int32_t)(c * crow);
    le[c] = (int32_t)min(cutoff, (int64_t)(c + 1) * crow);
  }
}
__global__ void iota_rows_kernel(int32_t *out, int64_t rows, int cols) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < rows * cols; e += (int64_t)gridDim.x * blockDim.x)
    out[e] = (int32_t)(e % cols);
}

}  // namespace

void launch_chunk_lists(int32_t *lb, int32_t *le, int nch, int64_t crow, int64_t cutoff, const float *center,
                        int dim, float *cents, hipStream_t st) {
  const int64_t n = (int64_t)nch * dim;
  if (n <= 0) return;
  hipLaunchKernelGGL(chunk_lists_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, lb, le, nch, crow, cutoff,
                     center, dim, cents);
}
void launch_iota_rows(int32_t *out, int64_t rows, int cols, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return;
  hipLaunchKernelGGL(iota_rows_kernel, dim3(gblk(rows * cols)), dim3(256), 0, st, out, rows, cols);
}

int scan_sample_values() { return SV; }
int scan_tile_dim(int dim) { return tile_dim_of(dim); }
int scan_qmax(int dt) { return qmax_of(dt); }
bool scan_supported(int dim, int metric, int k1) {
  return (metric == L2 || metric == IP) && tile_dim_of(dim) > 0 && k1 >= 1 && k1 <= 512;  // (> 64: deep refine)
}

void launch_scan_sample(const StreamArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  const int dt = a.dt > 0 ? a.dt : a.dim;
  PYR_SCAN_BY_DIM(launch_sample_dm)
}

bool scan_sample_mode_supported(int dt) { return nw_of(dt) == SAMPLE_TILES && dt / 16 <= 16; }
void launch_scan_sample_mode(const StreamArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  const int dt = a.dt > 0 ? a.dt : a.dim;
  PYR_SCAN_BY_DIM(launch_scan_sample_dm)
}

void launch_scan_main(const StreamArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  const int dt = a.dt > 0 ? a.dt : a.dim;
  PYR_SCAN_BY_DIM(launch_scan_dm)
}

}  // namespace pyr
