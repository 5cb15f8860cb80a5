// filter.hip -- MFMA candidate filter + exact refine for the FLAT / IVF-Flat scans (gfx950).
//
// The reference's scores are fixed fp32 operation sequences (VectorMath.cs): sub, mul,
// add per element, 8-lane Vector accumulators and a horizontal tree.  Those can only be
// reproduced on the VALU (3 instructions per element, kernels.hip scan_fast).  This file
// gets the same answers at matrix-core rate:
//
//   1. mfma_filter: for every (query, row) pair of a work item an APPROXIMATE score from
//      fp32 MFMA (v_mfma_f32_32x32x2_f32): L2 -> 2 q.x - |x|^2 (the per-query constant
//      -|q|^2 is added later), IP -> q.x.  Each (query, slot) keeps its top-K1 (K1 = k +
//      margin) by approximate score, with the same shared per-query bound machinery as
//      the exact scan (ScanArgs::gthr).
//   2. the partial lists are merged (merge_keys_kernel) into each query's top-K1 by
//      approximate score; s~_K1 = the K1-th approximate score.
//   3. refine_kernel: exact reference scores of the K1 candidates (the same restatement
//      as the exact scan and the oracle), top-k by (score desc, key asc), and a
//      certificate: every row outside the candidate set has approximate score <= s~_K1,
//      and |approx - reference| <= E(q) for every row (fp32 error bounds, see
//      refine_kernel), so if the k-th exact candidate score is > s~_K1 + E no excluded
//      row can be in the top-k and the result equals the exact scan's.  Queries whose
//      certificate fails are listed and re-run through the exact scan by the engine.
//
// So the returned ids and scores stay bit-identical to the CPU restatement; only the
// work per pair moves from 3 VALU instructions per dimension to fp32 MFMA.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace pyr {
namespace {

typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bool better(float s1, uint32_t k1, float s2, uint32_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

__device__ __forceinline__ size_t blk_off(int64_t r, int d, int D) {
  return ((size_t)(r >> 3) * (size_t)D + (size_t)d) * 8 + (size_t)(r & 7);
}

constexpr int RT = 32;       // rows per stage (one 32x32 MFMA tile per wave)
constexpr int SCR = RT + 4;  // score-transpose row stride (floats)
constexpr int CB = 16;       // candidate buffer entries per owner
constexpr int CBS = CB + 1;  // buffer stride (odd: the owners' appends hit distinct banks)

// LDS layout of mfma_filter.  fp32 mode: [2 buffers][RT][RSTR] floats.  bf16x3 mode:
// [2 buffers][hi, lo][RT][BSTR] bf16 (BSTR = D + 8: the 16-byte row pad makes the
// ds_read_b128 B fragments conflict-free); then the score transpose [4][32][SCR] and the
// owners' candidate buffers (scores [128][CB], keys [128][CB]).
template <int D, bool BF, int NW = 4>
struct FilterLds {
  static constexpr int RSTR = D + 4;      // padded row stride: conflict-free ds_read_b128 / ds_write_b32
  static constexpr int BSTR = D + 8;      // bf16 row stride
  static constexpr int TILE = BF ? RT * BSTR : RT * RSTR;  // floats per fp32 tile / bf16 per hi or lo tile
  static constexpr size_t tiles_bytes() { return BF ? sizeof(uint16_t) * 4 * TILE : sizeof(float) * 2 * TILE; }
  static constexpr size_t bytes() { return tiles_bytes() + sizeof(float) * NW * 32 * SCR + 8 * NW * 32 * CBS; }
};

// ---------------------------------------------------------------------------
// mfma_filter: one work item (ScanItem) = up to 128 queries x a row range.  Wave w owns
// queries 32w..32w+31 of the item; its A operand (the queries) stays in registers for the
// whole item: lane l holds query (l & 31), dims [(l >> 5) * D/2, (l >> 5) * D/2 + D/2).
// Rows stream HBM -> registers -> LDS (row-major, padded) 32 at a time, double buffered.
// Per stage each wave runs D/2 MFMAs of 32x32x2 (C[query][row] += 2 dims per step; the
// two lane halves split the dimension range), then moves its C tile through a
// wave-private LDS transpose so that lane i (< 32) sees query i's 32 row scores, filters
// them against the query's K1-th best / shared bound and inserts survivors into the
// query's LDS list.
// ---------------------------------------------------------------------------
// Insert (v, key) into a register-resident sorted (desc) list of compile-time length KR:
// a branch-free compare-and-shift network (no LDS round trips; the owner lanes of a wave
// run it together whenever any of them has a candidate, so it must be cheap).
template <int KR>
__device__ __forceinline__ void reg_insert(float (&s)[KR], uint32_t (&kk)[KR], float v, uint32_t key) {
  bool b[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) b[j] = better(v, key, s[j], kk[j]);  // monotone: false..false true..true
#pragma unroll
  for (int j = KR - 1; j >= 1; --j) {
    s[j] = b[j - 1] ? s[j - 1] : (b[j] ? v : s[j]);
    kk[j] = b[j - 1] ? kk[j - 1] : (b[j] ? key : kk[j]);
  }
  s[0] = b[0] ? v : s[0];
  kk[0] = b[0] ? key : kk[0];
}

// BF = bf16x3 mode: q.x as qh.xh + qh.xl + ql.xh on v_mfma_f32_32x32x16_bf16, where
// q = qh + ql (+ |eps| <= 2^-16 |q|) is the two-term bf16 split of each fp32 value (x
// likewise, split once per block while staging rows into LDS).  Relative error per
// product <= 3.1 * 2^-16 plus fp32 accumulation over 3D terms; refine_kernel's c_bf term
// covers it, so the certified results stay exact.  5.3x the fp32 MFMA rate.
// NW = waves per block (32 queries each): 4 (two blocks per CU) or 8 (one block per CU,
// every staged row tile serves 256 queries: half the HBM / L2 row traffic of NW = 4).
template <int D, int MET, bool IVF, int KR, bool BF, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void mfma_filter(FilterArgs a) {
  using L = FilterLds<D, BF, NW>;
  constexpr int NT = 64 * NW;  // threads per block
  static_assert(NW == 4 || (BF && NW == 8), "8-wave blocks only in bf16x3 mode");
  constexpr int KH = D / 2;  // fp32 k-steps: lanes 0-31 take dims [0, KH), lanes 32-63 [KH, D)
  constexpr int KS = D / 16;  // bf16 k-steps: lane half h takes dims 16s + 8h .. +7 of step s
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // XCD-major item mapping (a.xcd; grid a multiple of 8): block b runs on XCD b % 8, so
  // giving each XCD a contiguous run of items puts a list chunk's query groups (adjacent
  // items) on one XCD at about the same time -- the later groups read the rows from its L2
  int item = blockIdx.x;
  if (a.xcd) {
    const int per = (*a.n_items + 7) >> 3;
    item = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
    if ((int)(blockIdx.x >> 3) >= per) return;
  }
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  float *rt = smem;                                          // fp32: [2][RT][RSTR]
  uint16_t *bt = reinterpret_cast<uint16_t *>(smem);         // bf16: [2][hi, lo][RT][BSTR]
  // a.single (bf16x3): one row-tile buffer (two barriers per stage) so that three blocks fit a CU
  const bool single = BF && a.single;
  float *scw = smem + (single ? L::tiles_bytes() / 2 : L::tiles_bytes()) / sizeof(float);  // [NW][32][SCR]

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int i32 = lane & 31, h = lane >> 5;
  float *sc = scw + w * 32 * SCR;

  // A operand, bf16x3 mode: query 32w + i32, split into hi / lo fragments per k-step
  bf8v qh[BF ? KS : 1], ql[BF ? KS : 1];
  if constexpr (BF) {
    const int i = 32 * w + i32;
    const int qi = i < it.qcnt ? (IVF ? a.qlist[it.qbeg + i] / a.nparts : it.qbeg + i) : -1;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float v[8];
      if (qi >= 0) {
        const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)qi * D + 16 * s + 8 * h);
        const float4 v0 = qp[0], v1 = qp[1];
        v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
        v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.0f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        qh[s][j] = (__bf16)v[j];
        ql[s][j] = (__bf16)(v[j] - (float)qh[s][j]);
      }
    }
  }
  // A operand, fp32 mode: query 32w + i32 of the item, dims h*KH .. h*KH + KH - 1
  float qa[BF ? 1 : KH];
  if constexpr (!BF) {
    const int i = 32 * w + i32;
    if (i < it.qcnt) {
      const int qi = IVF ? a.qlist[it.qbeg + i] / a.nparts : it.qbeg + i;
      const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)qi * D + h * KH);
#pragma unroll
      for (int p = 0; p < KH / 4; ++p) {
        const float4 v = qp[p];
        qa[4 * p] = v.x;
        qa[4 * p + 1] = v.y;
        qa[4 * p + 2] = v.z;
        qa[4 * p + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < KH; ++s) qa[s] = 0.0f;
    }
  }
  const bool wave_active = 32 * w < it.qcnt;

  // owners: lane i32 of wave w (lower half) owns query 32w + i32
  const int oq = 32 * w + i32;
  const bool owner = h == 0 && oq < it.qcnt;
  int oslot = 0, qown = 0;
  float gs = -INFINITY;
  uint32_t published = 0;
  if (owner) {
    oslot = IVF ? a.qlist[it.qbeg + oq] + it.part : (it.qbeg + oq) * a.nparts + it.part;
    qown = IVF ? a.qlist[it.qbeg + oq] / a.nparts : it.qbeg + oq;
    if (a.gthr) gs = key_score(__hip_atomic_load(a.gthr + qown, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  // this owner's candidate buffer (scores, keys) in LDS, nbuf entries
  float *bs = scw + NW * 32 * SCR + (w * 32 + i32) * CBS;
  uint32_t *bk = reinterpret_cast<uint32_t *>(scw + NW * 32 * SCR + NW * 32 * CBS) + (w * 32 + i32) * CBS;
  int nbuf = 0;
  float ts[KR];  // this owner's top-KR by approximate score, sorted desc; (-inf, NONE) = empty
  uint32_t tk[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) {
    ts[j] = -INFINITY;
    tk[j] = KEY_NONE;
  }

  // stage staging: RT rows of the blocked store = RT/8 groups of [D][8]; float4 v of a
  // group holds rows (v&1)*4 .. +3 at dim v>>1 (kernels.hip blk_off)
  const int r0 = it.row_begin;  // multiple of 8
  const int nst = (it.row_end - r0 + RT - 1) / RT;
  constexpr int NV = RT * D / 4;  // float4 per stage
  constexpr int LOADS = BF ? 1 : NV / NT;
  static_assert(BF || NV % NT == 0, "stage must split evenly over the block");
  // bf16x3 staging works on float4 pairs (dims 2p, 2p+1 of the same 4 rows: float4 v and
  // v + 2 of a group) so each row's two bf16 halves are written as one 32-bit word
  constexpr int NP = NV / 2;                   // float4 pairs per stage
  constexpr int PL = BF ? (NP + NT - 1) / NT : 1;  // pairs per thread
  const float4 *src = reinterpret_cast<const float4 *>(a.rows);
  const int gmax = ((it.row_end + 7) >> 3) - 1;  // last group with rows of this item
  float4 pf[LOADS];
  float4 pa[PL], pb[PL];
  auto load_stage = [&](int stg) {
    if constexpr (BF) {
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int pr = tid + NT * i;
        if (NP % NT == 0 || pr < NP) {
          const int gl = pr / D, pp = pr % D;
          const int v0 = 4 * (pp >> 1) + (pp & 1);
          const int g = min((r0 >> 3) + stg * (RT / 8) + gl, gmax);  // clamp: rows past the end unused
          pa[i] = src[(size_t)g * (2 * D) + v0];
          pb[i] = src[(size_t)g * (2 * D) + v0 + 2];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LOADS; ++i) {
        const int v = tid + NT * i;
        const int g = min((r0 >> 3) + stg * (RT / 8) + v / (2 * D), gmax);  // clamp: rows past the end unused
        pf[i] = src[(size_t)g * (2 * D) + v % (2 * D)];
      }
    }
  };
  auto split2 = [](float x0, float x1, uint32_t &hi, uint32_t &lo) {
    const __bf16 h0 = (__bf16)x0, h1 = (__bf16)x1;
    const __bf16 l0 = (__bf16)(x0 - (float)h0), l1 = (__bf16)(x1 - (float)h1);
    hi = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    lo = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  };
  auto store_stage = [&](int buf) {
    if constexpr (BF) {
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int pr = tid + NT * i;
        if (NP % NT == 0 || pr < NP) {
          const int gl = pr / D, pp = pr % D;
          const int row = gl * 8 + (pp & 1) * 4;
          uint32_t *dh = reinterpret_cast<uint32_t *>(bt + (2 * buf) * L::TILE + row * L::BSTR + 2 * (pp >> 1));
          uint32_t *dl = dh + L::TILE / 2;
          constexpr int W = L::BSTR / 2;  // row stride in 32-bit words
          uint32_t hi, lo;
          split2(pa[i].x, pb[i].x, hi, lo);
          dh[0] = hi;
          dl[0] = lo;
          split2(pa[i].y, pb[i].y, hi, lo);
          dh[W] = hi;
          dl[W] = lo;
          split2(pa[i].z, pb[i].z, hi, lo);
          dh[2 * W] = hi;
          dl[2 * W] = lo;
          split2(pa[i].w, pb[i].w, hi, lo);
          dh[3 * W] = hi;
          dl[3 * W] = lo;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LOADS; ++i) {
        const int v = tid + NT * i;
        const int gl = v / (2 * D), vv = v % (2 * D);
        float *dst = rt + buf * L::TILE + (gl * 8 + (vv & 1) * 4) * L::RSTR + (vv >> 1);
        dst[0] = pf[i].x;
        dst[L::RSTR] = pf[i].y;
        dst[2 * L::RSTR] = pf[i].z;
        dst[3 * L::RSTR] = pf[i].w;
      }
    }
  };

  // this lane's C column (a row) per stage: visibility and |x|^2 are loaded one stage
  // ahead, with that stage's rows, so the stage that uses them never waits on a load
  // (vmcnt is in order: a load issued behind the row prefetch would drain it)
  uint8_t lv_next = 0;
  float xsq_next = 0.0f;
  auto load_meta = [&](int stg) {
    const int rc = min(r0 + stg * RT + i32, it.row_end - 1);
    lv_next = a.live[rc];
    if (MET == L2) xsq_next = a.rsq[rc];
  };
  if (nst > 0) {
    load_meta(0);
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();

  for (int st = 0; st < nst; ++st) {
    const int cur = single ? 0 : st & 1;
    const int row = r0 + st * RT + i32;
    const bool rvalid = row < it.row_end && (uint32_t)row < a.row_limit && lv_next;
    const float xsq = xsq_next;
    if (st + 1 < nst) {
      load_meta(st + 1);
      if (!(a.ablate & 4)) load_stage(st + 1);
    }
    if (wave_active && !(a.ablate & 8)) {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
      if constexpr (BF) {
        const uint16_t *bh = bt + (2 * cur) * L::TILE + i32 * L::BSTR + 8 * h;
        const uint16_t *bl = bh + L::TILE;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf8v xh = *reinterpret_cast<const bf8v *>(bh + 16 * s);
          const bf8v xl = *reinterpret_cast<const bf8v *>(bl + 16 * s);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql[s], xh, acc, 0, 0, 0);  // small terms first
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh[s], xl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh[s], xh, acc, 0, 0, 0);
        }
      } else {
        const float *bp = rt + cur * L::TILE + i32 * L::RSTR + h * KH;
#pragma unroll
        for (int s4 = 0; s4 < KH / 4; ++s4) {
          const float4 b = *reinterpret_cast<const float4 *>(bp + 4 * s4);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[4 * s4 + 0], b.x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[4 * s4 + 1], b.y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[4 * s4 + 2], b.z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[4 * s4 + 3], b.w, acc, 0, 0, 0);
        }
      }
      // C[i][j]: lane column j = i32 (row), register r -> query (r&3) + 8(r>>2) + 4h
      if (!(a.ablate & 2)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = (r & 3) + 8 * (r >> 2) + 4 * h;
          const float s = MET == L2 ? 2.0f * acc[r] - xsq : acc[r];
          sc[qi * SCR + i32] = rvalid ? s : -INFINITY;
        }
      } else if (acc[0] == 12345.0f) {
        sc[i32] = acc[1];  // keep the MFMAs alive in the ablated build
      }
    }
    if (!single && st + 1 < nst && !(a.ablate & 4)) store_stage(cur ^ 1);
    __syncthreads();  // next tile staged (single: every wave done with this tile); score transpose visible
    if (single && st + 1 < nst && !(a.ablate & 4)) store_stage(0);

    // pre-filter against the owner's bound (the full (score, key) test follows): lane half
    // h tests rows 16h .. 16h + 15 of query i32, the owner joins the two masks
    const float lo = __shfl(fmaxf(gs, ts[KR - 1]), i32);
    uint32_t hmask = 0;
    if (oq < it.qcnt && !(a.ablate & 1)) {
      const float *sch = sc + i32 * SCR + (RT / 2) * h;
#pragma unroll
      for (int j = 0; j < RT / 2; ++j) {
        const float v = sch[j];
        if (v > -INFINITY && v >= lo) hmask |= 1u << j;
      }
    }
    const uint32_t upper = __shfl(hmask, i32 + 32);
    if (owner && !(a.ablate & 1)) {
      const float *scp = sc + i32 * SCR;
      const int rb = r0 + st * RT;
      uint32_t pass = hmask | (upper << (RT / 2));
      if (a.ablate & 16) {  // measurement: filter without inserting
        if (pass == 0x12345u) ts[0] = lo;
        pass = 0;
      }
      if (a.dbg) {  // measurement only
        const uint32_t np = __popc(pass);
        atomicAdd(a.dbg + 1, np);
        atomicAdd(a.dbg + 2, 1u);
        uint32_t mx = np;
        for (int o = 16; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 32));
        if (i32 == 0) atomicAdd(a.dbg, mx);
      }
      // Survivors go to the owner's LDS buffer (cheap appends); the register list is
      // updated only when some owner's buffer would overflow (then every owner of the wave
      // drains its buffer and inserts this stage directly).  The 32 owners run the insert
      // network in lockstep, so draining CB buffered candidates at once costs max-over-owners
      // of the buffered counts instead of a sum over stages of per-stage maxima.
      const bool direct = (a.ablate & 32) || __any(nbuf + __popc(pass) > CB);
      if (direct) {
        for (int i = 0; i < nbuf; ++i) {
          const float v = bs[i];
          const uint32_t key = bk[i];
          if (better(v, key, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, key);
        }
        nbuf = 0;
        while (pass) {
          const int j = __builtin_ctz(pass);
          pass &= pass - 1;
          const float v = scp[j];
          const uint32_t key = a.key_base | (uint32_t)(rb + j);
          if (better(v, key, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, key);
        }
      } else {
        while (pass) {
          const int j = __builtin_ctz(pass);
          pass &= pass - 1;
          bs[nbuf] = scp[j];
          bk[nbuf] = a.key_base | (uint32_t)(rb + j);
          ++nbuf;
        }
      }
      if (a.gthr && (st & a.pub_mask) == a.pub_mask) {  // publish this list's KR-th best, refresh the bound
        if (tk[KR - 1] != KEY_NONE && score_key(ts[KR - 1]) > published) {
          published = score_key(ts[KR - 1]);
          atomicMax(a.gthr + qown, published);
        }
        gs = fmaxf(gs, key_score(__hip_atomic_load(a.gthr + qown, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
      }
    }
    if (single) __syncthreads();  // the next tile is staged
  }
  if (owner) {
    for (int i = 0; i < nbuf; ++i) {  // drain the candidate buffer
      const float v = bs[i];
      const uint32_t key = bk[i];
      if (better(v, key, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, key);
    }
    if (a.gthr && tk[KR - 1] != KEY_NONE && score_key(ts[KR - 1]) > published)
      atomicMax(a.gthr + qown, score_key(ts[KR - 1]));
    float *ps = a.part_s + (size_t)oslot * KR;
    uint32_t *pk = a.part_k + (size_t)oslot * KR;
#pragma unroll
    for (int j = 0; j < KR; ++j) {
      ps[j] = ts[j];
      pk[j] = tk[j];
    }
  }
}

// ---------------------------------------------------------------------------
// Exact restatements (VectorMath.cs) for the refine step -- the operation order of
// kernels.hip em_* and oracle/oracle.c, on one blocked-store row.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float hsum8(const float *v) {
  float lo = (v[0] + v[1]) + (v[2] + v[3]);
  float hi = (v[4] + v[5]) + (v[6] + v[7]);
  return lo + hi;
}

// V = 1: L2Squared (VectorMath.cs:39-70) / DotProduct (:8-37);
// V = 4: L2SquaredUnsafe (:188-253) / DotProductUnsafe (:128-186).  Any D (the tail runs in order).
// (kernels.hip em_* hold the one-lane form; the refine spreads it over 8 lanes, below.)

// hsum8 over the 8 lanes of an aligned lane group, lane l holding v[l]: the same three levels of
// pairwise adds (fp32 adds commute, so every lane of the group ends with the identical value)
__device__ __forceinline__ float hsum8_lanes(float v) {
  v = v + __shfl_xor(v, 1);  // (v0 + v1), (v2 + v3), ...
  v = v + __shfl_xor(v, 2);  // lo = (v0 + v1) + (v2 + v3), hi
  return v + __shfl_xor(v, 4);  // lo + hi
}

// exact_score with its 8 accumulator lanes spread over an 8-lane group: lane l (0..7) runs the
// chains of accumulator l (a1..a4[l] for V = 4, acc[l] for the 8-wide loop), in the same order, and
// the group reduces them as hsum8 does.  Every lane of the group returns the score.
// DT > 0: the dimension as a compile-time constant (every loop unrolls, so all of a row's loads are in
// flight at once; the additions keep their order)
template <int V, int MET, int DT = 0, bool RM = false>
__device__ float exact_score_l8(const float *q, const float *rows, int64_t r, int Dr, int l) {
  const int D = DT > 0 ? DT : Dr;
  constexpr int UNR32 = DT > 0 ? DT / 32 : 1, UNR8 = DT > 0 ? DT / 8 : 4;
  // RM: rows is row-major (a row's dims contiguous: the 8 lanes of a group read 32 B together instead
  // of 8 scattered sectors of the blocked store)
  auto X = [&](int d) { return RM ? rows[(size_t)r * D + d] : rows[blk_off(r, d, D)]; };
  float sum = 0.0f;
  int i = 0;
  if (V == 4 && D >= 32) {
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll UNR32
    for (; i <= D - 32; i += 32)
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const float x = X(i + 8 * v + l);
        float t;
        if (MET == L2) {
          const float d = q[i + 8 * v + l] - x;
          t = d * d;
        } else {
          t = q[i + 8 * v + l] * x;
        }
        a[v] = a[v] + t;
      }
    const float fin = ((a[0] + a[1]) + a[2]) + a[3];
    sum = sum + hsum8_lanes(fin);
  }
  if (i <= D - 8) {
    float acc = 0.0f;
#pragma unroll UNR8
    for (; i <= D - 8; i += 8) {
      const float x = X(i + l);
      if (MET == L2) {
        const float d = q[i + l] - x;
        acc = acc + d * d;
      } else {
        acc = acc + q[i + l] * x;
      }
    }
    sum = sum + hsum8_lanes(acc);
  }
  // the scalar tail (VectorMath.cs:243-250 / :182-185 and the safe forms' remainder loops), in order;
  // every lane of the group adds the same terms
  for (; i < D; ++i) {
    const float x = X(i);
    if (MET == L2) {
      const float d = q[i] - x;
      sum = sum + d * d;
    } else {
      sum = sum + q[i] * x;
    }
  }
  return MET == L2 ? -sum : sum;
}

// One wave per query: lane c < K1 re-scores candidate c exactly, ranks it among the
// candidates by (exact score desc, key asc); lanes with rank < k write the result.
// Certificate (file header), with s~_K1 the merged K1-th approximate score:
//   L2: approx = 2 q.x - |x|^2 - |q|^2,  IP: approx = q.x, and for every row
//   |approx - reference| <= E = c_err * u * (|q| + X)^2   (L2)
//                              c_err * u * |q| * X       (IP)
// with X >= every row norm of the index and u = 2^-24: the fp32 MFMA dot is an fmaf
// chain of D terms (error <= D u sum|q_i x_i| <= D u |q||x|), |x|^2 and |q|^2 are fp32
// sums (<= D u |.|^2 each), one more rounding combines them, and the reference's own
// sum is within (D/8 + 5) u (|q| + |x|)^2 of the real value: < (3.2 D + 6) u (|q|+|x|)^2
// in all, against c_err = 4 D + 64 (engine).  The bf16x3 filter adds c_bf u |q| X
// (kernels.h filter_bf16x3_cerr) and an absolute term for flushed subnormal halves.  If fewer than K1 candidates exist no row
// was excluded and the result is exact as it stands.
template <int V, int MET, int DT>
__global__ __launch_bounds__(256) void refine_kernel(RefineArgs a) {
  const int lane = threadIdx.x & 63;
  int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  if (a.qsel) {  // a device-sized subset (the failures of an earlier certificate): no host round trip
    if (q >= *a.nsel) return;
    q = a.qsel[q];
  }
  const int D = DT > 0 ? DT : a.dim, k1 = a.k1, k = a.k;
  constexpr int UNR8 = DT > 0 ? DT / 8 : 4;
  const int ld = a.ld > 0 ? a.ld : k1;
  const float *qp = a.queries + (size_t)q * D;
  float part = 0.0f;  // |q|^2, any order (covered by E)
  for (int d = lane; d < D; d += 64) part += qp[d] * qp[d];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
  const float qsq = part;
  float qa = 0.0f;  // max |q_i|: the fp16 filter's query scale (filter16.hip pow2_scale)
  if (a.q16) {
    for (int d = lane; d < D; d += 64) qa = fmaxf(qa, fabsf(qp[d]));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) qa = fmaxf(qa, __shfl_xor(qa, off));
  }

  const float *ms = a.ms + (size_t)q * ld;
  const int32_t *mk = a.mk + (size_t)q * ld;
  uint32_t key = KEY_NONE;
  float s = -INFINITY;
  if (lane < k1 && mk[lane] >= 0) key = (uint32_t)mk[lane];
  // exact scores, 8 candidates per pass (an 8-lane group per candidate), then candidate c's score
  // moves to lane c
  for (int p = 0; 8 * p < k1; ++p) {
    const int c = 8 * p + (lane >> 3);
    const int32_t kc = __shfl((int)key, c);  // (k1 <= 64: every candidate's key sits on lane c)
    const int64_t rk = kc >= 0 ? (int64_t)kc : 0;
    float sc;
    if (MET == L2 && a.cosine) {  // VectorMath.Cosine (:102-109) with the cached norms
      const float dot = a.rows_rm ? exact_score_l8<V, IP, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                                  : exact_score_l8<V, IP, DT, false>(qp, a.rows, rk, D, lane & 7);
      const float qn = a.qnorm[q], xn = a.rnorm[rk];
      sc = (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
    } else {
      sc = a.rows_rm ? exact_score_l8<V, MET, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                     : exact_score_l8<V, MET, DT, false>(qp, a.rows, rk, D, lane & 7);
    }
    const float t = __shfl(sc, 8 * (lane & 7));
    if ((lane >> 3) == p && key != KEY_NONE) s = t;
  }
  int rank = 0, valid = 0;
  for (int c = 0; c < k1; ++c) {
    const float sc = __shfl(s, c);
    const uint32_t kc = __shfl(key, c);
    if (kc == KEY_NONE) continue;
    ++valid;
    if (key != KEY_NONE && better(sc, kc, s, key)) ++rank;
  }
  const int nout = min(valid, k);
  if (key != KEY_NONE && rank < k) {
    a.out_s[(size_t)q * k + rank] = s;
    a.out_l[(size_t)q * k + rank] = a.row_labels ? a.row_labels[key] : (int64_t)key;
  }
  if (lane >= nout && lane < k) {
    a.out_s[(size_t)q * k + lane] = -INFINITY;
    a.out_l[(size_t)q * k + lane] = -1;
  }
  bool ok = true;
  // K1 candidates (rows, or a part's floor placeholder KEY_FLOOR = -2 that stands for rows the scan
  // dropped at or below its score): rows were excluded, check the margin against the K1-th score
  if (mk[k1 - 1] != -1) {
    float skth = -INFINITY;
    for (int c = 0; c < k1; ++c) {
      const int rc = __shfl(rank, c);
      const uint32_t kc = __shfl(key, c);
      const float sc = __shfl(s, c);
      if (kc != KEY_NONE && rc == k - 1) skth = sc;
    }
    const double u = 5.9604644775390625e-8;  // 2^-24
    const double qn = sqrt((double)qsq) * (1.0 + 1e-5);
    if (a.resid && a.ub) {
      // upper-bound candidates (stream16.hip, stream_ub_terms): every row left out -- below T_q, a
      // region's floor, or merged below the K1-th -- has a reference score at most the K1-th entry
      if (MET == L2 && a.cosine) {
        // the bounds are L2 scores s of the unit vectors: 1 + s / 2 bounds q^.x^, within (D/2 + 66) u of
        // the real cosine, the reference Cosine within (D/4 + 28) u of it (cos_rerank_kernel)
        const double pk = 1.0 + 0.5 * (double)ms[k1 - 1];
        const float qn = a.qnorm[q];
        ok = nout == k && (double)skth > pk + (2.0 * D + 256.0) * u && qn >= 1e-6f && isfinite(qn) &&
             !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
      } else {
        ok = nout == k && skth > ms[k1 - 1];
      }
      if (lane == 0) {
        if (a.out_c) a.out_c[q] = nout;
        if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
      }
      return;
    }
    if (a.resid) {
      // IVF fp16 filter over residual tiles (filter16.hip, stream16.hip): approx estimates the score
      // itself,  L2: -|q - x|^2 = 2 (q-c).(x-c) - |x-c|^2 - |q-c|^2,  IP: q.x = q.(x-c) + q.c,
      // so for a row of list l its error is relative to the residuals: fp16 rows and queries
      // c_bf u A_l X_l (A_l = |q - c_l| for L2, |q| for IP; X_l = max |x - c_l| over the list), fp32
      // sums / adds (D + 8) u (A_l + X_l)^2, subnormal halves (c_abs A_l, and the query's, below
      // 2^-36 sqrt(D) A_l X_l), IP's q.c constant (D + 8) u |q||c_l|.  The reference's own sum: L2
      // adds non-negative terms, so R = T (1 +- g), g = (D/8 + 8) u; IP |R - T| <= g |q| max|x|.
      // Per list: a probed list none of whose rows can reach skth whatever the filter
      // saw -- L2: |q - c_l| - X_l >= r with r^2 = -skth (1 + 2 c_err u); IP: q.c_l + |q| X_l plus its
      // roundings below skth -- adds no error term; E is the largest term of the other lists.
      const double g = (D / 8.0 + 8.0) * u;
      const double r = sqrt(fmax(0.0, -(double)skth) * (1.0 + 2.0 * a.c_err * u) + 1e-30) * (1.0 + 1e-6);
      double emax = 0.0;
      // FLAT (no probes): one center, list 0
      // 8 probes per pass, an 8-lane group per probe, lane j of it summing dims j, j + 8, ...
      const int np = a.probes ? a.nprobe : 1;
      // probe ids of 64 probes at a time, one per lane, handed to the 8-lane groups by shuffle (no
      // dependent id load inside the passes)
      int pid = 0;
      for (int p0 = 0; p0 < np; p0 += 8) {
        if ((p0 & 63) == 0)
          pid = a.probes && p0 + lane < np ? a.probes[(size_t)q * a.nprobe + p0 + lane] : 0;
        const int p = p0 + (lane >> 3), j = lane & 7;
        const int lp = __shfl(pid, (p0 & 63) + (lane >> 3));
        float d2 = 0.0f, c2 = 0.0f, qc = 0.0f;
        if (p < np) {
          const float *c = a.cents + (size_t)lp * D;
          // the error terms follow the query the filter scored: the unit query for Cosine (qcert)
          const float *qe = a.qcert ? a.qcert + (size_t)q * D : qp;
#pragma unroll UNR8
          for (int d = j; d < D; d += 8) {
            const float t = qe[d] - c[d];
            d2 += t * t;
            c2 += c[d] * c[d];
            qc += qe[d] * c[d];
          }
        }
#pragma unroll
        for (int off = 1; off <= 4; off <<= 1) {
          d2 += __shfl_xor(d2, off);
          c2 += __shfl_xor(c2, off);
          qc += __shfl_xor(qc, off);
        }
        if (p < np) {
          const double Xr = sqrt((double)key_score(a.list_rmax_r[lp])) * (1.0 + 1e-5);
          const double cn = sqrt((double)c2) * (1.0 + 1e-5);
          double el = 0.0;
          if (MET == L2) {
            const double Al = sqrt((double)d2) * (1.0 + 1e-5) + 1e-30;
            const double Alo = sqrt((double)d2) * (1.0 - 1e-5);
            // (fp32 |q - c|^2: relative error <= (D + 8) u, far inside the 1e-5 margins)
            if (!a.tri || Alo - Xr < r) {
              const double X = a.tri ? fmin(Xr, Al + r) : Xr;
              el = a.c_bf * u * Al * X + a.c_err * u * (Al + X) * (Al + X) + a.c_abs * Al +
                   2.0 * 1.4551915228366852e-11 * sqrt((double)D) * Al * X;
            }
          } else {
            const double Xf = sqrt((double)key_score(a.list_rmax ? a.list_rmax[lp] : *a.max_rsq)) * (1.0 + 1e-5);
            // every row x of l: q.x <= q.c + |q| X_l; fp32 q.c is within (D + 8) u |q||c| of the real
            // value, the reference's sum within g |q||x|
            const double hi = (double)qc + qn * Xr + (g + a.c_err * u) * qn * (cn + Xr + Xf);
            if (!a.tri || hi >= (double)skth)
              el = a.c_bf * u * qn * Xr + a.c_err * u * qn * Xr + a.c_abs * qn +
                   1.4551915228366852e-11 * sqrt((double)D) * qn * Xr + a.c_err * u * qn * cn + g * qn * Xf;
          }
          emax = fmax(emax, el);
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) emax = fmax(emax, __shfl_xor(emax, off));
      const double ak = (double)ms[k1 - 1];
      if (MET == L2 && a.cosine) {
        // unit-row L2 approximations (FlatIndex::search_cosine): a row left out has -|q^ - x^|^2 <= ak + emax
        // (real arithmetic), so q^.x^ <= 1 + (ak + emax) / 2, within (D/4 + 28) u of its cosine; the
        // reference Cosine within (D/4 + 28) u of that (cos_rerank_kernel)
        const float qn = a.qnorm[q];
        ok = nout == k && (double)skth > 1.0 + 0.5 * (ak + emax) + (2.0 * D + 256.0) * u && qn >= 1e-6f &&
             isfinite(qn) && !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
      } else if (MET == L2) {
        ok = nout == k && (double)skth > (ak + emax) + g * fabs(ak + emax);
      } else {
        ok = nout == k && (double)skth > ak + emax;
      }
      if (lane == 0) {
        if (a.out_c) a.out_c[q] = nout;
        if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
      }
      return;
    }
    // X bounds the norm of every row this query's scan could have excluded: the largest |x|^2
    // of its probed lists (IVF), else of the whole store
    uint32_t xk = 0;
    if (a.list_rmax) {
      for (int p = lane; p < a.nprobe; p += 64) xk = max(xk, a.list_rmax[a.probes[(size_t)q * a.nprobe + p]]);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) xk = max(xk, (uint32_t)__shfl_xor((int)xk, off));
    } else {
      xk = *a.max_rsq;
    }
    double X = sqrt((double)key_score(xk)) * (1.0 + 1e-5);
    if (MET == L2 && a.tri) {
      // Rows far from the query cannot reach skth whatever the filter saw: the reference's L2 sum
      // adds non-negative terms, so its value is |q - x|^2 (1 +- 22u) (D <= 128; c_err u is far
      // above that), and |q - x| >= |x| - |q|.  A row with |x| >= |q| + r, r^2 = -skth (1 + 2 c_err u),
      // therefore scores below skth; only rows with |x| < |q| + r need the error bound, so X may
      // be lowered to |q| + r (one large-norm outlier in a probed list then costs nothing).
      const double r = sqrt(fmax(0.0, -(double)skth) * (1.0 + 2.0 * a.c_err * u) + 1e-30) * (1.0 + 1e-6);
      X = fmin(X, qn + r);
    }
    double e = (MET == L2 ? a.c_err * u * (qn + X) * (qn + X) : a.c_err * u * qn * X) +
                     a.c_bf * u * qn * X + (a.c_bf > 0.0 ? 1e-30 * (1.0 + qn + X) * D : 0.0);  // bf16 subnormals
    if (a.q16) {
      // fp16 filter: the rows' subnormal halves (c_abs |q|) and the query's, 2^-25 sqrt(D) X / sq
      double sqs = 1.0;
      if (qa > 0.0f && isfinite(qa)) {
        int ex;
        frexp((double)qa, &ex);
        sqs = ldexp(1.0, 14 - ex);
      }
      e += a.c_abs * qn + (MET == L2 ? 2.0 : 1.0) * 2.9802322387695312e-08 * sqrt((double)D) * X / sqs;
    }
    const double approx_k1 = MET == L2 ? (double)ms[k1 - 1] - (double)qsq : (double)ms[k1 - 1];
    ok = nout == k && (double)skth > approx_k1 + e;
    if (!a.q16 && a.max_rsq && a.max_rsq[1] != 0u) ok = false;  // a non-finite row the filter cannot score
  }
  if (lane == 0) {
    if (a.out_c) a.out_c[q] = nout;
    if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
  }
}

// ---- Cosine on the filter path (BruteForceVectorIndex.cs:354) ----
// The candidates come from an exact L2 search of the unit queries q^ = q * (1 / |q|) over the unit rows
// x^ (an L2 FLAT index over the same slots, its labels = the slots; its fp16 tiles are centred on the
// unit rows' mean, so the filter's error is relative to the residuals).  On unit vectors the L2 order
// is the cosine order: 1 - |q^ - x^|^2 / 2 = q^.x^.  Its scores s_j = -L2SquaredUnsafe(q^, x^) are
// exact, so p_j = 1 + s_j / 2 <= p_K2 for every row left out.  With cos_j the real-arithmetic cosine
// and u = 2^-24:
//   ComputeNorm (VectorMath.cs:72-99) sums non-negative squares in 8 lanes of D/8 terms, a 3-level
//   tree and a scalar tail: relative error <= (D/8 + 8) u, so the norm's <= (D/16 + 5) u, and a unit
//   component x_i * fl(1 / |x|) is within e = (D/16 + 7) u of x_i / |x|;
//   |q^|^2, |x^|^2 are within 2e of 1 and q^.x^ within 2e of cos_j, so 1 - |q^ - x^|^2 / 2 is within
//   4e of cos_j; L2SquaredUnsafe adds non-negative terms (4 x 8 lanes, trees, tails): relative error
//   <= (D/8 + 18) u of a distance <= 4.1, i.e. (D/4 + 37) u in p;  |p_j - cos_j| <= (D/2 + 66) u;
//   the reference Cosine dot / (|q| |x|) (DotProductUnsafe, within (D/8 + 16) u sum |q_i x_i|) is
//   within (D/4 + 28) u of cos_j.
// A row left out therefore has a reference score <= p_K2 + (3D/4 + 94) u, and the exact top-k of the
// candidates is the search's when the k-th exact score exceeds p_K2 + E, E = (2D + 256) u.  A row with
// a norm below 1e-6 scores 0 (VectorMath.cs:105) but sits at unit distance (x^ = 0): once the store has
// held such a row (zflag) the k-th score must also exceed 0.  A query with a zero or non-finite norm,
// or a store holding a non-finite row, fails the certificate.
template <int DT>
__global__ __launch_bounds__(256) void cos_rerank_kernel(CosRerankArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  const int D = DT > 0 ? DT : a.dim, kc = a.kc, k = a.k;
  const float *qp = a.queries + (size_t)q * D;
  const float qn = a.qnorm[q];
  const int ccount = a.cand_c[q];
  uint32_t key = KEY_NONE;
  if (lane < kc && lane < ccount && a.cand_l[(size_t)q * kc + lane] >= 0) key = (uint32_t)a.cand_l[(size_t)q * kc + lane];
  float s = -INFINITY;
  for (int p = 0; 8 * p < kc; ++p) {
    const int c = 8 * p + (lane >> 3);
    const int32_t kk = __shfl((int)key, c);
    const int64_t rk = kk >= 0 ? (int64_t)kk : 0;
    const float dot = a.rows_rm ? exact_score_l8<4, IP, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                                : exact_score_l8<4, IP, DT, false>(qp, a.rows, rk, D, lane & 7);
    const float xn = a.rnorm[rk];
    const float sc = (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
    const float t = __shfl(sc, 8 * (lane & 7));
    if ((lane >> 3) == p && key != KEY_NONE) s = t;
  }
  int rank = 0, valid = 0;
  for (int c = 0; c < kc; ++c) {
    const float sc = __shfl(s, c);
    const uint32_t kk = __shfl(key, c);
    if (kk == KEY_NONE) continue;
    ++valid;
    if (key != KEY_NONE && better(sc, kk, s, key)) ++rank;
  }
  const int nout = min(valid, k);
  if (key != KEY_NONE && rank < k) {
    a.out_s[(size_t)q * k + rank] = s;
    a.out_l[(size_t)q * k + rank] = a.row_labels[key];
  }
  if (lane >= nout && lane < k) {
    a.out_s[(size_t)q * k + lane] = -INFINITY;
    a.out_l[(size_t)q * k + lane] = -1;
  }
  bool ok = true;
  if (ccount >= kc) {  // rows were left out: the margin against the K2-th inner product
    float skth = -INFINITY;
    for (int c = 0; c < kc; ++c) {
      const int rc = __shfl(rank, c);
      const uint32_t kk = __shfl(key, c);
      const float sc = __shfl(s, c);
      if (kk != KEY_NONE && rc == k - 1) skth = sc;
    }
    const double u = 5.9604644775390625e-8;  // 2^-24
    const double pk = 1.0 + 0.5 * (double)a.cand_s[(size_t)q * kc + kc - 1];
    ok = nout == k && (double)skth > pk + (2.0 * D + 256.0) * u;
    if (a.zflag && *a.zflag != 0u && !(skth > 0.0f)) ok = false;
  }
  if (!(qn >= 1e-6f) || !isfinite(qn) || (a.max_rsq && a.max_rsq[1] != 0u)) ok = false;
  if (lane == 0) {
    if (a.out_c) a.out_c[q] = nout;
    if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
  }
}

// unit vectors: out row i = x_i * (1 / n_i), or 0 when n_i < 1e-6 (the reference's zero-norm rule) or
// n_i is not finite.  blocked: rows of a blocked store at slots[i] (norms indexed by slot), else
// row-major x with norms[i].
__global__ void unit_rows_kernel(const float *x, const int64_t *slots, const float *norms, int64_t n, int D,
                                 float *out, uint32_t *zflag, const uint8_t *live) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / D;
    const int d = (int)(e % D);
    const int64_t r = slots ? slots[i] : i;
    const float nr = norms[r];
    const float v = slots ? x[blk_off(r, d, D)] : x[e];
    const bool unit = nr >= 1e-6f && isfinite(nr);
    out[e] = unit ? v * (1.0f / nr) : 0.0f;
    if (zflag && d == 0 && !unit && (!live || live[r])) *zflag = 1u;
  }
}

// result rows of the exact re-run (sub-batch order) back to their queries
__global__ void scatter_results_kernel(const int32_t *qidx, int64_t n, int k, const float *ss, const int64_t *sl,
                                       const int32_t *sc, float *out_s, int64_t *out_l, int32_t *out_c) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * k) return;
  const int64_t i = e / k;
  const int j = (int)(e % k);
  const int64_t q = qidx[i];
  out_s[q * k + j] = ss[e];
  out_l[q * k + j] = sl[e];
  if (j == 0 && out_c) out_c[q] = sc[i];
}

__global__ void gather_queries_kernel(const float *q, const int32_t *qidx, int64_t n, int D, float *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    out[e] = q[(size_t)qidx[i] * D + e % D];
  }
}

// |x|^2 of blocked rows (slots[i], or i when slots is null) and the running maximum
// (score_key-encoded, only grows) that the refine certificate bounds row norms with
__global__ void sqnorms_kernel(const float *rows, const int64_t *slots, int64_t n, int D, float *out,
                               uint32_t *max_key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots ? slots[i] : i;
  float s = 0.0f;
  for (int d = 0; d < D; ++d) {
    const float x = rows[blk_off(r, d, D)];
    s = s + x * x;
  }
  out[r] = s;
  // a NaN / inf row is left out of the norm bound (one bad row would fail every later certificate);
  // the fp16 tile filters carry it in meta (+inf: always a candidate), the bf16x3 / fp32 filters
  // cannot score it (hi = inf, lo = inf - inf = NaN), so max_key[1] marks the store and their
  // certificate fails
  if (isfinite(s)) atomicMax(max_key, score_key(s));
  else max_key[1] = 1u;
}

// per-list max of |x|^2 (score_key, finite rows only) over rows [lb[l], le[l]): the refine
// certificate of an IVF query bounds row norms over its probed lists only
__global__ __launch_bounds__(256) void list_rmax_kernel(const float *rsq, const int32_t *lb, const int32_t *le,
                                                        int nlist, uint32_t *out) {
  const int l = blockIdx.x;
  if (l >= nlist) return;
  uint32_t m = 0;
  for (int r = lb[l] + (int)threadIdx.x; r < le[l]; r += 256) {
    const float v = rsq[r];
    if (isfinite(v)) m = max(m, score_key(v));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  __shared__ uint32_t wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[l] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

template <int D, int MET, bool IVF, int KR, bool BF, int NW>
void launch_filter_p(const FilterArgs &a, int max_items, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  allow_max_lds(reinterpret_cast<const void *>(&mfma_filter<D, MET, IVF, KR, BF, NW>), attr);
  const size_t lds = FilterLds<D, BF, NW>::bytes() - (BF && a.single ? FilterLds<D, BF, NW>::tiles_bytes() / 2 : 0);
  const int grid = a.xcd ? (max_items + 7) / 8 * 8 : max_items;
  hipLaunchKernelGGL((mfma_filter<D, MET, IVF, KR, BF, NW>), dim3(grid), dim3(64 * NW), lds, st, a);
}

template <int D, int MET, bool IVF, int KR>
void launch_filter_t(const FilterArgs &a, int max_items, hipStream_t st) {
  if (a.prec == FILTER_BF16X3) {
    if (a.waves == 8) launch_filter_p<D, MET, IVF, KR, true, 8>(a, max_items, st);
    else launch_filter_p<D, MET, IVF, KR, true, 4>(a, max_items, st);
  } else {
    launch_filter_p<D, MET, IVF, KR, false, 4>(a, max_items, st);
  }
}

template <int D, int MET, bool IVF>
void launch_filter_k(const FilterArgs &a, int max_items, hipStream_t st) {
  if (a.k1 == 16) launch_filter_t<D, MET, IVF, 16>(a, max_items, st);
  else if (a.k1 == 32) launch_filter_t<D, MET, IVF, 32>(a, max_items, st);
  else launch_filter_t<D, MET, IVF, 64>(a, max_items, st);
}

template <int D>
void launch_filter_d(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  const bool ivf = a.qlist != nullptr;
  if (metric == L2) {
    if (ivf) launch_filter_k<D, L2, true>(a, max_items, st);
    else launch_filter_k<D, L2, false>(a, max_items, st);
  } else {
    if (ivf) launch_filter_k<D, IP, true>(a, max_items, st);
    else launch_filter_k<D, IP, false>(a, max_items, st);
  }
}

}  // namespace

bool filter_supported(int dim, int metric, int k1) {
  if (metric != L2 && metric != IP) return false;
  if (dim != 32 && dim != 64 && dim != 128) return false;
  return k1 == 16 || k1 == 32 || k1 == 64;  // register list capacities (mfma_filter KR)
}

void launch_filter(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  switch (a.dim) {
    case 32: launch_filter_d<32>(a, metric, max_items, st); return;
    case 64: launch_filter_d<64>(a, metric, max_items, st); return;
    default: launch_filter_d<128>(a, metric, max_items, st); return;
  }
}

void launch_cos_rerank(const CosRerankArgs &a, hipStream_t st) {
  if (a.nq <= 0) return;
  const dim3 g(nblk(a.nq, 4)), b(256);
  switch (a.dim) {
    case 32: hipLaunchKernelGGL(cos_rerank_kernel<32>, g, b, 0, st, a); return;
    case 64: hipLaunchKernelGGL(cos_rerank_kernel<64>, g, b, 0, st, a); return;
    case 128: hipLaunchKernelGGL(cos_rerank_kernel<128>, g, b, 0, st, a); return;
    default: hipLaunchKernelGGL(cos_rerank_kernel<0>, g, b, 0, st, a); return;
  }
}

void launch_unit_rows(const float *x, const int64_t *slots, const float *norms, int64_t n, int32_t dim, float *out,
                      hipStream_t st, uint32_t *zflag, const uint8_t *live) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n * dim + 255) / 256, int64_t(1) << 22);
  hipLaunchKernelGGL(unit_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, slots, norms, n, dim, out,
                     zflag, live);
}

void launch_refine(const RefineArgs &a, int metric, int V, hipStream_t st) {
  if (a.nq <= 0) return;
  const dim3 g(nblk(a.nq, 4)), b(256);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, g, b, 0, st, a); };
  // the common dimensions as compile-time constants (fully unrolled row loads), others at run time
  auto by_dim = [&](auto k0, auto k32, auto k64, auto k128) {
    switch (a.dim) {
      case 32: go(k32); return;
      case 64: go(k64); return;
      case 128: go(k128); return;
      default: go(k0); return;
    }
  };
  if (V == 4) {
    if (metric == L2) by_dim(refine_kernel<4, L2, 0>, refine_kernel<4, L2, 32>, refine_kernel<4, L2, 64>, refine_kernel<4, L2, 128>);
    else by_dim(refine_kernel<4, IP, 0>, refine_kernel<4, IP, 32>, refine_kernel<4, IP, 64>, refine_kernel<4, IP, 128>);
  } else {
    if (metric == L2) by_dim(refine_kernel<1, L2, 0>, refine_kernel<1, L2, 32>, refine_kernel<1, L2, 64>, refine_kernel<1, L2, 128>);
    else by_dim(refine_kernel<1, IP, 0>, refine_kernel<1, IP, 32>, refine_kernel<1, IP, 64>, refine_kernel<1, IP, 128>);
  }
}

void launch_gather_queries(const float *q, const int32_t *qidx, int64_t n, int32_t dim, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_queries_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, q, qidx, n, dim, out);
}

void launch_scatter_results(const int32_t *qidx, int64_t n, int32_t k, const float *ss, const int64_t *sl,
                            const int32_t *sc, float *out_s, int64_t *out_l, int32_t *out_c, hipStream_t st) {
  if (n <= 0 || k <= 0) return;
  hipLaunchKernelGGL(scatter_results_kernel, dim3(nblk(n * k, 256)), dim3(256), 0, st, qidx, n, k, ss, sl, sc, out_s,
                     out_l, out_c);
}

void launch_list_rmax(const float *rsq, const int32_t *lb, const int32_t *le, int32_t nlist, uint32_t *out,
                      hipStream_t st) {
  if (nlist <= 0) return;
  hipLaunchKernelGGL(list_rmax_kernel, dim3(nlist), dim3(256), 0, st, rsq, lb, le, nlist, out);
}

void launch_sqnorms(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float *out, uint32_t *max_key,
                    hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sqnorms_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, slots, n, dim, out, max_key);
}

}  // namespace pyr
