// filter16r.hip -- the fp16 list scan with the ROWS as the MFMA A operand (gfx950).
//
// Same contract as filter16.hip (approximate scores over the store's fp16 row tiles -> per (query,
// part) top-K1 candidates -> merge -> certified exact refine, refine_kernel in filter.hip), shaped
// so that a streamed tile serves every query of its list and no wave waits on another wave's
// candidates (round-2 profile: each list chunk was streamed once per 128-query group and 53 % of
// wave time waited at the tile barrier for the wave with the most LDS appends):
//
//  * One block of NW waves per work item of NW x QG groups of 16 queries (default 8 x 4 = 512): wave w
//    takes groups w, w + NW, ...  Items are (list, row chunk, <= NW x QG x 16 queries; a list's queries split
//    into equal groups), so at the I1 batch every list chunk is one item and is streamed from HBM
//    once per launch.  Tiles go HBM -> LDS by LDS-DMA (glds, f16util.h) into an 8-slot ring, one
//    block barrier per two tiles.
//  * v_mfma_f32_16x16x32_f16 with A = 16 rows of the tile (the h16 fragments filter16w reads as its
//    B operand; the 16x16x32 A and B lane layouts coincide) and B = 16 queries: in the C layout lane
//    (c, g) holds query c of the group and rows 4g .. 4g + 3 of each 16-row half, so a query's
//    scale, residual constant and threshold are lane scalars and its four lanes see disjoint rows.
//  * Candidates stay in the lane: each lane keeps a sorted top-L of (approximate score, row) over the
//    rows it sees, inserted under its own exec mask (no LDS buffers, no owner drains).  Once per item
//    a query's four lane lists are reduced to its top-K1.  A lane whose list filled may have dropped
//    rows scoring at most its L-th entry (the lane's floor); where the largest floor exceeds part of
//    the query's top-K1, those entries are written as (floor, KEY_FLOOR) placeholders: the merge
//    ranks them like rows, so the merged K1-th score bounds every row a part dropped, and the refine
//    skips them when re-scoring.  (With L = 8, a floor reaches the top-k only when one lane saw 9 of
//    a query's best rows in one part.)
//  * Threshold per (query, lane): max(the shared bound, a bound that 16 entries of the query's four
//    lists reach, the lane's own L-th entry), the first two refreshed every RF tiles; the bound of
//    the four lists is published to the shared bound (non-returning atomicMax).
// The approximate score (fp16 residual tiles, query split, per-row meta) and its error bound are
// filter16.hip's unchanged (kernels.h filter_f16_cerr).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <type_traits>

#include "kernels.h"

namespace pyr {
namespace {

#include "f16util.h"

// a bound that at least KR entries of a query's four lane lists (lanes c, c + 16, c + 32, c + 48,
// each sorted descending) reach: every lane holds KR / 4 entries >= its (KR/4 - 1)-th, and, with
// L >= KR / 2, two lanes hold KR entries >= the second largest of their (KR/2 - 1)-th
template <int KR, int L>
__device__ __forceinline__ float quad_bound(const float (&s)[L]) {
  float b = s[KR / 4 - 1];
  b = fminf(b, __shfl_xor(b, 16));
  b = fminf(b, __shfl_xor(b, 32));
  if constexpr (L >= KR / 2) {
    const float v = s[KR / 2 - 1], o = __shfl_xor(v, 16);
    const float hi = fmaxf(v, o), lo = fminf(v, o);
    const float hi2 = __shfl_xor(hi, 32), lo2 = __shfl_xor(lo, 32);
    b = fmaxf(b, fmaxf(fminf(hi, hi2), fmaxf(lo, lo2)));
  }
  if constexpr (L >= KR) {  // one lane alone holds KR entries >= its (KR - 1)-th
    float v = s[KR - 1];
    v = fmaxf(v, __shfl_xor(v, 16));
    v = fmaxf(v, __shfl_xor(v, 32));
    b = fmaxf(b, v);
  }
  return b;
}

// sorted insert of (v, k) into a lane list (v beats the last entry: the caller's condition); ties
// keep the earlier row first (rows reach a lane in increasing order)
template <int L>
__device__ __forceinline__ void lane_insert(float (&s)[L], uint32_t (&k)[L], float v, uint32_t key) {
  bool b[L];
#pragma unroll
  for (int p = 0; p < L; ++p) b[p] = v > s[p];
#pragma unroll
  for (int p = L - 1; p >= 1; --p) {
    s[p] = b[p - 1] ? s[p - 1] : (b[p] ? v : s[p]);
    k[p] = b[p - 1] ? k[p - 1] : (b[p] ? key : k[p]);
  }
  s[0] = b[0] ? v : s[0];
  k[0] = b[0] ? key : k[0];
}

// D: 32 / 64 / 128.  KR: K1.  Q2: two-term fp16 queries (2 MFMAs per k-step).  L: lane list depth.
// NW: waves per block, QG: 16-query groups per wave (NW * QG * 16 queries per item; 4 * NW waves per
// CU at 64 * NW threads: NW = 16 -> 128 VGPRs, NW = 8 -> 256).  NST: ring slots.  STEP: tiles per
// block barrier.  RF: tiles between shared-bound refreshes.
template <int D, int MET, int KR, bool Q2, int L, int NW, int QG, int NST, int STEP, int RF>
__global__ __launch_bounds__(64 * NW, NW / 4) void mfma_filter16r(FilterArgs a) {
  constexpr int TB = 32 * D * 2;    // h16 bytes per 32-row tile
  constexpr int NCH = TB / 1024;    // 1 KiB pieces per tile (2, 4 or 8): waves 0 .. NCH-1 load them
  constexpr int SLOT = TB + 256;    // tile + meta (rows 0-31 twice)
  constexpr int KS = D / 32;        // 16x16x32 k-steps
  static_assert(NCH <= NW, "one piece per wave");
  static_assert(QG >= 1 && QG <= 4, "a lane group g reads back group g % QG's bound");
  static_assert(4 * L >= KR, "four lane lists hold K1 entries");
  static_assert(STEP == 1 || STEP == 2, "tiles per barrier");
  static_assert(NST >= 3 * STEP, "ring too shallow");
  static_assert(RF % STEP == 0 && RF >= NST, "a refresh's reads land before the next one");
  __shared__ __attribute__((aligned(16))) char ring[NST * SLOT];
  __shared__ __attribute__((aligned(16))) uint32_t bounds_l[NW * 64];
  const uint32_t ring_base = (uint32_t)(size_t)(lds_void *)ring;

  // measurement only (a.tdbg, PYR_FILTER_DEBUG=2): wave-cycle buckets [prologue, wait + barrier,
  // refresh + issue, compute, epilogue, total, items, tiles]
  const bool tm = a.tdbg != nullptr;
  unsigned long long t_0 = tm ? __builtin_amdgcn_s_memtime() : 0, t_p = t_0, tb[5] = {0, 0, 0, 0, 0};
  auto mark = [&](int b) {
    if (!tm) return;
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    tb[b] += now - t_p;
    t_p = now;
  };
  int item = blockIdx.x;
  if (a.xcd) {
    const int per = (*a.n_items + 7) >> 3;
    item = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
    if ((int)(blockIdx.x >> 3) >= per) return;
  }
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int c = lane & 15, g = lane >> 4;
  const int ngt = (it.qcnt + 15) >> 4;                        // 16-query groups of the item
  const int ngw = w < ngt ? min(QG, (ngt - w + NW - 1) / NW) : 0;  // this wave's: w, w + NW, ...

  // ---- per group j: query c of group w + NW j; B operand = its dims 32s + 8g .. +7 (scaled, split) ----
  h8v qh[QG][KS], ql[QG][KS];
  float fq[QG], cq[QG], thr[QG], te[QG], gs[QG];
  int qi[QG], oslot[QG];
  bool qv[QG];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    const int qs = 16 * (w + NW * j) + c;
    qv[j] = j < ngw && qs < it.qcnt;
    qi[j] = qv[j] ? (a.qlist ? a.qlist[it.qbeg + qs] / a.nparts : it.qbeg + qs) : -1;
    oslot[j] = qv[j] ? (a.qlist ? a.qlist[it.qbeg + qs] + it.part : (it.qbeg + qs) * a.nparts + it.part) : 0;
    float qx[KS][8];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (qv[j]) {
        const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)qi[j] * D + 32 * s + 8 * g);
        const float4 v0 = qp[0], v1 = qp[1];
        qx[s][0] = v0.x; qx[s][1] = v0.y; qx[s][2] = v0.z; qx[s][3] = v0.w;
        qx[s][4] = v1.x; qx[s][5] = v1.y; qx[s][6] = v1.z; qx[s][7] = v1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) qx[s][e] = 0.0f;
      }
    }
    // residual mode (filter16w): B-side query q - c (L2) or q (IP), constant cq completes the score
    float cc = 0.0f;
    if (a.cents && j < ngw) {
      const float *cp = a.cents + (size_t)it.list * D;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float cv = cp[32 * s + 8 * g + e];
          if (MET == L2) {
            qx[s][e] = qx[s][e] - cv;
            cc += qx[s][e] * qx[s][e];
          } else {
            cc += qx[s][e] * cv;
          }
        }
    }
    cc += __shfl_xor(cc, 16);
    cc += __shfl_xor(cc, 32);
    cq[j] = MET == L2 ? -cc : cc;
    float amax = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(qx[s][e]));
    amax = fmaxf(amax, __shfl_xor(amax, 16));
    amax = fmaxf(amax, __shfl_xor(amax, 32));
    const float sq = pow2_scale(amax);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = qx[s][e] * sq;  // exact (power of two)
        qh[j][s][e] = (_Float16)v;
        ql[j][s][e] = (_Float16)(v - (float)qh[j][s][e]);
      }
    fq[j] = (MET == L2 ? 2.0f : 1.0f) / (sq * a.sx);
    gs[j] = -INFINITY;
    if (qv[j] && a.gthr) gs[j] = key_score(__hip_atomic_load(a.gthr + qi[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    thr[j] = qv[j] ? lower_thr(gs[j], cq[j]) : INFINITY;  // an unused query slot takes no rows
    te[j] = thr[j];
  }
  // lane lists (pre-constant scores y; score = y + cq), absolute rows
  float ls[QG][L];
  uint32_t lk[QG][L];
#pragma unroll
  for (int j = 0; j < QG; ++j)
#pragma unroll
    for (int p = 0; p < L; ++p) {
      ls[j][p] = -INFINITY;
      lk[j][p] = KEY_NONE;
    }
  // shared-bound traffic of a refresh: lanes g < QG publish for group g (one atomic instruction),
  // every lane reads back the bound of query c of group g % QG (one LDS-DMA); unused slots aim at
  // the wave's first query (a max with 0 / a read: no effect), never all at one address
  const int qfirst = a.qlist && ngw > 0 ? a.qlist[it.qbeg + 16 * w] / a.nparts : it.qbeg + 16 * w;
  int pub_q = qfirst;
#pragma unroll
  for (int j = 0; j < QG; ++j)
    if (g % QG == j && qv[j]) pub_q = qi[j];

  const int r0 = it.row_begin;  // multiple of 32
  const int nt = (it.row_end - r0 + 31) / 32;
  const int64_t rlim64 = min((int64_t)it.row_end, (int64_t)a.row_limit);
  const int rlim = (int)rlim64;
  const char *hsrc = reinterpret_cast<const char *>(a.h16);
  const int lpt = (w < NCH ? 1 : 0) + (w == NW - 1 ? 1 : 0);  // this wave's loads per tile
  auto issue = [&](int t) {
    const size_t tile = (size_t)(r0 / 32 + t);
    const uint32_t base = ring_base + (uint32_t)((t % NST) * SLOT);
    if (w < NCH) glds<16>(hsrc + tile * TB + (size_t)w * 1024 + lane * 16, base + w * 1024);
    if (w == NW - 1) glds<4>(a.meta + tile * 32 + (lane & 31), base + TB);
  };
#pragma unroll
  for (int t = 0; t < NST - STEP; ++t)
    if (t < nt) issue(t);

  float sink = 0.0f;  // measurement only (ablations)
  uint32_t passes = 0;  // measurement only (a.dbg): candidate-loop iterations of this wave
  int rstep = -(1 << 20);  // step of the last refresh (its 2 vector-memory ops count in the waits)
  bool have_b = false;     // a bounds read is in bounds_l
  const int extra = a.gthr ? 2 : 0;

  // one tile of the wave's NG groups: scores on the matrix cores, then the candidate loop
  auto tile = [&](auto ngc, const char *slot, int rt, const float (&mr)[2][4]) {
    constexpr int NG = decltype(ngc)::value;
    const char *frag = slot + (g * 32 + c) * 16;
    f4v acc[NG][2];
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][b][i] = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const h8v x0 = *reinterpret_cast<const h8v *>(frag + s * 2048);
      const h8v x1 = *reinterpret_cast<const h8v *>(frag + s * 2048 + 256);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        if (Q2) {  // small term first
          acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x0, ql[j][s], acc[j][0], 0, 0, 0);
          acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x1, ql[j][s], acc[j][1], 0, 0, 0);
        }
        acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x0, qh[j][s], acc[j][0], 0, 0, 0);
        acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x1, qh[j][s], acc[j][1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      // y = f acc + meta for the lane's 8 rows (16 b + 4 g + i); while any lane of the wave has a row
      // beating its threshold, every such lane inserts its best one (the lowest row among equal
      // scores: rows enter a list in order) -- iterations = the wave's most candidates in one lane,
      // usually 0 or 1, rather than one pass per (half, row) that any lane needs
      float y[8];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) y[4 * b + i] = fmaf(fq[j], acc[j][b][i], mr[b][i]);
      if (a.ablate & 64) {
        sink += y[0] > te[j] ? y[7] : 0.0f;
        continue;
      }
      float mx = fmaxf(fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])), fmaxf(fmaxf(y[4], y[5]), fmaxf(y[6], y[7])));
      while (__builtin_amdgcn_ballot_w64(mx > te[j])) {
        ++passes;
        if (mx > te[j]) {
          int kk = 7;
#pragma unroll
          for (int k = 6; k >= 0; --k) kk = y[k] == mx ? k : kk;
          lane_insert<L>(ls[j], lk[j], mx, (uint32_t)(rt + 16 * (kk >> 2) + 4 * g + (kk & 3)));
#pragma unroll
          for (int k = 0; k < 8; ++k) y[k] = k == kk ? -INFINITY : y[k];
        }
        te[j] = fmaxf(thr[j], ls[j][L - 1]);
        mx = fmaxf(fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])), fmaxf(fmaxf(y[4], y[5]), fmaxf(y[6], y[7])));
      }
    }
  };

  mark(0);
  for (int st = 0; st < nt; ++st) {
    if (STEP == 2 && (st & 1)) goto compute;
    {
      // tiles st .. last landed: at most the younger tiles' loads (and a refresh's two ops issued
      // after tile `last` was) may be outstanding.  A wave that loads no tile pieces needs no wait:
      // the barrier orders the loaders' pieces for it.  (No other vector-memory op may sit in the
      // loop: a spilled register's scratch reload would count here -- the kernel is sized to spill
      // nothing.)
      const int last = min(st + STEP, nt) - 1;
      if (lpt > 0) {
        const int younger = max(0, min(NST - 2 * STEP, nt - 1 - last));
        const int ex = (rstep > st + STEP - NST && rstep < st) ? extra : 0;
        wait_vm_le<2 * (NST - 2 * STEP) + 2>(lpt * younger + ex);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      mark(1);
      if (a.gthr && ngw > 0 && (st / STEP) % (RF / STEP) == RF / STEP - 1) {
        if (lpt == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the previous refresh's read
        uint32_t pub = 0u;
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          if (j >= ngw) continue;
          const float bnd = quad_bound<KR, L>(ls[j]);
          if (have_b) gs[j] = fmaxf(gs[j], key_score(bounds_l[64 * w + 16 * j + c]));
          if (qv[j]) {
            if (g == j && bnd > -INFINITY) pub = score_key(bnd + cq[j]);  // <= the stored score of >= K1 entries
            thr[j] = fmaxf(lower_thr(gs[j], cq[j]), bnd);
            te[j] = fmaxf(thr[j], ls[j][L - 1]);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // bounds_l read before the DMA rewrites it
        if (g < QG) atomicMax(a.gthr + pub_q, pub);
        glds<5>(a.gthr + pub_q, (uint32_t)(size_t)(lds_void *)bounds_l + 256 * w);
        have_b = true;
        rstep = st;
      } else if (ngw > 0) {  // other steps: the bound 16 entries of the query's four lane lists reach
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          if (j >= ngw) continue;
          const float bnd = quad_bound<KR, L>(ls[j]);
          if (qv[j]) {
            thr[j] = fmaxf(thr[j], bnd);
            te[j] = fmaxf(te[j], thr[j]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < STEP; ++u)
        if (st + NST - STEP + u < nt) issue(st + NST - STEP + u);
      mark(2);
    }
  compute:
    if (ngw == 0) continue;
    const char *slot = ring + (st % NST) * SLOT;
    if (a.ablate & 128) {
      sink += reinterpret_cast<const float *>(slot + TB)[lane & 31];
      continue;
    }
    // per half b: rows 16 b + 4 g + i of the tile
    const float4 m0 = *reinterpret_cast<const float4 *>(slot + TB + 16 * g);
    const float4 m1 = *reinterpret_cast<const float4 *>(slot + TB + 64 + 16 * g);
    float mr[2][4] = {{m0.x, m0.y, m0.z, m0.w}, {m1.x, m1.y, m1.z, m1.w}};
    const int rt = r0 + 32 * st;
    if (rt + 32 > rlim) {  // rows past the item / the scan limit
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rt + 16 * b + 4 * g + i >= rlim) mr[b][i] = -INFINITY;
    }
    if (QG >= 4 && ngw >= 4) tile(std::integral_constant<int, (QG >= 4 ? 4 : 1)>{}, slot, rt, mr);
    else if (QG >= 3 && ngw == 3) tile(std::integral_constant<int, (QG >= 3 ? 3 : 1)>{}, slot, rt, mr);
    else if (QG >= 2 && ngw == 2) tile(std::integral_constant<int, (QG >= 2 ? 2 : 1)>{}, slot, rt, mr);
    else tile(std::integral_constant<int, 1>{}, slot, rt, mr);
    mark(3);
  }

  // ---- the query's four lane lists -> its top-K1 of this part (+ floor placeholders) ----
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    if (j >= ngw) continue;
    float fl = ls[j][L - 1];  // the lanes' floors: a full list may have dropped rows <= its last entry
    fl = fmaxf(fl, __shfl_xor(fl, 16));
    fl = fmaxf(fl, __shfl_xor(fl, 32));
    float *ps = a.part_s + (size_t)oslot[j] * KR;
    uint32_t *pk = a.part_k + (size_t)oslot[j] * KR;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      float bs = ls[j][0];
      uint32_t bk = lk[j][0];
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float os = __shfl_xor(bs, off);
        const uint32_t ok = (uint32_t)__shfl_xor((int)bk, off);
        if (better(os, ok, bs, bk)) {
          bs = os;
          bk = ok;
        }
      }
      if (bk != KEY_NONE && lk[j][0] == bk) {  // rows are unique: the one lane holding the head pops it
#pragma unroll
        for (int p = 0; p < L - 1; ++p) {
          ls[j][p] = ls[j][p + 1];
          lk[j][p] = lk[j][p + 1];
        }
        ls[j][L - 1] = -INFINITY;
        lk[j][L - 1] = KEY_NONE;
      }
      if (g == (r & 3) && qv[j]) {
        float so;
        uint32_t ko;
        if (bk == KEY_NONE || bs < fl) {
          so = fl > -INFINITY ? fl + cq[j] : -INFINITY;
          ko = fl > -INFINITY ? KEY_FLOOR : KEY_NONE;
        } else {
          so = bs + cq[j];
          ko = a.key_base | bk;
        }
        ps[r] = so;
        pk[r] = ko;
      }
    }
    if ((a.ablate & (64 | 128)) && g == 0 && qv[j]) ps[0] = sink;
  }
  // (after the loop: a counter atomic inside it would break the counted vmcnt waits)
  if (a.dbg && lane == 0 && ngw > 0) atomicAdd(a.dbg, passes);
  if (tm) {
    mark(4);
    if (lane == 0) {
      for (int b = 0; b < 5; ++b) atomicAdd(a.tdbg + b, tb[b]);
      atomicAdd(a.tdbg + 5, t_p - t_0);
      if (w == 0) atomicAdd(a.tdbg + 6, 1ull);
      atomicAdd(a.tdbg + 7, (unsigned long long)nt);
    }
  }
}

// PYR_RK_L=4 (tests only): 4-deep lane lists at D = 128, K1 = 16, so that lanes fill and floors
// (KEY_FLOOR placeholders) reach the merged top-K1 often -- the certificate must still hold
inline bool rk_l4() {
  const char *e = getenv("PYR_RK_L");
  return e && atoi(e) == 4;
}

// block shape of the list scan: PYR_RK_SHAPE=16 -> 16 waves x 2 groups (4 waves per SIMD, 128
// VGPRs), else 8 waves x QG groups (2 waves per SIMD, 256 VGPRs): QG = 4 with one-term queries,
// 3 with the two-term split (its query operands double)
inline int rk_shape() {
  const char *e = getenv("PYR_RK_SHAPE");
  return e ? atoi(e) : 8;
}

template <int D, int MET, int KR, bool Q2>
void launch_r(const FilterArgs &a, int max_items, hipStream_t st) {
  const int grid = a.xcd ? (max_items + 7) / 8 * 8 : max_items;
  constexpr int QG8 = Q2 ? 3 : 4;
  if (rk_shape() == 16) {
    hipLaunchKernelGGL((mfma_filter16r<D, MET, KR, Q2, 8, 16, 2, 8, 2, 8>), dim3(grid), dim3(1024), 0, st, a);
    return;
  }
  if constexpr (D == 128 && KR == 16) {
    if (rk_l4()) {
      hipLaunchKernelGGL((mfma_filter16r<D, MET, KR, Q2, 4, 8, QG8, 8, 2, 8>), dim3(grid), dim3(512), 0, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((mfma_filter16r<D, MET, KR, Q2, 8, 8, QG8, 8, 2, 8>), dim3(grid), dim3(512), 0, st, a);
}

template <int D, int MET>
void launch_rk(const FilterArgs &a, int max_items, hipStream_t st) {
  const bool q2 = a.prec != FILTER_F16X1;
  if (a.k1 == 16) q2 ? launch_r<D, MET, 16, true>(a, max_items, st) : launch_r<D, MET, 16, false>(a, max_items, st);
  else q2 ? launch_r<D, MET, 32, true>(a, max_items, st) : launch_r<D, MET, 32, false>(a, max_items, st);
}

template <int D>
void launch_rd(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  if (metric == L2) launch_rk<D, L2>(a, max_items, st);
  else launch_rk<D, IP>(a, max_items, st);
}

}  // namespace

int filter16r_qpb(int prec) {
  if (rk_shape() == 16) return 512;
  return prec == FILTER_F16X1 ? 512 : 384;
}

bool filter16r_supported(int dim, int metric, int k1) {
  if (metric != L2 && metric != IP) return false;
  if (dim != 32 && dim != 64 && dim != 128) return false;
  return k1 == 16 || k1 == 32;  // (K1 = 64 would need 16-deep lane lists: they spill at 128 VGPRs)
}

void launch_filter16r(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  switch (a.dim) {
    case 32: launch_rd<32>(a, metric, max_items, st); return;
    case 64: launch_rd<64>(a, metric, max_items, st); return;
    default: launch_rd<128>(a, metric, max_items, st); return;
  }
}

}  // namespace pyr
