// filter16.hip -- fp16 MFMA candidate filter over pre-encoded row tiles (gfx950).
//
// Same contract as filter.hip's mfma_filter (approximate scores -> per (query, slot) top-K1
// candidates -> merge -> exact refine with a certificate, failures re-run exactly), built for the
// list scan's two costs: bytes and staging.
//
//  * Rows are stored a second time, at write / build time, as fp16 in the exact order the MFMA B
//    operand wants (h16 tiles: 32 rows x D, [k-step s][lane half h][row i][8 halves], 64*D bytes),
//    scaled by a power of two sx so the store's largest |x| is below 2^14.  The scan reads 2 B per
//    dimension instead of 4, and a tile goes HBM -> LDS with global_load_lds (no registers, no
//    VALU split, conflict-free ds_read_b128 fragments since every 1 KiB piece is lane-linear).
//  * A per-row additive term (meta: -|x|^2 for L2, 0 for IP, -inf for a dead / padding row) travels
//    with the tile, so the score is one fma per (query, row): approx = f_q * acc + meta, with
//    f_q = (L2 ? 2 : 1) / (sq * sx) and sq the query's own power-of-two scale.
//  * Queries are split into two fp16 terms (qh + ql = q * sq to ~2^-22): q.x ~ qh.xh + ql.xh, two
//    v_mfma_f32_32x32x16_f16 per 16-deep k-step (PYR_FILTER_PREC=3: qh only, one MFMA).  The error
//    |q.x - approx/f| <= (2^-11 + 2^-22 + 2D u) sum|q_i x_i| + 2^-25 sum|q_i| / sx (x's fp16
//    rounding, q's split, fp32 accumulation, fp16 subnormals) is what refine_kernel's c_bf / abs
//    terms certify against (kernels.h filter_f16_cerr).
//  * The filter runs in the MFMA C layout: lane (i, h) holds row i's scores for 16 queries; each is
//    compared with that query's threshold (registers, refreshed from LDS after drains), survivors
//    are appended to the query's LDS buffer, and the query's owner lane inserts them into its
//    register top-K1 only when the buffer could overflow on the next tile.  No transpose, no
//    per-tile owner pass.  Block-level sync is one barrier per tile (the LDS ring).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <type_traits>

#include "kernels.h"

namespace pyr {
namespace {

#include "f16util.h"

constexpr int RT16 = 32;        // rows per tile (one 32x32 MFMA tile per wave)
#ifndef F16_AHEAD
#define F16_AHEAD 2  // filter16w: k-steps of B-fragment reads in flight (3: 5 VGPRs spilled, 2.56-2.62 vs 2.49-2.52 ms)
#endif
constexpr int CB16 = 48;        // candidate buffer entries per query (>= 32 + drain slack)

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

// LDS: two separate objects, so that the compiler can tell the LDS-DMA targets (ring, shared
// bounds) from the candidate state -- with one array it waits vmcnt(0) (the whole prefetch) before
// every candidate append.  Ring: NST slots [rows TB][meta: 64 floats, rows 0-31 twice].  State:
// thresholds [128], counts [128], candidate scores [128][CB16], keys [128][CB16] as row offsets in
// the item (u16: items span at most 65536 rows, filter16_max_rows()), the shared bounds [4][64].
// NST is as deep as two blocks per CU allow (80 KiB each): 5 at D = 128, 8 below.
template <int CB, int NQ = 128>
struct F16StateT {
  float thr[NQ];
  int cnt[NQ];
  float cs[NQ * CB];
  uint16_t ck[NQ * CB];
};
using F16State = F16StateT<CB16>;
template <int D, int NSTC = 0>  // NSTC: ring depth (0 = as deep as the LDS budget allows, capped at 8)
struct F16Lds {
  static constexpr int TB = RT16 * D * 2;               // h16 bytes per tile
  static constexpr int NCH = TB / 1024;                 // 1 KiB glds pieces per tile
  static constexpr int NR = NCH >= 4 ? NCH / 4 : 1;     // row pieces per loading wave per tile
  static constexpr int META = TB;                       // offset of the meta piece in a slot
  static constexpr int SLOT = TB + 256;
  static constexpr int BOUNDS = 4 * 256;                // shared-bound landing zone (one piece per wave)
  static constexpr int BUDGET = 80 * 1024 - (int)sizeof(F16State) - BOUNDS;
  static constexpr int NST_MAX = BUDGET / SLOT > 8 ? 8 : BUDGET / SLOT;
  static constexpr int NST = NSTC > 0 && NSTC < NST_MAX ? NSTC : NST_MAX;  // ring slots
  static constexpr int RING = NST * SLOT;
  static_assert(NST >= 3, "LDS ring too shallow");
  static_assert(NCH <= 4 ? true : NCH % 4 == 0, "row pieces must split evenly over 4 waves");
  // glds issued by wave w per tile: its row pieces, + the meta piece for wave 0
  static __device__ __forceinline__ int lpt(int w) {
    return (NCH >= 4 ? NR : (w < NCH ? 1 : 0)) + (w == 0 ? 1 : 0);
  }
};

// measurement only (a.tdbg): wave-uniform cycle buckets of the scan loop
struct CycleBuckets {
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t0 = 0, prev = 0;
  bool on = false;
  __device__ void start(bool enable) {
    on = enable;
    if (on) t0 = prev = __builtin_amdgcn_s_memtime();
  }
  __device__ void mark(int b) {
    if (!on) return;
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    acc[b] += now - prev;
    prev = now;
  }
  __device__ void flush(unsigned long long *out, int lane) {
    if (!on) return;
    acc[5] = __builtin_amdgcn_s_memtime() - t0;
    if (lane == 0)
      for (int b = 0; b < 8; ++b) atomicAdd(out + b, acc[b]);
  }
};

// STEP: tiles per block barrier.  STEP = 2 waits for and releases two tiles at a time (ring of
// 4 = the two being read + the next two in flight), halving the barriers and letting per-wave work
// (appends, drains) even out over two tiles; the drain checks stay per tile.
template <int D, int MET, int KR, bool Q2, int NSTC, int STEP>
__global__ __launch_bounds__(256, 2) void mfma_filter16(FilterArgs a) {
  using L = F16Lds<D, NSTC>;
  static_assert(STEP == 1 || STEP == 2, "tiles per barrier");
  static_assert(L::NST >= 2 * STEP + (STEP == 1 ? 1 : 0), "ring too shallow for the step");
  constexpr int KS = D / 16;
  constexpr int NST = L::NST;
  __shared__ __attribute__((aligned(16))) char ring[L::RING];
  __shared__ __attribute__((aligned(16))) uint32_t bounds_l[L::BOUNDS / 4];
  __shared__ __attribute__((aligned(16))) F16State state16;
  const uint32_t ring_base = (uint32_t)(size_t)(lds_void *)ring;  // LDS byte address (M0 of the DMA)
  float *const thr_l = state16.thr;
  int *const cnt_l = state16.cnt;
  float *const cs_l = state16.cs;
  uint16_t *const ck_l = state16.ck;

  int item = blockIdx.x;
  if (a.xcd) {  // XCD-major mapping (filter.hip): a list chunk's query groups share an XCD's L2
    const int per = (*a.n_items + 7) >> 3;
    item = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
    if ((int)(blockIdx.x >> 3) >= per) return;
  }
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int i32 = lane & 31, h = lane >> 5;
  CycleBuckets cb;
  cb.start(a.tdbg != nullptr);

  // ---- A operand: query 32w + i32, dims 16s + 8h .. +7 of k-step s, scaled and split ----
  const int qslot = 32 * w + i32;
  const int qi = qslot < it.qcnt ? (a.qlist ? a.qlist[it.qbeg + qslot] / a.nparts : it.qbeg + qslot) : -1;
  float qv[KS][8];
  float amax = 0.0f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (qi >= 0) {
      const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)qi * D + 16 * s + 8 * h);
      const float4 v0 = qp[0], v1 = qp[1];
      qv[s][0] = v0.x; qv[s][1] = v0.y; qv[s][2] = v0.z; qv[s][3] = v0.w;
      qv[s][4] = v1.x; qv[s][5] = v1.y; qv[s][6] = v1.z; qv[s][7] = v1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[s][j] = 0.0f;
    }
  }
  // IVF residual mode (a.cents): the tiles hold x - c of the item's list c, so the A operand is
  // q - c (L2) or q (IP), and a per (query, list) constant completes the score:
  //   L2: -|q - x|^2 = 2 (q-c).(x-c) - |x-c|^2 - |q-c|^2,   IP: q.x = q.(x-c) + q.c
  float cq = 0.0f;
  if (a.cents) {
    const float *c = a.cents + (size_t)it.list * D;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float cv = c[16 * s + 8 * h + j];
        if (MET == L2) {
          qv[s][j] = qv[s][j] - cv;
          cq += qv[s][j] * qv[s][j];
        } else {
          cq += qv[s][j] * cv;
        }
      }
    cq += __shfl_xor(cq, 32);
    if (MET == L2) cq = -cq;
  }
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(qv[s][j]));
  amax = fmaxf(amax, __shfl_xor(amax, 32));
  const float sq = pow2_scale(amax);
  h8v qh[KS], ql[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = qv[s][j] * sq;  // exact (power of two)
      qh[s][j] = (_Float16)v;
      ql[s][j] = (_Float16)(v - (float)qh[s][j]);
    }
  // C layout: register r of lane (i32, h) is query (r & 3) + 8 (r >> 2) + 4h of the wave
  const float myf = (MET == L2 ? 2.0f : 1.0f) / (sq * a.sx);
  float f[16], cqr[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    f[r] = __shfl(myf, (r & 3) + 8 * (r >> 2) + 4 * h);
    cqr[r] = __shfl(cq, (r & 3) + 8 * (r >> 2) + 4 * h);
  }

  // ---- owners (lane i32 < 32 of each wave): query 32w + i32, its top-KR and partial slot ----
  const bool owner = h == 0 && qslot < it.qcnt;
  int oslot = 0, qown = 0;
  float gs = -INFINITY;
  if (owner) {
    oslot = a.qlist ? a.qlist[it.qbeg + qslot] + it.part : (it.qbeg + qslot) * a.nparts + it.part;
    qown = qi;
    if (a.gthr) gs = key_score(__hip_atomic_load(a.gthr + qown, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  float ts[KR];
  uint32_t tk[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) {
    ts[j] = -INFINITY;
    tk[j] = KEY_NONE;
  }
  uint32_t published = 0;
  float sink = 0.0f;  // measurement only (ablations): keeps the ablated work live
  int bst = -1;  // tile at which the shared bounds were last read into bounds_l (-1: never)
  if (h == 0) {
    // an unused query slot of an active wave scores zero queries: +inf keeps its rows out of the
    // buffers (with -inf every row would survive for it and force a drain every tile)
    thr_l[qslot] = qslot < it.qcnt ? gs : INFINITY;
    cnt_l[qslot] = 0;
  }

  // ---- tile loads: rows as lane-linear 1 KiB pieces spread over the waves, meta (one 256-B piece,
  // lanes 32-63 repeating rows 0-31) by wave 0 ----
  const int r0 = it.row_begin;  // multiple of 32
  const int nt = (it.row_end - r0 + RT16 - 1) / RT16;
  const char *hsrc = reinterpret_cast<const char *>(a.h16);
  const int lpt = L::lpt(w);  // this wave's loads per tile (its counted waits)
  // tile t -> ring slot t % NST (LDS-DMA; issued in inline asm, see glds())
  auto issue = [&](int t) {
    const size_t tile = (size_t)(r0 / RT16 + t);
    const uint32_t base = ring_base + (uint32_t)((t % NST) * L::SLOT);
    if (L::NCH >= 4 || w < L::NCH) {
#pragma unroll
      for (int p = 0; p < L::NR; ++p) {
        const int c = L::NCH >= 4 ? w * L::NR + p : w;
        glds<16>(hsrc + tile * L::TB + (size_t)c * 1024 + lane * 16, base + c * 1024);
      }
    }
    if (w == 0) glds<4>(a.meta + tile * RT16 + (lane & 31), base + L::META);
  };
  __syncthreads();  // thresholds / counts initialised (the first barrier of the loop orders the rest)
#pragma unroll
  for (int t = 0; t < NST - STEP; ++t)
    if (t < nt) issue(t);

  // thr[r]: query q(r, h)'s threshold moved to the pre-constant score y = f * acc + meta (the
  // score is y + cq): t - cq lowered by a margin that covers both roundings (y + cq rounded >= t
  // implies y >= t - cq - ulp terms), so every row with score >= t passes (a few below it may too;
  // the owners' insertion compares the exact buffered scores).  A -inf threshold becomes -FLT_MAX
  // (dead / padding rows, y = -inf, never pass), +inf (unused query slot) stays +inf.
  float thr[16];
  auto load_thr = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 t4 = *reinterpret_cast<const float4 *>(thr_l + 32 * w + 8 * j + 4 * h);
      const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = tv[e], c = cqr[4 * j + e];
        const float lowered = (t - c) - 0x1p-20f * (fabsf(t) + fabsf(c));
        thr[4 * j + e] = isinf(t) ? (t > 0.0f ? t : -FLT_MAX) : fmaxf(lowered, -FLT_MAX);
      }
    }
  };
  load_thr();
  const bool wave_active = 32 * w < it.qcnt;
  int cnt[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) cnt[r] = 0;
  // register counts -> LDS for the owners (lane 0 of each half writes its 16 queries'); DS ops of
  // one wave complete in order, so the owners' reads after the wave barrier see them
  auto publish_counts = [&]() {
    if (i32 == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) cnt_l[32 * w + (r & 3) + 8 * (r >> 2) + 4 * h] = cnt[r];
    }
    __builtin_amdgcn_wave_barrier();
  };

  cb.mark(6);
  // refresh the shared bounds every pub_mask + 1 tiles, i.e. every (pub_mask + 1) / STEP steps
  const int rmask = max(1, (a.pub_mask + 1) / STEP) - 1;
  for (int st = 0; st < nt; ++st) {
    if (STEP == 2 && (st & 1)) goto compute;  // the odd tile of a step landed with the even one
    {
    // tiles st .. st+STEP-1 have landed for this wave once at most the younger tiles' loads are
    // outstanding (the compiler does not see the LDS-DMA, so these waits are the only ones ordering
    // it; extra loads issued after them -- the shared bounds, publishes -- only make it stricter)
    const int last = min(st + STEP, nt) - 1;
    wait_vm_le<3 * (NST - 2)>(lpt * max(0, min(NST - 2 * STEP, nt - 1 - last)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of this step landed; the previous step fully read
    cb.mark(0);
    if (a.gthr && ((st / STEP) & rmask) == rmask && wave_active) {
      // every pub_mask + 1 tiles: take the query's shared bound (other items' progress) read by the
      // previous refresh -- an LDS-DMA issued pub_mask + 1 (>= NST - 1) tiles ago, so this tile's
      // counted wait covered it -- publish this list's K1-th best (an atomic nothing waits for) and
      // read the bound again for the next refresh.  No wait on a returning atomic in the loop.
      // the previous read is consumed only once NST - 2 younger tiles' loads have been issued after
      // it (then the counted wait at the top of this iteration covered it)
      const bool landed = bst >= 0 && st - bst >= NST - 2;
      if (owner) {
        if (landed) {
          const float g = key_score(bounds_l[64 * w + i32]);
          if (g > gs) {
            gs = g;
            thr_l[qslot] = fmaxf(thr_l[qslot], gs);
            if (a.dbg) atomicAdd(a.dbg + 3, 1u);  // measurement only: refreshes that raised the bound
          }
        }
        if (tk[KR - 1] != KEY_NONE && score_key(ts[KR - 1]) > published) {
          published = score_key(ts[KR - 1]);
          atomicMax(a.gthr + qown, published);
        }
      }
      if (landed || bst < 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the read above before the DMA rewrites it
        glds<5>(a.gthr + (qi >= 0 ? qi : 0), (uint32_t)(size_t)(lds_void *)bounds_l + 256 * w);
        bst = st;
      }
      __builtin_amdgcn_wave_barrier();
      load_thr();
    }
#pragma unroll
    for (int u = 0; u < STEP; ++u)  // into the slots the previous step used
      if (st + NST - STEP + u < nt) issue(st + NST - STEP + u);
    cb.mark(1);
    }
  compute:
    if (!wave_active) continue;
    cb.acc[7] += 1;
    const char *slot = ring + (st % NST) * L::SLOT;
    if (a.ablate & 128) {  // measurement only: the tile stream alone
      sink += reinterpret_cast<const float *>(slot + L::META)[i32];
      continue;
    }
    f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const h8v xh = *reinterpret_cast<const h8v *>(slot + ((s * 2 + h) * 32 + i32) * 16);
      if (Q2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ql[s], xh, acc, 0, 0, 0);  // small term first
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(qh[s], xh, acc, 0, 0, 0);
    }
    const int row = r0 + st * RT16 + i32;
    float m = reinterpret_cast<const float *>(slot + L::META)[i32];
    if (row >= it.row_end || (uint32_t)row >= a.row_limit) m = -INFINITY;
    float y[16];
    uint64_t bm[16];  // wave-uniform survivor masks per register
    uint64_t anyb = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      y[r] = fmaf(f[r], acc[r], m);
      bm[r] = __ballot(y[r] >= thr[r]);
      anyb |= bm[r];
    }
    cb.mark(2);
    if (a.ablate & 64) {  // measurement only: stream + MFMA + scores, no candidates
      sink += anyb ? y[0] : 0.0f;
      continue;
    }
    if (anyb == 0) continue;
    // survivors -> the queries' LDS buffers (at most 32 per query per tile: one per row).  The wave
    // owns its 32 queries' buffers, so the fill counts live in registers (cnt[r]: query q(r, h),
    // uniform over the half-wave) and a survivor's slot is its rank among the half's survivors.
    const uint16_t off = (uint16_t)(row - r0);
    if (a.dbg) {  // measurement only: survivors, survivor tiles
      int ns = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) ns += __builtin_popcountll(bm[r]);
      if (lane == 0) {
        atomicAdd(a.dbg + 1, (uint32_t)ns);
        atomicAdd(a.dbg, 1u);
      }
    }
    int cmax = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (bm[r] == 0) continue;
      const uint32_t lo = (uint32_t)bm[r], hi = (uint32_t)(bm[r] >> 32);
      const int plo = __builtin_popcount(lo), phi = __builtin_popcount(hi);
      // rank among the half's survivors: mbcnt counts the mask's bits below the lane over all 64
      const int rank = (int)__builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u)) - (h ? plo : 0);
      if (y[r] >= thr[r]) {
        const int q = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int idx = cnt[r] + rank;
        cs_l[q * CB16 + idx] = y[r] + cqr[r];
        ck_l[q * CB16 + idx] = off;
      }
      cnt[r] += h ? phi : plo;
      cmax = max(cmax, cnt[r]);
    }
    // the owners drain every buffer of the wave when one could overflow on the next tile
    cb.mark(3);
    if (!__any(cmax > CB16 - RT16)) continue;
    publish_counts();
    int c = 0;
    if (h == 0) c = cnt_l[qslot];
    if (owner) {
      for (int i = 0; i < c; ++i) {
        const float v = cs_l[qslot * CB16 + i];
        const uint32_t k2 = a.key_base | (uint32_t)(r0 + ck_l[qslot * CB16 + i]);
        if (better(v, k2, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, k2);
      }
      if (a.gthr && tk[KR - 1] != KEY_NONE && score_key(ts[KR - 1]) > published) {
        // publish this list's K1-th best (no return value: nothing waits for it; the shared bound
        // comes back through the periodic refresh)
        published = score_key(ts[KR - 1]);
        atomicMax(a.gthr + qown, published);
      }
      float t = gs;
      if (tk[KR - 1] != KEY_NONE) t = fmaxf(t, ts[KR - 1]);
      if (a.dbg) atomicAdd(a.dbg + 2, 1u);  // measurement only: drains
      thr_l[qslot] = t;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) cnt[r] = 0;
    __builtin_amdgcn_wave_barrier();
    load_thr();
    cb.mark(4);
  }
  publish_counts();
  if (owner) {
    const int c = cnt_l[qslot];
    for (int i = 0; i < c; ++i) {
      const float v = cs_l[qslot * CB16 + i];
      const uint32_t k2 = a.key_base | (uint32_t)(r0 + ck_l[qslot * CB16 + i]);
      if (better(v, k2, ts[KR - 1], tk[KR - 1])) reg_insert<KR>(ts, tk, v, k2);
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
    if (a.ablate & (64 | 128)) ps[0] = sink;
  }
  cb.flush(a.tdbg, lane);
}

// ---------------------------------------------------------------------------------------------
// mfma_filter16w: the same filter with 8 waves x 16 queries per 128-query item, on
// v_mfma_f32_16x16x32_f16.  A wave's per-query state shrinks to a quarter of the 32-query form
// (4 scores per lane per 16-row half tile, 4 thresholds, 4 counts) and each query's register
// top-K1 is spread over the query's 4 lanes (K1 / 4 entries each), so a wave fits 128 VGPRs:
// two 512-thread blocks per CU, 4 waves per SIMD (the 32-query kernel: 2).  Tiles, meta, partial
// lists and the certificate are unchanged; the h16 tile order serves the 16x16x32 B operand too
// (lane (c, g) of k-step s, rows 16b..16b+15: piece (4s + g), row 16b + c -- 256 contiguous bytes
// per lane group, conflict-free ds_read_b128).
//
// C layout (16x16x32): register i of lane (c = lane & 15, g = lane >> 4) is query 4g + i of the
// wave, data row c of the 16-row half b.  A operand: lane (c, g) holds query c, dims 32s + 8g .. +7.
// CB: candidate buffer entries per query (>= 32 + the drain threshold CB - 32).  Measured and not
// kept: CB = 40 with a 5-slot ring (3.04 vs 2.75 ms), CB = 32 with pre-drains and a 6-slot ring
// (3.31 vs 3.08 ms) -- more tiles in flight do not shorten the scan (profiles/r2_wide/).
// NW: waves per block, 8 (128-query items, two blocks per CU) or 16 (256-query items, one block per
// CU: each streamed tile serves twice the queries; PYR_FILTER_WAVES=16, measurement).
template <int D, int MET, int KR, bool Q2, int NSTC, int STEP, int CB = CB16, int NW = 8>
__global__ __launch_bounds__(64 * NW, 4) void mfma_filter16w(FilterArgs a) {
  constexpr int TB = RT16 * D * 2;                    // h16 bytes per tile
  constexpr int NCH = TB / 1024;                      // 1 KiB pieces per tile (2, 4 or 8)
  constexpr int SLOT = TB + 256;                      // tile + meta
  constexpr int STATE = (int)sizeof(F16StateT<CB, 16 * NW>);
  static_assert(CB > RT16, "a tile may add 32 survivors per query");
  constexpr int BOUNDS = NW * 256;
  constexpr int NST_MAX0 = ((NW == 8 ? 80 : 160) * 1024 - STATE - BOUNDS) / SLOT;
  constexpr int NST_MAX = NST_MAX0 > 8 ? 8 : NST_MAX0;
  constexpr int NST = NSTC > 0 && NSTC < NST_MAX ? NSTC : NST_MAX;
  static_assert(STEP == 1 || STEP == 2, "tiles per barrier");
  static_assert(NST >= 2 * STEP + (STEP == 1 ? 1 : 0), "ring too shallow for the step");
  static_assert(NCH <= NW, "one piece per wave at most");
  static_assert(KR % 4 == 0, "top-K1 spread over 4 lanes");
  constexpr int KS = D / 32;  // 16x16x32 k-steps
  constexpr int R = KR / 4;   // top-K1 entries per lane
  __shared__ __attribute__((aligned(16))) char ring[NST * SLOT];
  __shared__ __attribute__((aligned(16))) uint32_t bounds_l[BOUNDS / 4];
  __shared__ __attribute__((aligned(16))) F16StateT<CB, 16 * NW> state16;
  const uint32_t ring_base = (uint32_t)(size_t)(lds_void *)ring;
  float *const thr_l = state16.thr;
  int *const cnt_l = state16.cnt;
  float *const cs_l = state16.cs;
  uint16_t *const ck_l = state16.ck;

  int item = blockIdx.x;
  if (a.xcd) {
    const int per = (*a.n_items + 7) >> 3;
    item = ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
    if ((int)(blockIdx.x >> 3) >= per) return;
  }
  if (item >= *a.n_items) return;
  const ScanItem it = a.items[item];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int c16 = lane & 15, g = lane >> 4;

  // ---- A operand: query 16w + c16, dims 32s + 8g .. +7 of k-step s, scaled and split ----
  const int qslot = 16 * w + c16;
  const int qi = qslot < it.qcnt ? (a.qlist ? a.qlist[it.qbeg + qslot] / a.nparts : it.qbeg + qslot) : -1;
  float qv[KS][8];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (qi >= 0) {
      const float4 *qp = reinterpret_cast<const float4 *>(a.queries + (size_t)qi * D + 32 * s + 8 * g);
      const float4 v0 = qp[0], v1 = qp[1];
      qv[s][0] = v0.x; qv[s][1] = v0.y; qv[s][2] = v0.z; qv[s][3] = v0.w;
      qv[s][4] = v1.x; qv[s][5] = v1.y; qv[s][6] = v1.z; qv[s][7] = v1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[s][j] = 0.0f;
    }
  }
  // IVF residual mode: A = q - c (L2) or q (IP), cq the per (query, list) constant (filter16)
  float cq = 0.0f;
  if (a.cents) {
    const float *c = a.cents + (size_t)it.list * D;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float cv = c[32 * s + 8 * g + j];
        if (MET == L2) {
          qv[s][j] = qv[s][j] - cv;
          cq += qv[s][j] * qv[s][j];
        } else {
          cq += qv[s][j] * cv;
        }
      }
    cq += __shfl_xor(cq, 16);
    cq += __shfl_xor(cq, 32);
    if (MET == L2) cq = -cq;
  }
  float amax = 0.0f;
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(qv[s][j]));
  amax = fmaxf(amax, __shfl_xor(amax, 16));
  amax = fmaxf(amax, __shfl_xor(amax, 32));
  const float sq = pow2_scale(amax);
  h8v qh[KS], ql[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = qv[s][j] * sq;  // exact (power of two)
      qh[s][j] = (_Float16)v;
      ql[s][j] = (_Float16)(v - (float)qh[s][j]);
    }
  const float myf = (MET == L2 ? 2.0f : 1.0f) / (sq * a.sx);
  float f[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = __shfl(myf, 4 * g + i);

  // ---- owners: lanes (c16, g = 0); query 16w + c16's top-KR is spread over its 4 lanes: lane
  // (c16, g) holds entries R g .. R g + R - 1 (descending) ----
  const bool qvalid = qslot < it.qcnt;
  const bool owner = g == 0 && qvalid;
  int oslot = 0;
  float gs = -INFINITY;
  if (qvalid) {
    oslot = a.qlist ? a.qlist[it.qbeg + qslot] + it.part : (it.qbeg + qslot) * a.nparts + it.part;
    if (a.gthr) gs = key_score(__hip_atomic_load(a.gthr + qi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  float ts[R];
  uint32_t tk[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    ts[j] = -INFINITY;
    tk[j] = KEY_NONE;
  }
  // the query's K1-th entry (lane (c16, 3), entry R - 1), on all 4 of its lanes
  auto last_s = [&]() { return __shfl(ts[R - 1], 48 + c16); };
  auto last_k = [&]() { return (uint32_t)__shfl((int)tk[R - 1], 48 + c16); };
  uint32_t published = 0;
  float sink = 0.0f;
  int bst = -1;
  if (g == 0) {
    thr_l[qslot] = qvalid ? gs : INFINITY;
    cnt_l[qslot] = 0;
  }

  const int r0 = it.row_begin;
  const int nt = (it.row_end - r0 + RT16 - 1) / RT16;
  const char *hsrc = reinterpret_cast<const char *>(a.h16);
  const int lpt = (w < NCH ? 1 : 0) + (w == NW - 1 ? 1 : 0);  // pieces per tile; meta by the last wave
  auto issue = [&](int t) {
    const size_t tile = (size_t)(r0 / RT16 + t);
    const uint32_t base = ring_base + (uint32_t)((t % NST) * SLOT);
    if (w < NCH) glds<16>(hsrc + tile * TB + (size_t)w * 1024 + lane * 16, base + w * 1024);
    if (w == NW - 1) glds<4>(a.meta + tile * RT16 + (lane & 31), base + TB);
  };
  __syncthreads();
#pragma unroll
  for (int t = 0; t < NST - STEP; ++t)
    if (t < nt) issue(t);

  // thresholds of queries 4g + i moved to the pre-constant score y (filter16 load_thr)
  float thr[4];
  auto load_thr = [&]() {
    const float4 t4 = *reinterpret_cast<const float4 *>(thr_l + 16 * w + 4 * g);
    const float tv[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float t = tv[i], c = __shfl(cq, 4 * g + i);
      const float lowered = (t - c) - 0x1p-20f * (fabsf(t) + fabsf(c));
      thr[i] = isinf(t) ? (t > 0.0f ? t : -FLT_MAX) : fmaxf(lowered, -FLT_MAX);
    }
  };
  load_thr();
  const bool wave_active = 16 * w < it.qcnt;
  int cnt[4] = {0, 0, 0, 0};
  auto publish_counts = [&]() {
    if (c16 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) cnt_l[16 * w + 4 * g + i] = cnt[i];
    }
    __builtin_amdgcn_wave_barrier();
  };
  // distributed insert of (v, key) into the query's 4-lane list (all 4 lanes of the query call it)
  auto dist_insert = [&](float v, uint32_t key) {
    bool b[R];
#pragma unroll
    for (int j = 0; j < R; ++j) b[j] = better(v, key, ts[j], tk[j]);
    const float ps = __shfl(ts[R - 1], lane - 16);
    const uint32_t pk = (uint32_t)__shfl((int)tk[R - 1], lane - 16);
    // (every lane of the query takes part in the shuffles: a bpermute reads 0 from a disabled lane)
    const int pbi = __shfl((int)b[R - 1], lane - 16);
    const bool pb = g > 0 && pbi != 0;
#pragma unroll
    for (int j = R - 1; j >= 1; --j) {
      ts[j] = b[j - 1] ? ts[j - 1] : (b[j] ? v : ts[j]);
      tk[j] = b[j - 1] ? tk[j - 1] : (b[j] ? key : tk[j]);
    }
    ts[0] = pb ? ps : (b[0] ? v : ts[0]);
    tk[0] = pb ? pk : (b[0] ? key : tk[0]);
  };
  // the query's buffered candidates -> its list (cq added here: the buffer holds y)
  auto insert_buffer = [&](int n) {
    for (int i = 0; i < n; ++i) {
      const float v = cs_l[qslot * CB + i] + cq;
      const uint32_t k2 = a.key_base | (uint32_t)(r0 + ck_l[qslot * CB + i]);
      if (better(v, k2, last_s(), last_k())) dist_insert(v, k2);
    }
  };
  auto drain = [&]() {
    publish_counts();
    const int n = qvalid ? cnt_l[qslot] : 0;
    insert_buffer(n);
    const float ls = last_s();
    const uint32_t lk = last_k();
    if (owner) {
      if (a.gthr && lk != KEY_NONE && score_key(ls) > published) {
        published = score_key(ls);
        atomicMax(a.gthr + qi, published);
      }
      float t = gs;
      if (lk != KEY_NONE) t = fmaxf(t, ls);
      if (a.dbg) atomicAdd(a.dbg + 2, 1u);  // measurement only: drains
      thr_l[qslot] = t;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) cnt[i] = 0;
    __builtin_amdgcn_wave_barrier();
    load_thr();
  };
  // PYR_F16_PRIO=1: static priority for the younger half of the block (waves 4-7), the arbitration
  // loser of a SIMD's two waves of one block (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (a.prio && w >= 4) __builtin_amdgcn_s_setprio(1);
  const int rmask = max(1, (a.pub_mask + 1) / STEP) - 1;
  for (int st = 0; st < nt; ++st) {
    if (STEP == 2 && (st & 1)) goto compute;
    {
    const int last = min(st + STEP, nt) - 1;
    wait_vm_le<3 * (NST - 2)>(lpt * max(0, min(NST - 2 * STEP, nt - 1 - last)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (a.gthr && ((st / STEP) & rmask) == rmask && wave_active) {
      // shared-bound refresh (filter16): take the bound read by the previous refresh, publish the
      // list's K1-th best, read the bound again
      const bool landed = bst >= 0 && st - bst >= NST - 2;
      const float ls = last_s();
      const uint32_t lk = last_k();
      if (owner) {
        if (landed) {
          const float gv = key_score(bounds_l[64 * w + c16]);
          if (gv > gs) {
            gs = gv;
            thr_l[qslot] = fmaxf(thr_l[qslot], gs);
            if (a.dbg) atomicAdd(a.dbg + 3, 1u);
          }
        }
        if (lk != KEY_NONE && score_key(ls) > published) {
          published = score_key(ls);
          atomicMax(a.gthr + qi, published);
        }
      }
      if (landed || bst < 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        glds<5>(a.gthr + (qi >= 0 ? qi : 0), (uint32_t)(size_t)(lds_void *)bounds_l + 256 * w);
        bst = st;
      }
      __builtin_amdgcn_wave_barrier();
      load_thr();
    }
#pragma unroll
    for (int u = 0; u < STEP; ++u)
      if (st + NST - STEP + u < nt) issue(st + NST - STEP + u);
    }
  compute:
    if (!wave_active) continue;
    const char *slot = ring + (st % NST) * SLOT;
    if (a.ablate & 128) {
      sink += reinterpret_cast<const float *>(slot + TB)[lane & 31];
      continue;
    }
    f4v acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[b][i] = 0.0f;
    // the two halves' accumulation chains interleaved (each MFMA's result is not the next one's
    // input); every fragment read is issued up front and the scheduler is told to run them one
    // k-step ahead of the MFMAs (sched_group_barrier: 4 reads, then per k-step 4 MFMAs + the next
    // 2 reads), so the waves a block barrier releases together do not all wait on LDS per k-step
    const char *frag = slot + (g * 32 + c16) * 16;
    h8v xf[KS][2];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      xf[s][0] = *reinterpret_cast<const h8v *>(frag + s * 2048);
      xf[s][1] = *reinterpret_cast<const h8v *>(frag + s * 2048 + 256);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (Q2) {  // small term first
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql[s], xf[s][0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql[s], xf[s][1], acc[1], 0, 0, 0);
      }
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[s], xf[s][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[s], xf[s][1], acc[1], 0, 0, 0);
    }
    if constexpr (KS >= 2) {
      constexpr int AH = F16_AHEAD < KS ? F16_AHEAD : KS;  // k-steps of reads in flight
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * AH, 0);  // DS reads of k-steps 0 .. AH - 1
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, Q2 ? 4 : 2, 0);  // k-step s's MFMAs
        if (s + AH < KS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // k-step s + AH's reads
      }
    }
    const float *mrow = reinterpret_cast<const float *>(slot + TB);
    float y[2][4];
    uint64_t bm[2][4];
    uint64_t anyb = 0;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int row = r0 + st * RT16 + 16 * b + c16;
      float m = mrow[16 * b + c16];
      if (row >= it.row_end || (uint32_t)row >= a.row_limit) m = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[b][i] = fmaf(f[i], acc[b][i], m);
        bm[b][i] = __ballot(y[b][i] >= thr[i]);
        anyb |= bm[b][i];
      }
    }
    if (a.ablate & 64) {
      sink += anyb ? y[0][0] : 0.0f;
      continue;
    }
    if (anyb == 0) continue;
    // PYR_F16_PRIO=2 (default): a wave with survivors to append runs at raised priority, so the
    // block's slowest wave reaches the next barrier sooner
    if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
    if (a.dbg) {
      int ns = 0;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) ns += __builtin_popcountll(bm[b][i]);
      if (lane == 0) {
        atomicAdd(a.dbg + 1, (uint32_t)ns);
        atomicAdd(a.dbg, 1u);
      }
    }
    // survivors -> the queries' LDS buffers: query 4g + i's survivors of half b are the bits of
    // bm[b][i] in lane group g; a survivor's slot is its rank among them
    const uint64_t below = (1ull << (16 * g)) - 1ull;  // lanes of the lower groups
    int cmax = 0;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const uint16_t off = (uint16_t)(st * RT16 + 16 * b + c16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t mk = bm[b][i];
        if (mk == 0) continue;
        const int grp = __builtin_popcountll((mk >> (16 * g)) & 0xFFFFull);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u)) -
                         __builtin_popcountll(mk & below);
        if ((mk >> lane) & 1) {
          const int q = 16 * w + 4 * g + i;
          const int idx = cnt[i] + rank;
          cs_l[q * CB + idx] = y[b][i];
          ck_l[q * CB + idx] = off;
        }
        cnt[i] += grp;
        cmax = max(cmax, cnt[i]);
      }
    }
    if (__any(cmax > CB - RT16)) drain();
    if (a.prio == 2) __builtin_amdgcn_s_setprio(0);
  }
  publish_counts();
  insert_buffer(qvalid ? cnt_l[qslot] : 0);
  if (qvalid) {
    const float ls = last_s();
    const uint32_t lk = last_k();
    if (owner && a.gthr && lk != KEY_NONE && score_key(ls) > published) atomicMax(a.gthr + qi, score_key(ls));
    float *ps = a.part_s + (size_t)oslot * KR + R * g;
    uint32_t *pk = a.part_k + (size_t)oslot * KR + R * g;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      ps[j] = ts[j];
      pk[j] = tk[j];
    }
    if ((a.ablate & (64 | 128)) && g == 0) ps[0] = sink;
  }
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

// ring depth of the D = 128, K1 = 16 kernels (PYR_F16_NST, measurement knob: 3, 4 or 0 = deepest)
static int f16_nst() {
  const char *e = getenv("PYR_F16_NST");
  return e ? atoi(e) : 3;
}
// tiles per block barrier of the K1 = 16 kernels (PYR_F16_STEP, measurement knob: 2 = default, 1 =
// one tile per barrier: 3.81 -> 3.45 ms list scan at I1, profiles/r2_sweeps/r2st_sweep.log)
static int f16_step() {
  const char *e = getenv("PYR_F16_STEP");
  return e ? atoi(e) : 2;
}

// 8 waves x 16 queries (mfma_filter16w) for K1 = 16 and 32 (PYR_F16_WIDE: 1 = on, 0 = the 4 x 32 kernel)
static int f16_wide() {
  const char *e = getenv("PYR_F16_WIDE");
  return e ? atoi(e) : 1;
}

template <int D, int MET, int KR, bool Q2>
void launch16_p(const FilterArgs &a, int max_items, hipStream_t st) {
  // all LDS is static (79 KiB at D = 128): no dynamic-LDS attribute (a 160 KiB dynamic limit on top
  // of the static size makes the launch invalid)
  const int grid = a.xcd ? (max_items + 7) / 8 * 8 : max_items;
  if constexpr (KR == 32) {  // K1 = 32 on 8 waves spills ~10 VGPRs at 128 and still wins: k = 20 list scan
                             // 6.90 -> 3.94 ms (profiles/r2_final/sweep_k20_wide.log)
    if (f16_wide()) {
      hipLaunchKernelGGL((mfma_filter16w<D, MET, KR, Q2, 4, 2>), dim3(grid), dim3(512), 0, st, a);
      return;
    }
  }
  if constexpr (KR == 16) {
    if (a.waves == 16) {  // 256-query items (engine filter_qchunk)
      hipLaunchKernelGGL((mfma_filter16w<D, MET, KR, Q2, 4, 2, CB16, 16>), dim3(grid), dim3(1024), 0, st, a);
      return;
    }
    if (f16_wide()) {
      hipLaunchKernelGGL((mfma_filter16w<D, MET, KR, Q2, 4, 2>), dim3(grid), dim3(512), 0, st, a);
      return;
    }
  }
  if constexpr (KR == 16) {  // the K1 = 16 list scans: two tiles per barrier (default)
    if (f16_step() == 2) {
      hipLaunchKernelGGL((mfma_filter16<D, MET, KR, Q2, 4, 2>), dim3(grid), dim3(256), 0, st, a);
      return;
    }
  }
  if constexpr (D == 128 && KR == 16) {
    if (f16_nst() == 3) {
      hipLaunchKernelGGL((mfma_filter16<D, MET, KR, Q2, 3, 1>), dim3(grid), dim3(256), 0, st, a);
      return;
    }
    if (f16_nst() == 4) {
      hipLaunchKernelGGL((mfma_filter16<D, MET, KR, Q2, 4, 1>), dim3(grid), dim3(256), 0, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((mfma_filter16<D, MET, KR, Q2, 0, 1>), dim3(grid), dim3(256), 0, st, a);
}

template <int D, int MET>
void launch16_k(const FilterArgs &a, int max_items, hipStream_t st) {
  const bool q2 = a.prec != FILTER_F16X1;
  if (a.k1 == 16) q2 ? launch16_p<D, MET, 16, true>(a, max_items, st) : launch16_p<D, MET, 16, false>(a, max_items, st);
  else if (a.k1 == 32) q2 ? launch16_p<D, MET, 32, true>(a, max_items, st) : launch16_p<D, MET, 32, false>(a, max_items, st);
  else q2 ? launch16_p<D, MET, 64, true>(a, max_items, st) : launch16_p<D, MET, 64, false>(a, max_items, st);
}

template <int D>
void launch16_d(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  if (metric == L2) launch16_k<D, L2>(a, max_items, st);
  else launch16_k<D, IP>(a, max_items, st);
}

// ---- write / build side: fp16 tiles, per-row meta, the store's |x| maximum ----

// h16 tile element of (row r, dim d): tile r/32, k-step d/16, half (d/8)&1, row r%32, d%8
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

int filter16_max_rows() { return 65536; }  // candidate keys are u16 row offsets within an item

bool filter16_supported(int dim, int metric, int k1) {
  if (metric != L2 && metric != IP) return false;
  if (dim != 32 && dim != 64 && dim != 128) return false;
  return k1 == 16 || k1 == 32 || k1 == 64;
}

void launch_filter16(const FilterArgs &a, int metric, int max_items, hipStream_t st) {
  if (max_items <= 0) return;
  switch (a.dim) {
    case 32: launch16_d<32>(a, metric, max_items, st); return;
    case 64: launch16_d<64>(a, metric, max_items, st); return;
    default: launch16_d<128>(a, metric, max_items, st); return;
  }
}

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
