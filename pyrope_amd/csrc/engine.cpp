// engine.cpp -- device-resident index objects behind include/pyrope_ann.h.
//
// Each class restates one reference IVectorIndex implementation's observable
// semantics (storage order, buffer/list interplay, MaxScans, nprobe defaults,
// quirks) with the scan itself on the GPU.  Paths are relative to
// /root/reference/src/Pyrope.GarnetServer/.
#include "engine.h"
#include "persist.h"

#include <cmath>
#include <cstdio>

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstring>
#include <numeric>

namespace pyr {

// ---------------------------------------------------------------------------
// memory
// ---------------------------------------------------------------------------
// diagnostics only (PYR_DEBUG_ALLOC=<file>): every device allocation and free of the library appended to
// the file, so that the address of a GPU memory fault can be matched to the buffer it falls in
static void alloc_log(const char *what, const void *p, size_t n) {
  static const char *path = knob("PYR_DEBUG_ALLOC");
  if (!path || !*path) return;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (FILE *f = fopen(path, "a")) {
    fprintf(f, "%s %p %zu\n", what, p, n);
    fclose(f);
  }
}

void DevMem::ensure(size_t bytes) {
  if (bytes <= n && p) return;
  if (p) {
    alloc_log("free", p, n);
    HIPCHK(hipFree(p));
  }
  p = nullptr;
  n = 0;
  size_t want = std::max<size_t>(bytes, 256);
  if (hipMalloc(&p, want) != hipSuccess) {
    p = nullptr;
    throw Error(PYR_E_OOM, "device allocation of " + std::to_string(want) + " bytes failed");
  }
  alloc_log("alloc", p, want);
  n = want;
}

void DevMem::grow_keep(size_t bytes, size_t keep, hipStream_t st) {
  if (bytes <= n && p) return;
  void *q = nullptr;
  size_t want = std::max<size_t>(bytes, 256);
  if (hipMalloc(&q, want) != hipSuccess) throw Error(PYR_E_OOM, "device allocation of " + std::to_string(want) + " bytes failed");
  alloc_log("alloc", q, want);
  if (p && keep) HIPCHK(hipMemcpyAsync(q, p, std::min(keep, n), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  if (p) {
    alloc_log("free", p, n);
    HIPCHK(hipFree(p));
  }
  p = q;
  n = want;
}

void DevMem::release() {
  if (p) {
    alloc_log("free", p, n);
    (void)hipFree(p);
  }
  p = nullptr;
  n = 0;
}

static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

void RowStore::reserve(int64_t slots, hipStream_t st) {
  if (slots <= cap) return;
  ++gen;
  // whole 32-slot tiles (the fp16 filter's unit; a multiple of the blocked layout's 8)
  int64_t nc = round_up(std::max<int64_t>(slots, std::max<int64_t>(cap * 3 / 2, 64)), 32);
  rows.grow_keep(sizeof(float) * nc * dim, sizeof(float) * cap * dim, st);
  live.grow_keep(nc, cap, st);
  labels.grow_keep(sizeof(int64_t) * nc, sizeof(int64_t) * cap, st);
  rsq.grow_keep(sizeof(float) * nc, sizeof(float) * cap, st);
  if (cosine) norms.grow_keep(sizeof(float) * nc, sizeof(float) * cap, st);
  if (!rmax.p) {
    // [0] score_key of the largest finite |x|^2 (0: below any float), [1] nonzero once a row with a
    // non-finite |x|^2 was stored (the bf16x3 / fp32 filters cannot certify against such a row)
    rmax.ensure(2 * sizeof(uint32_t));
    HIPCHK(hipMemsetAsync(rmax.p, 0, 2 * sizeof(uint32_t), st));
  }
  // new tail: not visible, zero rows (padding rows of a group are never scored)
  HIPCHK(hipMemsetAsync(live.as<uint8_t>() + cap, 0, nc - cap, st));
  HIPCHK(hipMemsetAsync(rows.as<float>() + cap * dim, 0, sizeof(float) * (nc - cap) * dim, st));
  HIPCHK(hipMemsetAsync(rsq.as<float>() + cap, 0, sizeof(float) * (nc - cap), st));
  if (cosine) HIPCHK(hipMemsetAsync(norms.as<float>() + cap, 0, sizeof(float) * (nc - cap), st));
  if (f16) {
    rrm.grow_keep(sizeof(float) * nc * dim, sizeof(float) * cap * dim, st);
    HIPCHK(hipMemsetAsync(rrm.as<float>() + cap * dim, 0, sizeof(float) * (nc - cap) * dim, st));
    if (center16) rsq16.grow_keep(sizeof(float) * nc, sizeof(float) * cap, st);
    h16.grow_keep(sizeof(uint16_t) * nc * tdim(), sizeof(uint16_t) * cap * tdim(), st);
    meta.grow_keep(sizeof(float) * nc, sizeof(float) * cap, st);
    HIPCHK(hipMemsetAsync(static_cast<char *>(h16.p) + sizeof(uint16_t) * cap * tdim(), 0,
                          sizeof(uint16_t) * (nc - cap) * tdim(), st));
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(meta.as<float>() + cap), (int)0xFF800000u, nc - cap,
                             st));  // -inf: not a row
    if (!amaxd.p) amaxd.ensure(sizeof(uint32_t));
  }
  cap = nc;
}

static float pow2_scale_host(float amax) {  // max |x_i| * sx < 2^14 (filter16.hip pow2_scale)
  if (!(amax > 0.0f) || !std::isfinite(amax)) return 1.0f;
  int e;
  std::frexp(amax, &e);
  return std::ldexp(1.0f, 14 - e);
}

// Concurrent searches share one store: the refresh runs under a lock and completes (stream
// synchronized) before another search can take the cached pointer.  It runs only after a write or
// a change of the error-bound constants, never in a steady-state search (hipGraph capture included).
static bool capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(st, &cs));
  return cs == hipStreamCaptureStatusActive;
}

const float *RowStore::row_terms(int met, float kr, float kx, hipStream_t st) {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if (mub_gen == gen && mub_met == met && mub_kr == kr && mub_kx == kx && mub.n >= sizeof(float) * cap) {
    if (!mub_done && st != mub_st) {  // refreshed on another stream: order after it (once seen done, never again)
      if (hipEventQuery(mub_ev) == hipSuccess) mub_done = true;
      else if (capturing(st)) HIPCHK(hipEventSynchronize(mub_ev));  // (no event edge into a capture)
      else HIPCHK(hipStreamWaitEvent(st, mub_ev, 0));
    }
    return mub.as<float>();
  }
  if (capturing(st))
    throw Error(PYR_E_STATE, "the index changed since its last search and its per-row terms must be refreshed: "
                             "run one search outside the stream capture first");
  mub.ensure(sizeof(float) * std::max<int64_t>(cap, 1));
  launch_row_terms(meta.as<float>(), resid || center16 ? rsq16.as<float>() : rsq.as<float>(), rsq.as<float>(), cap,
                   met, kr, kx, mub.as<float>(), st);
  HIPCHK(hipGetLastError());
  if (!mub_ev) HIPCHK(hipEventCreateWithFlags(&mub_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(mub_ev, st));
  mub_st = st;
  mub_done = false;
  mub_gen = gen;
  mub_met = met;
  mub_kr = kr;
  mub_kx = kx;
  return mub.as<float>();
}

void RowStore::encode16(const int64_t *d_slots, int64_t cnt, hipStream_t st) {
  if (!f16 || cap == 0) return;
  ++gen;
  if (!d_slots) cnt = cap;
  if (cnt <= 0) return;
  // FLAT L2 centering: tiles hold x - center (one "list"), meta -|x - center|^2
  const float *ctr = center16 && resid ? center.as<float>() : nullptr;
  if (ctr) launch_resid_sq(rows.as<float>(), cnt, dim, ctr, nullptr, rsq16.as<float>(), st, d_slots,
                           rmax_r.as<uint32_t>());
  HIPCHK(hipMemsetAsync(amaxd.p, 0, sizeof(uint32_t), st));
  launch_absmax(rows.as<float>(), d_slots, cnt, dim, amaxd.as<uint32_t>(), st, ctr, nullptr);
  uint32_t bits = 0;
  HIPCHK(hipMemcpyAsync(&bits, amaxd.p, sizeof(bits), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  float am;
  std::memcpy(&am, &bits, sizeof(am));
  if (sx == 0.0f || std::max(am, amax) * sx >= 16384.0f) {  // first rows, or a larger row: new scale, all slots
    amax = std::max(am, amax);
    sx = pow2_scale_host(amax);
    if (ctr && d_slots)  // every slot is re-encoded: their residual norms too
      launch_resid_sq(rows.as<float>(), cap, dim, ctr, nullptr, rsq16.as<float>(), st, nullptr, rmax_r.as<uint32_t>());
    launch_encode16(rows.as<float>(), nullptr, cap, dim, sx, h16.p, st, ctr, nullptr, meta_norms(), tdim());
    launch_meta16(nullptr, cap, met16, meta_norms(), live.as<uint8_t>(), meta.as<float>(), st);
  } else {
    amax = std::max(am, amax);
    launch_encode16(rows.as<float>(), d_slots, cnt, dim, sx, h16.p, st, ctr, nullptr, meta_norms(), tdim());
    launch_meta16(d_slots, cnt, met16, meta_norms(), live.as<uint8_t>(), meta.as<float>(), st);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
}

// Slots are mapped host memory the write kernel reads in place (no copy call).  An event closes every group
// of G slots; a group is reused only once its event (K writes ago) has completed.
char *PinnedRing::take(size_t need, int *slot) {
  constexpr int G = 8;
  if (need > bytes) {  // (re)allocate every slot: wait for their readers first
    for (int g = 0; g < K / G; ++g)
      if (ev[g]) HIPCHK(hipEventSynchronize(ev[g]));
    for (int i = 0; i < K; ++i) {
      if (host[i]) HIPCHK(hipHostFree(host[i]));
      host[i] = nullptr;
    }
    bytes = std::max<size_t>(need, 4096);
    for (int i = 0; i < K; ++i) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&host[i]), bytes, hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dev[i]), host[i], 0));
    }
    for (int g = 0; g < K / G; ++g)
      if (!ev[g]) HIPCHK(hipEventCreateWithFlags(&ev[g], hipEventDisableTiming));
    next = 0;
  }
  const int i = next;
  next = (next + 1) % K;
  if (i % G == 0) HIPCHK(hipEventSynchronize(ev[i / G]));  // the group's readers have run (normally long ago)
  *slot = i;
  return host[i];
}
void PinnedRing::done(int slot, hipStream_t st) {
  if (slot % 8 == 7) HIPCHK(hipEventRecord(ev[slot / 8], st));
}
PinnedRing::~PinnedRing() {
  for (int i = 0; i < K; ++i)
    if (host[i]) (void)hipHostFree(host[i]);  // (hipHostFree waits for the device)
  for (int g = 0; g < K; ++g)
    if (ev[g]) (void)hipEventDestroy(ev[g]);
}

// measurement only (PYR_WRITE_PROF=1): host time of the write path's sections, printed at exit
struct WriteProf {
  bool on = knob("PYR_WRITE_PROF") != nullptr;
  double t[8] = {};
  int64_t n = 0;
  ~WriteProf() {
    if (on && n)
      fprintf(stderr, "[write prof] %lld calls, us per call: prep %.2f amax %.2f stage %.2f launch %.2f done %.2f add-host %.2f after %.2f note %.2f\n",
              (long long)n, 1e6 * t[0] / n, 1e6 * t[1] / n, 1e6 * t[2] / n, 1e6 * t[3] / n, 1e6 * t[4] / n,
              1e6 * t[5] / n, 1e6 * t[6] / n, 1e6 * t[7] / n);
  }
};
static WriteProf &wprof() {
  static WriteProf p;
  return p;
}
struct WSec {
  int i;
  std::chrono::steady_clock::time_point t0;
  explicit WSec(int s) : i(s), t0(wprof().on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point()) {}
  ~WSec() {
    if (wprof().on) wprof().t[i] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
};

bool wprof_on() { return wprof().on; }
void wprof_add(int i, double sec) { wprof().t[i] += sec; }
void note_write_call() {
  if (wprof().on) ++wprof().n;
}

// rows a write may take through the small-batch path (RowStore::write)
static int64_t small_write_rows() {
  const char *e = knob("PYR_SMALL_WRITE");  // 0: the bulk path always (A/B)
  return e ? atoll(e) : 64;
}

// FLAT L2 tiles: the center becomes the mean of the live rows (fp64 sums on the device), every slot is
// re-encoded against it (residual norms, scale, tiles, meta).  Synchronizes st.
void RowStore::recenter(hipStream_t st) {
  if (!(f16 && center16 && resid) || n <= 0) return;
  DevMem sums;
  sums.ensure(sizeof(double) * dim + sizeof(unsigned long long));
  HIPCHK(hipMemsetAsync(sums.p, 0, sizeof(double) * dim + sizeof(unsigned long long), st));
  double *ds = sums.as<double>();
  launch_live_sums(rows.as<float>(), live.as<uint8_t>(), n, dim, ds, reinterpret_cast<unsigned long long *>(ds + dim),
                   st);
  std::vector<double> h(dim + 1);
  HIPCHK(hipMemcpyAsync(h.data(), sums.p, sizeof(double) * (dim + 1), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  unsigned long long c;
  std::memcpy(&c, &h[dim], sizeof(c));
  center_rows = n;
  if (c == 0) return;
  for (int d = 0; d < dim; d++) hcenter[d] = (float)(h[d] / (double)c);
  HIPCHK(hipMemcpyAsync(center.p, hcenter.data(), sizeof(float) * dim, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(rmax_r.p, 0, sizeof(uint32_t), st));
  sx = 0.0f;  // a new scale from the new residuals, every slot re-encoded
  amax = 0.0f;
  encode16(nullptr, cap, st);
}

bool RowStore::write(const float *x, const int64_t *slots, const int64_t *labs, int64_t cnt, hipStream_t st,
                     DevMem &stage_x, DevMem &stage_i, bool x_dev, uint8_t *q8ok, bool need_slots) {
  if (cnt <= 0) return true;
  const uint64_t g0 = gen;
  ++gen;
  // small-batch path: the rows' largest |x_i| (of x - center) is taken on the host, so the scale decision
  // needs no device read-back; one pinned copy, one fused kernel, no synchronization
  if (!x_dev && !need_slots && cnt <= small_write_rows() && dim <= SMALL_WRITE_MAX_DIM &&
      (!f16 || (sx > 0.0f && (center16 ? resid : !resid)))) {
    float am = 0.0f;
    WSec sec_am(1);
    if (f16)
      for (int64_t i = 0; i < cnt; i++)
        for (int d = 0; d < dim; d++) {
          const float v = std::fabs(resid ? x[(size_t)i * dim + d] - hcenter[d] : x[(size_t)i * dim + d]);
          if (std::isfinite(v)) am = std::max(am, v);
        }
    if (!f16 || std::max(am, amax) * sx < 16384.0f) {
      const size_t xb = sizeof(float) * cnt * dim, ib = sizeof(int64_t) * cnt;
      int slot = -1;
      WSec sec_st(2);
      SmallWriteArgs a{};
      SmallWriteRows inl;
      const bool inline_rows = cnt <= SMALL_INLINE_ROWS && cnt * dim <= SMALL_INLINE_FLOATS;
      if (inline_rows) {  // the rows travel as kernel arguments
        std::memcpy(inl.x, x, xb);
        std::memcpy(inl.slot, slots, ib);
        std::memcpy(inl.lab, labs, ib);
      } else {  // the kernel reads a mapped host slot in place
        char *h = ring.take(xb + 2 * ib, &slot);
        std::memcpy(h, x, xb);
        std::memcpy(h + xb, slots, ib);
        std::memcpy(h + xb + ib, labs, ib);
        const char *dh = ring.dev[slot];
        a.x = reinterpret_cast<const float *>(dh);
        a.slots = reinterpret_cast<const int64_t *>(dh + xb);
        a.labs = a.slots + cnt;
      }
      a.cnt = (int32_t)cnt;
      a.dim = dim;
      a.dp = tdim();
      a.rows = rows.as<float>();
      a.rrm = f16 ? rrm.as<float>() : nullptr;
      a.labels = labels.as<int64_t>();
      a.live = live.as<uint8_t>();
      a.norms = cosine ? norms.as<float>() : nullptr;
      a.rsq = rsq.as<float>();
      a.rmax = rmax.as<uint32_t>();
      if (f16) {
        a.h16 = h16.as<_Float16>();
        a.sx = sx;
        a.center = resid ? center.as<float>() : nullptr;
        a.rsq16 = rsq16.as<float>();
        a.rmax_r = rmax_r.as<uint32_t>();
        a.meta = meta.as<float>();
        a.met16 = met16;
        amax = std::max(am, amax);
      }
      a.q8ok = q8ok;
      // the cached per-row terms stay current: the kernel writes these rows' terms too
      const bool mub_ok = f16 && mub_gen == g0 && mub.n >= sizeof(float) * cap;
      if (mub_ok) {
        a.mub = mub.as<float>();
        a.mkr = mub_kr;
        a.mkx = mub_kx;
        a.mmet = mub_met;
      }
      {
        WSec sec_l(3);
        launch_write_small(a, st, inline_rows ? &inl : nullptr);
        HIPCHK(hipGetLastError());
      }
      WSec sec_d(4);
      if (slot >= 0) ring.done(slot, st);
      if (mub_ok) mub_gen = gen;
      return true;
    }
  }
  const size_t xb = sizeof(float) * cnt * dim;
  stage_i.ensure(sizeof(int64_t) * cnt * 2);
  int64_t *di = stage_i.as<int64_t>();
  const float *src = x;
  if (!x_dev) {
    stage_x.ensure(xb);
    HIPCHK(hipMemcpyAsync(stage_x.p, x, xb, hipMemcpyHostToDevice, st));
    src = stage_x.as<float>();
  }
  HIPCHK(hipMemcpyAsync(di, slots, sizeof(int64_t) * cnt, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(di + cnt, labs, sizeof(int64_t) * cnt, hipMemcpyHostToDevice, st));
  launch_scatter_blocked(src, di, cnt, dim, rows.as<float>(), st);
  if (f16) launch_scatter_rowmajor(src, di, cnt, dim, rrm.as<float>(), st);
  launch_scatter_i64(labels.as<int64_t>(), di, di + cnt, cnt, st);
  launch_scatter_u8(live.as<uint8_t>(), di, 1, cnt, st);
  if (cosine) launch_norms_slots(rows.as<float>(), di, cnt, dim, norms.as<float>(), st);
  launch_sqnorms(rows.as<float>(), di, cnt, dim, rsq.as<float>(), rmax.as<uint32_t>(), st);
  HIPCHK(hipGetLastError());
  if (f16 && center16 && !resid) {
    // the first rows written fix the center: their mean (finite values), computed on the host (a device
    // source is read back once, for this first write only)
    std::vector<float> xh;
    if (x_dev) {
      xh.resize((size_t)cnt * dim);
      HIPCHK(hipMemcpyAsync(xh.data(), x, xb, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      x = xh.data();
    }
    std::vector<double> acc(dim, 0.0);
    std::vector<int64_t> num(dim, 0);
    for (int64_t i = 0; i < cnt; i++)
      for (int d = 0; d < dim; d++) {
        const float v = x[(size_t)i * dim + d];
        if (std::isfinite(v)) {
          acc[d] += v;
          num[d]++;
        }
      }
    std::vector<float> &c = hcenter;
    c.assign(dim, 0.0f);
    for (int d = 0; d < dim; d++) c[d] = num[d] ? (float)(acc[d] / (double)num[d]) : 0.0f;
    center_rows = std::max<int64_t>(n, 1);
    center.ensure(sizeof(float) * dim);
    rmax_r.ensure(sizeof(uint32_t));
    HIPCHK(hipMemcpyAsync(center.p, c.data(), sizeof(float) * dim, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(rmax_r.p, 0, sizeof(uint32_t), st));
    rsq16.grow_keep(sizeof(float) * cap, 0, st);
    resid = true;
    sx = 0.0f;  // encode every slot with the center (first write: the scale is set from these rows)
    amax = 0.0f;
  }
  encode16(di, cnt, st);
  HIPCHK(hipStreamSynchronize(st));  // staging buffers are reused by the next call
  if (stage_x.n > (size_t(256) << 20)) stage_x.release();  // bulk loads: do not pin GBs of staging
  return false;
}

void RowStore::set_live(const std::vector<int64_t> &slots, uint8_t v, hipStream_t st, DevMem &stage) {
  if (slots.empty()) return;
  ++gen;
  stage.ensure(sizeof(int64_t) * slots.size());
  HIPCHK(hipMemcpyAsync(stage.p, slots.data(), sizeof(int64_t) * slots.size(), hipMemcpyHostToDevice, st));
  launch_scatter_u8(live.as<uint8_t>(), stage.as<int64_t>(), v, (int64_t)slots.size(), st);
  if (f16) launch_meta16(stage.as<int64_t>(), (int64_t)slots.size(), met16, meta_norms(), live.as<uint8_t>(),
                         meta.as<float>(), st);
  HIPCHK(hipStreamSynchronize(st));
  for (int64_t s : slots) hlive[s] = v;
}


// One batch may repeat a label (an id upserted twice in one call): every occurrence maps to one
// slot and the reference applies the calls in order, so the LAST vector wins.  Earlier rows of a
// repeated slot are dropped here (scattered writes of several rows to one slot would race on the
// device).  The slot of each label stays the one its first occurrence got.  Returns false when
// nothing repeats (x, labels, n, slots untouched).
static bool keep_last_writes(const float *&x, const int64_t *&labels, int64_t &n, std::vector<int64_t> &slots,
                             int dim, int64_t nslots, std::vector<float> &xs, std::vector<int64_t> &ls) {
  if (n < 2) return false;
  std::vector<uint8_t> keep((size_t)n, 1);
  bool drop = false;
  if (n < 4096) {
    std::unordered_map<int64_t, int> hit;
    for (int64_t i = n - 1; i >= 0; i--)
      if (hit[slots[i]]++) keep[i] = 0, drop = true;
  } else {
    std::vector<uint8_t> hit((size_t)nslots, 0);
    for (int64_t i = n - 1; i >= 0; i--) {
      if (hit[slots[i]]) keep[i] = 0, drop = true;
      hit[slots[i]] = 1;
    }
  }
  if (!drop) return false;
  std::vector<int64_t> ss;
  for (int64_t i = 0; i < n; i++) {
    if (!keep[i]) continue;
    xs.insert(xs.end(), x + i * dim, x + (i + 1) * dim);
    ls.push_back(labels[i]);
    ss.push_back(slots[i]);
  }
  slots.swap(ss);
  x = xs.data();
  labels = ls.data();
  n = (int64_t)ls.size();
  return true;
}

// ---------------------------------------------------------------------------
// Index base
// ---------------------------------------------------------------------------
Index::Index(const pyr_index_desc &d) : desc(d), dim(d.dim), metric(d.metric), device(d.device) {
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&wst, hipStreamNonBlocking));
}

Index::~Index() {
  (void)hipSetDevice(device);
  if (wst) (void)hipStreamSynchronize(wst);
  if (wev) (void)hipEventDestroy(wev);
  free_ws.clear();
  stream_ws.clear();
  if (wst) (void)hipStreamDestroy(wst);
}

void Index::note_write() {
  if (!wev) HIPCHK(hipEventCreateWithFlags(&wev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(wev, wst));
  ++wgen;
}

void Index::order_after_writes(Workspace &ws) {
  if (ws.wgen_seen == wgen || !wev) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(ws.st, &cs));
  if (cs == hipStreamCaptureStatusActive) HIPCHK(hipEventSynchronize(wev));  // (no cross-capture event edge)
  else HIPCHK(hipStreamWaitEvent(ws.st, wev, 0));
  ws.wgen_seen = wgen;
}

std::unique_ptr<Workspace> Index::take_ws() {
  std::unique_ptr<Workspace> w;
  {
    std::lock_guard<std::mutex> g(ws_mu);
    if (!free_ws.empty()) {
      w = std::move(free_ws.back());
      free_ws.pop_back();
    }
  }
  if (!w) {
    w = std::make_unique<Workspace>();
    HIPCHK(hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking));
    w->own_stream = true;
  }
  order_after_writes(*w);
  return w;
}

void Index::give_ws(std::unique_ptr<Workspace> w) {
  std::lock_guard<std::mutex> g(ws_mu);
  free_ws.push_back(std::move(w));
}

Workspace &Index::ws_for_stream(hipStream_t st) {
  Workspace *w;
  {
    std::lock_guard<std::mutex> g(ws_mu);
    auto &p = stream_ws[st];
    if (!p) {
      p = std::make_unique<Workspace>();
      p->st = st;
    }
    w = p.get();
  }
  order_after_writes(*w);
  return *w;
}

void Index::ivf_layout(int64_t *, int64_t *, uint8_t *, int64_t *total) const {
  (void)total;
  throw Error(PYR_E_STATE, "index kind has no IVF layout");
}
void Index::pq_state(float *, int32_t *, uint8_t *) const { throw Error(PYR_E_STATE, "index kind is not IVF_PQ"); }

Profiler &prof() {
  static Profiler p;
  return p;
}
void Profiler::drain() {
  for (auto &r : pending) {
    (void)hipEventSynchronize(r.b);
    float t = 0;
    if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) ms[r.phase] += t;
    calls[r.phase]++;
    work[r.phase] += r.work;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  pending.clear();
}
void Profiler::reset() {
  drain();
  for (int i = 0; i < PH_N; i++) ms[i] = 0, calls[i] = 0, work[i] = 0;
}
PhaseTimer::PhaseTimer(int ph, hipStream_t s, int64_t w) : phase(ph), st(s), work(w) {
  if (!prof().on) return;
  if (hipEventCreate(&a) == hipSuccess) (void)hipEventRecord(a, st);
}
PhaseTimer::~PhaseTimer() {
  if (!a) return;
  hipEvent_t b;
  if (hipEventCreate(&b) != hipSuccess) return;
  (void)hipEventRecord(b, st);
  std::lock_guard<std::mutex> g(prof().m);
  prof().pending.push_back({phase, a, b, work});
}

void fill_empty_results(float *d_s, int64_t *d_l, int32_t *d_c, int64_t nq, int k, hipStream_t st) {
  launch_fill_results(d_s, d_l, d_c, nq, k, st);
}

// ---------------------------------------------------------------------------
// helpers shared by the scans
// ---------------------------------------------------------------------------
struct ScanPlan {
  int chunk_rows = 0, nchunks = 0, nitems = 0, qchunk = QCHUNK;
};

static ScanPlan plan_flat(int64_t nrows, int64_t nq, int dim, int k, int max_parts, int qchunk = 0) {
  ScanPlan p;
  p.qchunk = qchunk > 0 ? qchunk : fast_path(dim, k) ? QCHUNK : QCHUNK_GENERIC;
  const int64_t nqc = (nq + p.qchunk - 1) / p.qchunk;
  // ~2048 items = 4 full rounds of 512 resident blocks (256 CUs x 2); rounding DOWN keeps the
  // item count at or below that: rounding up (e.g. 79 query groups x 26 chunks = 2054 items)
  // left a fifth round of 6 items that cost a whole item duration.  256-query items run one block
  // per CU: 1024 items = 4 rounds.
  int64_t want = std::max<int64_t>(1, (p.qchunk > QCHUNK ? 1024 : 2048) / nqc);
  want = std::min<int64_t>(want, std::max<int64_t>(1, nrows / 1024));
  want = std::min<int64_t>(want, max_parts);
  p.chunk_rows = (int)round_up((nrows + want - 1) / want, 32);  // whole fp16 tiles (filter16.hip)
  if (p.chunk_rows <= 0) p.chunk_rows = 32;
  p.nchunks = (int)((nrows + p.chunk_rows - 1) / p.chunk_rows);
  p.nitems = (int)(p.nchunks * nqc);
  return p;
}

// scan rows [0,nrows) of `rs` for all queries into partial slots q*nparts + part_off + c
static void flat_scan(const RowStore &rs, int64_t nrows, const ScanPlan &p, const float *d_q, const float *d_qn,
                      int64_t nq, int k, int V, int met, int nparts, int part_off, uint32_t key_base, Workspace &ws,
                      float *part_s, uint32_t *part_k, bool second = false, uint32_t *gthr = nullptr) {
  DevMem &items = second ? ws.items2 : ws.items;
  DevMem &nitems = second ? ws.nitems2 : ws.nitems;
  items.ensure(sizeof(ScanItem) * std::max(p.nitems, 1));
  nitems.ensure(sizeof(int32_t) * 16);  // the count + 9 queue bounds (ivf_scan_kernel)
  make_flat_items(items.as<ScanItem>(), nitems.as<int32_t>(), nrows, p.chunk_rows, nq, part_off, p.qchunk, ws.st);
  ScanArgs a{};
  a.rows = rs.rows.as<float>();
  a.live = rs.live.as<uint8_t>();
  a.rnorm = rs.cosine ? rs.norms.as<float>() : nullptr;
  a.queries = d_q;
  a.queries_t = ws.qt.as<float>();  // filled by prep_queries for the same d_q
  a.qnorm = d_qn;
  a.items = items.as<ScanItem>();
  a.n_items = nitems.as<int32_t>();
  a.qlist = nullptr;
  a.limits = nullptr;
  a.nparts = nparts;
  a.k = k;
  a.key_base = key_base;
  a.dim = rs.dim;
  a.part_s = part_s;
  a.part_k = part_k;
  a.gthr = gthr;
  launch_scan(a, met, V, p.nitems, ws.st);
}

// Per-query shared top-k bound of one search (ScanArgs::gthr), reset to -inf.
// PYR_GTHR=0 disables it (A/B measurement); results are identical either way.
static bool bounds_enabled() {
  const char *e = knob("PYR_GTHR");
  return !(e && atoi(e) == 0);
}
static uint32_t *shared_bounds(Workspace &ws, int64_t nq) {
  if (!bounds_enabled() || nq <= 0) return nullptr;
  ws.gthr.ensure(sizeof(uint32_t) * nq);
  WordFill z;
  z.add(ws.gthr.p, nq, score_key(-INFINITY));
  launch_fill_words(z, ws.st);
  return ws.gthr.as<uint32_t>();
}

// The per-slice counters of a stream search (work-list histograms, candidate counts and floors, the
// persistent-block item counters, the two certificate failure counts) reset by ONE kernel (WordFill).  A
// search must stay capturable into a hipGraph and replayable: hipMemsetAsync nodes of a captured graph
// write stale values from its second replay on in the HIP runtime PyTorch ships, which is what faulted the
// second replay of a captured FLAT search (scripts/diag/graph_memset.py; DESIGN.md §4 "hipGraph replays").
static WordFill stream_counters_fill(Workspace &ws, int64_t nq, int nlist) {
  ws.ivf_cnt.ensure(sizeof(int32_t) * std::max(nlist, 1));
  ws.ivf_fill.ensure(sizeof(int32_t) * std::max(nlist, 1));
  ws.scn.ensure(sizeof(int32_t) * std::max<int64_t>(nq, 1));
  ws.scf.ensure(sizeof(uint32_t) * std::max<int64_t>(nq, 1));
  ws.swork.ensure(sizeof(int32_t) * 16);
  ws.fail_cnt.ensure(sizeof(int32_t));
  ws.fail_cnt2.ensure(sizeof(int32_t));
  WordFill z;
  z.add(ws.ivf_cnt.p, nlist, 0);
  z.add(ws.ivf_fill.p, nlist, 0);
  z.add(ws.scn.p, nq, 0);
  z.add(ws.scf.p, nq, 0);
  z.add(ws.swork.p, 16, 0);  // two item counters, or two sets of 8 per-XCD queue counters (pq32)
  z.add(ws.fail_cnt.p, 1, 0);
  z.add(ws.fail_cnt2.p, 1, 0);
  return z;
}
static void reset_stream_counters(Workspace &ws, int64_t nq, int nlist) {
  launch_fill_words(stream_counters_fill(ws, nq, nlist), ws.st);
}
// the same words zeroed by the next coarse ranking's first launch (CoarseIndex::probe), or by a fill of their own
// right after it (flush_stream_counters): one launch less on the IVF search
static void defer_stream_counters(Workspace &ws, int64_t nq, int nlist) {
  ws.pz = stream_counters_fill(ws, nq, nlist);
  ws.pz_set = true;
}
static void flush_stream_counters(Workspace &ws) {
  if (ws.pz_set) launch_fill_words(ws.pz, ws.st);
  ws.pz_set = false;
}
// the device re-run's per-query unit counters (IvfRerunArgs::done): zeroed once when allocated, then left
// zero by every launch (each merge resets its query's)
static int32_t *rerun_done(Workspace &ws, int64_t max_fail) {
  const bool off = knob("PYR_RERUN_FUSED") && atoi(knob("PYR_RERUN_FUSED")) == 0;  // A/B: separate merge
  if (off) return nullptr;
  const size_t need = sizeof(int32_t) * (size_t)std::max<int64_t>(max_fail, 1);
  if (ws.rrdone.n < need) {
    ws.rrdone.ensure(need);
    WordFill z;
    z.add(ws.rrdone.p, (int64_t)(ws.rrdone.n / sizeof(int32_t)), 0);
    launch_fill_words(z, ws.st);
  }
  return ws.rrdone.as<int32_t>();
}
struct DeferredCounters {  // a deferred fill never outlives the search that set it (an exception included)
  Workspace &ws;
  ~DeferredCounters() { ws.pz_set = false; }
};

// IVF-PQ LUT list scan kernel: 2 = pq_adc4 (default, k <= 256), 0 = the first-cut pq_scan (PYR_PQ_ADC=0; A/B
// only, same results; also what a shape past pq_adc4's LDS takes: D > 2048 at k > 64, D > 4096)
static int pq_adc_mode() {
  const char *e = knob("PYR_PQ_ADC");
  return e ? atoi(e) : 2;
}

// ---------------------------------------------------------------------------
// Stream-and-emit scan + certified exact refine (scan.hip, stream16.hip, filter.hip).  Same results as
// the exact scans (certified per query, failures re-run exactly on the device); PYR_FILTER=0 forces the
// exact scans, PYR_FILTER_MARGIN sets the minimum K1 - k (default 4, see filter_k1).
// ---------------------------------------------------------------------------
static bool filter_enabled() {
  const char *e = knob("PYR_FILTER");
  return !(e && atoi(e) == 0);
}
// fp16 tiles are kept where the stream scan can use them (L2 / IP, tile dims up to 768)
static bool store16(int dim, int metric) { return (metric == L2 || metric == IP) && scan_tile_dim(dim) > 0; }
// the tile dimension of a store of dim (zero-padded for the stream scan)
static int store16_dt(int dim) { return scan_tile_dim(dim); }
// the query operands and the sample of the stream scan: at tile dim = dim = 32 / 64 / 128 sprep + the
// 8-wave sample (sample16.hip), which shares each sampled tile across the item's queries through LDS
// (0.15 ms at I1); elsewhere scan.hip's one-wave-per-32-queries sample (0.29 ms at I1: every group
// re-reads the sampled tiles).  Both write the same bq / qsc / samp.  PYR_SCAN_SAMPLE=1: scan.hip's
// sample at every dim (measurement only).
// prep_only: the operands without the sample where the native-dim pass allows it (the one-wave pass writes
// both; its sample values are then simply not read)
// Round 5: at those dims the sample itself runs on the main scan kernel (scan.hip SMP: 16 waves, one sampled
// tile each, 32x32x16 MFMAs, every query group of the item) after sprep's operands; PYR_SAMPLE16=1 keeps
// sample16_kernel (A/B: both write the same samp layout; T_q may differ in its last bits, the answers do not).
static void stream_sample(const StreamArgs &sa, int met, int maxi, hipStream_t st, bool prep_only = false) {
  const char *e = knob("PYR_SCAN_SAMPLE");
  const int dt = sa.dt > 0 ? sa.dt : sa.dim;
  const bool s16 = knob("PYR_SAMPLE16") && atoi(knob("PYR_SAMPLE16")) == 1;
  if (!(e && atoi(e) == 1) && dt == sa.dim && sample16_supported(sa.dim, met)) {
    if (s16 || !scan_sample_mode_supported(dt)) {
      launch_sample16(sa, met, maxi, st, prep_only);
    } else {
      launch_sample16(sa, met, maxi, st, true);  // the operands only
      if (!prep_only) launch_scan_sample_mode(sa, met, maxi, st);
    }
  } else {
    launch_scan_sample(sa, met, maxi, st);
  }
}
// T_q = the R-th largest sample value.  Any R is correct (rows below T_q are represented by floor
// placeholders at T_q and the certificate decides); R trades emitted rows against queries with fewer
// than k real candidates.  The sample holds a fraction f of a query's probed rows (I1: ~5 %), so about
// R / f rows reach T_q, and a query falls short of K1 = 16 only when R of its 15 best rows were
// sampled: P ~ C(15, R) f^R, 7.8e-5 at R = 6, f = 0.05.  Short lists sample most of their rows
// (f -> 1): there a small R leaves ~R real candidates, below k, and every such query fails its
// certificate -- so R = clamp(ceil(6 K1 f), 3 K1 / 8, K1) per query (sselect_kernel): ~6 K1 emitted rows
// at small f, R = K1 once f >= 1/6.  Every emitted row costs the scan a wave-uniform branch and an LDS
// atomic: at I1, R = 8 -> 6 cuts the scan from 0.904 to 0.853 ms with no re-run, R = 5 re-runs 9 of 10,000
// queries (+0.16 ms), R = 4 51 (+0.55 ms) (profiles/r4_scan/sweep_sample_rank*.log).  PYR_STREAM_RANK
// fixes R.
static void stream_rank(int k1, int32_t &rmin, int32_t &rmax, double &et) {
  if (const char *e = knob("PYR_STREAM_RANK")) {
    rmin = rmax = std::max(1, atoi(e));
    et = 0.0;
    return;
  }
  // PYR_STREAM_RMIN / PYR_STREAM_ET (measurement only): the floor of R and the emitted-row target per K1
  // Deep K1 (128 / 256 / 512, k > 60): 3 K1 rows and R >= K1 / 8 -- a query's 1,024 sample values give a
  // threshold that close to its K1-th row without short queries (round 5's 6 K1 and 3 K1 / 8 emitted ~3,700 rows
  // per query at K1 = 512, and the emission set the scan's cost: 4.2 of a k = 256 search's 5.8 ms at I1)
  const bool deep = k1 > STREAM_KO;
  const char *rm = knob("PYR_STREAM_RMIN"), *ev = knob("PYR_STREAM_ET");
  rmin = std::max(1, rm ? atoi(rm) : deep ? k1 / 8 : (3 * k1 + 7) / 8);
  rmax = std::max(rmin, k1);
  et = (ev ? atof(ev) : deep ? 3.0 : 6.0) * k1;
}
// candidate buffer per query (PYR_STREAM_CAP; a query emits ~6 K1 rows, 96 at I1: a full buffer only
// raises its floor, and the certificate decides) and rows per list chunk (PYR_STREAM_CHUNK)
static int stream_cap() {
  const char *e = knob("PYR_STREAM_CAP");
  return e ? std::max(8, atoi(e)) : 2048;
}
static int64_t stream_chunk() {
  const char *e = knob("PYR_STREAM_CHUNK");
  return round_up(e ? std::max<int64_t>(32, atoll(e)) : 5120, 32);
}

// Queries per slice of a stream search: the per-query buffers (candidate buffer, counts, merged candidates,
// fail lists, thresholds) and the per-(query, probe) ones (fp16 query operands of the tile dimension, their
// scale pair, the sample values, the probe id and work-list slot) stay within 16 GiB (the
// per-position buffers dominate at many probes, e.g. a FLAT store of 1,000 chunks).
static int64_t stream_slice_queries(int64_t nq, int probes, int dt, int cap, int sv) {
  const int64_t per_q = (int64_t)cap * 8 + 8 + 8 * STREAM_KO + 16 + (int64_t)probes * (2 * dt + 8 + 4 * sv + 8);
  int64_t qs = (int64_t(16) << 30) / per_q;
  if (const char *e = knob("PYR_SLICE_QUERIES")) qs = std::min<int64_t>(qs, atoll(e));  // tests: force slicing
  return std::max<int64_t>(1, std::min<int64_t>(nq, qs));
}

// HBM plan of an IVF_FLAT index and of one stream-path search on it (pyr_ivf_memory_plan): the
// allocations commit_lists and search_stream / stream_slice make, restated as arithmetic so that a
// multi-GPU launch can size a rank before it allocates (the M8 rank shape: tests/test_dist.py).  These are
// steady-state bytes: building a shard holds the new list store beside the old one plus the row-major and
// blocked temporaries of every row (dist.rank_build_peak_bytes).
void ivf_memory_plan(int dim, int64_t nrows, int nlist, int64_t max_len, int64_t nq, int nprobe, int k,
                     int64_t *index_bytes, int64_t *workspace_bytes) {
  const int64_t D = dim, DT = std::max(dim, scan_tile_dim(dim));  // DT: the fp16 tiles' (padded) dimension
  const int64_t slots = round_up(nrows, 32) + (int64_t)nlist * 32;  // lists padded to 32-row tiles
  // rows (blocked fp32) + row-major fp32 copy + fp16 tiles + meta, row terms, |x|^2, |x - c|^2, live, label
  const int64_t per_row = 4 * D + 4 * D + 2 * DT + 4 + 4 + 4 + 4 + 1 + 8;
  const int64_t cent = (int64_t)nlist * (D * 4 * 3 + 4 * 6 + 8);  // centroids (blocked, row-major, unit), per-list
  if (index_bytes) *index_bytes = slots * per_row + cent;
  if (!workspace_bytes) return;
  const int probes = std::max(0, std::min(nprobe, nlist));
  // search_stream: chunking and the 16 GiB slice of candidate buffers
  const int cap = stream_cap();
  IvfChunking ch{(int32_t)stream_chunk(), 1, 0};
  ch.cmax = ivf_list_chunks((int)max_len, ch);
  if ((int64_t)probes * ch.cmax > MAX_PARTS) {
    const int64_t room = std::max<int64_t>(1, MAX_PARTS / std::max(probes, 1));
    ch.chunk = (int32_t)round_up(std::max<int64_t>(32, (max_len + room - 1) / room), 32);
    ch.cmax = ivf_list_chunks((int)max_len, ch);
  }
  const int64_t nparts = (int64_t)probes * ch.cmax;
  const int64_t qs = stream_slice_queries(nq, probes, (int)DT, cap, scan_sample_values());
  int64_t w = 0;
  // coarse ranking: probe lists of the whole batch, <= 256 MB of centroid scores per launch
  w += 4 * nq * probes;
  const int64_t qb = std::max<int64_t>(1, std::min<int64_t>(int64_t(1) << 21, (int64_t(1) << 26) / std::max(nlist, 1)));
  w += 4 * std::min(nq, qb) * nlist + 4 * std::min(nq, qb);
  // per slice (the buffers are sized for the largest slice and reused)
  const int64_t npos = qs * probes;
  (void)nparts;
  w += (int64_t)sizeof(ScanItem) * ivf_max_items(qs, probes, nlist, scan_qmax(DT), ch, 0) + 4 * npos +
       16 * ((int64_t)nlist + 1);
  w += 2 * npos * DT + 8 * npos + 4 * npos * scan_sample_values() + 4 * qs;  // query operands, samples, T_q
  w += 8 * qs * cap + 8 * qs;                                                  // candidate buffers + counts/floors
  w += 8 * qs * STREAM_KO + 16 * qs;                                           // merged candidates, fail lists
  w += 8 * ivf_rerun_part_keys(qs, probes, k);                                 // device re-run scratch
  *workspace_bytes = w;
}
// measurement only (PYR_STREAM_EMIT_ALL=1; tests/test_gpu_bounds.py): the main list scans run without the
// sampled thresholds, so every visible row of the scanned lists is emitted with its upper bound (with a
// PYR_STREAM_CAP large enough, pyr_index_debug_candidates then returns every row's bound)
static bool emit_all() {
  const char *e = knob("PYR_STREAM_EMIT_ALL");
  return e && atoi(e) != 0;
}
static StreamArgs main_scan_args(const StreamArgs &sa) {
  StreamArgs m = sa;
  if (emit_all()) m.thr = nullptr;
  return m;
}
// (concurrent searches hold the index shared: the three fields are written and read together under ws_mu)
void Index::note_stream_slice(Workspace &ws, int64_t nq, int cap) {
  std::lock_guard<std::mutex> g(ws_mu);
  dbg_ws = &ws;
  dbg_nq = nq;
  dbg_cap = cap;
}
void Index::debug_candidates(int64_t nq, int32_t cap, float *h_ub, int64_t *h_label, int32_t *h_cnt) {
  Workspace *w;
  {
    std::lock_guard<std::mutex> g(ws_mu);
    if (!dbg_ws) throw Error(PYR_E_STATE, "no stream-scan search ran on this index");
    if (nq != dbg_nq || cap != dbg_cap) throw Error(PYR_E_ARG, "nq / cap differ from the last stream-scan slice");
    w = dbg_ws;
  }
  Workspace &ws = *w;
  HIPCHK(hipStreamSynchronize(ws.st));
  std::vector<uint2> c((size_t)nq * cap);
  HIPCHK(hipMemcpy(c.data(), ws.scand.p, sizeof(uint2) * c.size(), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(h_cnt, ws.scn.p, sizeof(int32_t) * nq, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < c.size(); ++i) {
    uint32_t b = c[i].x;
    memcpy(&h_ub[i], &b, 4);
    h_label[i] = key_label(c[i].y);
  }
}
static int filter_ablate() {  // measurement only (StreamArgs::ablate)
  const char *e = knob("PYR_FILTER_ABLATE");
  return e ? atoi(e) : 0;
}
// K1 = candidates per query: the smallest register-list capacity (16, 32, 64) leaving at
// least 4 candidates beyond k (PYR_FILTER_MARGIN overrides the 4); 0 = filter unavailable
static int filter_k1(int k) {
  int m = 4;
  if (const char *e = knob("PYR_FILTER_MARGIN")) m = std::max(0, atoi(e));
  for (int c : {16, 32, 64})
    if (k + m <= c) return c;
  return 0;
}
// error-bound constant of the refine certificate (filter.hip refine_kernel); PYR_FILTER_CERR
// overrides it for tests (a huge value fails every certificate -> every query re-runs exactly)
static double filter_cerr(int dim) {
  if (const char *e = knob("PYR_FILTER_CERR")) return atof(e);
  return 4.0 * dim + 64.0;
}

// Cosine over a unit-row L2 store (FlatIndex::search_cosine_stream): the candidates are re-scored with
// the reference Cosine on the raw rows of the index itself, and the certificate is taken in cosine units
struct CosRefine {
  const RowStore *raw;     // the Cosine index's store (raw rows, norms, labels, non-finite flag)
  const float *queries;    // raw queries
  const float *qnorm;      // ComputeNorm per query
  const uint32_t *zflag;   // a zero-norm row was written
  // k > 60: the Cosine index's exact scan of n raw queries (the deep refine's certificate failures)
  std::function<void(const float *, int64_t, float *, int64_t *, int32_t *)> exact;
};

// the stream scans' candidate merge and certified refine fused into one kernel (filter.hip
// merge_refine_kernel); PYR_MERGE_REFINE=0 (A/B) and PYR_STREAM_DEBUG (it reads the merged candidates back)
// take cand_merge + the two refine launches
// the candidate buffer per query of a deep (K1 > 64) search: a query emits ~7.5 K1 rows at I1 (T_q's floor
// rank 3 K1 / 8 over a ~5 % sample), so 16 K1 keeps a full buffer rare (its floor would fail the certificate)
static int deep_cap(int k1) { return std::max(stream_cap(), 16 * k1); }
// PYR_DEEP_REFINE=0: an IVF search with k > 60 takes the exact scan (A/B; read per search)
static bool deep_refine_on() {
  const char *e = knob("PYR_DEEP_REFINE");
  return !(e && atoi(e) == 0);
}
// the refine depth for k > 60 (deep_refine_kernel): 128 / 256 >= k + the margin, 0 past that or when the
// candidate buffer's sort would not fit 60 KiB of LDS
// IVF_PQ (pq = true): k within K1 / 2 -- its fp16 decode filter bounds the ADC sum more loosely than the IVF_FLAT
// tiles bound the exact score (k = 100 at depth 128 failed ~5 % of the queries, profiles/r6_pqdeep)
static int deep_k1(int k, bool pq = false) {
  int m = 4;
  if (const char *e = knob("PYR_FILTER_MARGIN")) m = std::max(0, atoi(e));
  // k within 0.8 K1: k = 200 at depth 256 failed 2,453 of 10,000 I1 queries, k = 252 at 256 nearly all
  // (profiles/r5_late/deepk_ab.log)
  for (int c : {128, 256, 512})
    if (k + m <= c && (pq ? 2 * k <= c || c == 512 : 5 * k <= 4 * c))
      return deep_refine_lds_bytes(deep_cap(c), c) <= 144 * 1024 ? c : 0;
  return 0;
}

// PYR_MAXSCANS_STREAM=0: an IVF search with a MaxScans budget takes the exact scan (A/B; read per search)
static bool max_scans_stream() {
  const char *e = knob("PYR_MAXSCANS_STREAM");
  return !(e && atoi(e) == 0);
}

// PYR_IVF_BUFFER_STREAM=0: an IVF_FLAT search with a non-empty buffer takes the exact scan (A/B; read per search)
static bool buffer_stream() {
  const char *e = knob("PYR_IVF_BUFFER_STREAM");
  return !(e && atoi(e) == 0);
}

static bool merge_refine_fused() {
  const char *e = knob("PYR_MERGE_REFINE");
  return !(e && atoi(e) == 0) && !knob("PYR_STREAM_DEBUG");
}

// list-sharded search (IvfFlatIndex::shard_search, shard.hip): a slice's thresholds T_q (from the home
// ranks' plans) and its record output (exact local top-k + the bound of the rows left out, per query)
struct ShardCtx {
  const float *thr;
  uint8_t *rec;
  const int32_t *rem = nullptr;  // MaxScans: the plans' remaining budgets per (query, probe), row stride rstride
  int rstride = 0;
};

// re-run the listed queries through the exact scan and put their rows in place
template <class F>
static void filter_fallback(Workspace &ws, int64_t nf, const float *d_q, int dim, int k, float *d_s, int64_t *d_l,
                            int32_t *d_c, F &&exact) {
  if (nf <= 0) return;
  PhaseTimer t(PH_FALLBACK, ws.st, nf);
  ws.fq.ensure(sizeof(float) * nf * dim);
  ws.fs.ensure(sizeof(float) * nf * k);
  ws.fl.ensure(sizeof(int64_t) * nf * k);
  ws.fc.ensure(sizeof(int32_t) * nf);
  launch_gather_queries(d_q, ws.fail.as<int32_t>(), nf, dim, ws.fq.as<float>(), ws.st);
  exact(ws.fq.as<float>(), nf, ws.fs.as<float>(), ws.fl.as<int64_t>(), ws.fc.as<int32_t>());
  launch_scatter_results(ws.fail.as<int32_t>(), nf, k, ws.fs.as<float>(), ws.fl.as<int64_t>(), ws.fc.as<int32_t>(),
                         d_s, d_l, d_c, ws.st);
}

// per-batch query preparation shared by every scan of one search: cosine norms, and the
// lane-major copy the fast scan kernel loads its query registers from
static void prep_queries(const float *d_q, int64_t nq, int dim, int met, Workspace &ws) {
  if (met == COS) {
    ws.qn.ensure(sizeof(float) * std::max<int64_t>(nq, 1));
    launch_norms(d_q, nq, dim, 0, ws.qn.as<float>(), ws.st);
  }
  if (fast_path(dim, 1) && nq > 0) {
    ws.qt.ensure(sizeof(float) * nq * dim);
    launch_transpose_queries(d_q, nq, dim, ws.qt.as<float>(), ws.st);
  }
}

// ---------------------------------------------------------------------------
// k-means on the GPU (KMeansUtils.cs:10-68)
// ---------------------------------------------------------------------------

void assign_gpu(const float *d_x, int64_t n, int dim, const float *d_cents, int k, int met, int32_t *d_assign,
                hipStream_t st) {
  if (n <= 0) return;
  // centroid store (blocked) as the scanned rows; data rows as the queries; top-1 with ties -> lowest index
  RowStore cs;
  cs.dim = dim;
  cs.cosine = met == COS;
  cs.reserve(round_up(k, 8), st);
  launch_to_blocked(d_cents, nullptr, k, dim, cs.rows.as<float>(), 0, st);
  fill_u8(cs.live.as<uint8_t>(), 1, k, st);
  if (cs.cosine) launch_norms(cs.rows.as<float>(), k, dim, 1, cs.norms.as<float>(), st);
  Workspace ws;
  ws.st = st;
  prep_queries(d_x, n, dim, met, ws);
  ScanPlan p;
  p.qchunk = fast_path(dim, 1) ? QCHUNK : QCHUNK_GENERIC;
  p.chunk_rows = (int)round_up(k, 8);
  p.nchunks = 1;
  p.nitems = (int)((n + p.qchunk - 1) / p.qchunk);
  DevMem ps, pk;
  ps.ensure(sizeof(float) * n);
  pk.ensure(sizeof(uint32_t) * n);
  flat_scan(cs, k, p, d_x, met == COS ? ws.qn.as<float>() : nullptr, n, 1, 1, met, 1, 0, 0, ws, ps.as<float>(),
            pk.as<uint32_t>());
  launch_keys_to_assign(pk.as<uint32_t>(), n, d_assign, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
}

int kmeans_train_gpu(const float *d_x, int64_t n, int dim, int k, int met, int max_iter, int seed, float *d_cents,
                     hipStream_t st) {
  if (n == 0) return 0;                      // :12
  if (k <= 0) k = 1;                         // :13
  if (k > n) k = (int)n;                     // :14
  // :20 data.OrderBy(_ => rnd.Next()).Take(k): one Next() per row in row order, stable by (key, row)
  NetRandom rnd(seed);
  std::vector<std::pair<int32_t, int32_t>> keys((size_t)n);
  for (int64_t i = 0; i < n; i++) keys[i] = {rnd.next(), (int32_t)i};
  std::partial_sort(keys.begin(), keys.begin() + k, keys.end());
  std::vector<int32_t> init(k);
  for (int i = 0; i < k; i++) init[i] = keys[i].second;
  keys.clear();
  keys.shrink_to_fit();
  DevMem didx;
  didx.ensure(sizeof(int32_t) * k);
  HIPCHK(hipMemcpyAsync(didx.p, init.data(), sizeof(int32_t) * k, hipMemcpyHostToDevice, st));
  launch_gather_rows(d_x, didx.as<int32_t>(), k, dim, d_cents, st);

  DevMem assign, ktmp, iin, members, counts, coff, temp, tmp, flags, changed;
  assign.ensure(sizeof(int32_t) * n);
  ktmp.ensure(sizeof(int32_t) * n);
  iin.ensure(sizeof(int32_t) * n);
  members.ensure(sizeof(int32_t) * n);
  counts.ensure(sizeof(int32_t) * (k + 1));
  coff.ensure(sizeof(int32_t) * (k + 1));
  const size_t tb = sort_temp_bytes(n, k);
  temp.ensure(tb);
  tmp.ensure(sizeof(float) * k * dim);
  flags.ensure(sizeof(int32_t) * k);
  changed.ensure(sizeof(int32_t));
  for (int it = 0; it < max_iter; it++) {     // :22
    assign_gpu(d_x, n, dim, d_cents, k, met, assign.as<int32_t>(), st);  // :34-38
    sort_by_key(assign.as<int32_t>(), n, k, ktmp.as<int32_t>(), iin.as<int32_t>(), members.as<int32_t>(),
                counts.as<int32_t>(), coff.as<int32_t>(), temp.p, tb, st);  // :40-43 members in data order
    launch_kmeans_update(d_x, members.as<int32_t>(), coff.as<int32_t>(), k, dim, d_cents, tmp.as<float>(),
                         flags.as<int32_t>(), changed.as<int32_t>(), st);  // :46-62
    int32_t ch = 0;
    HIPCHK(hipMemcpyAsync(&ch, changed.p, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (!ch) break;                            // :64
  }
  return k;
}


// ---------------------------------------------------------------------------
// index images (IVectorIndex.Snapshot / Load; persist.h)
// ---------------------------------------------------------------------------
static void check_image(const ImageReader &r, int kind, const Index &ix) {
  if (r.kind != kind) throw Error(PYR_E_FORMAT, "the image holds another index kind");
  if (r.dim != ix.dim)
    throw Error(PYR_E_FORMAT, "the image has dimension " + std::to_string(r.dim) + ", the index " + std::to_string(ix.dim));
  // the metric is recorded but, like the reference's IvfStateDto.Metric (IvfFlatVectorIndex.cs:259-
  // 298 never reads it), not enforced: rows are re-derived (norms, |x|^2) for the loading index
  (void)ix.metric;
}

// rows at `slots` of a blocked store -> row-major device rows in stage_x (slot order)
static void gather_slots(const RowStore &s, const std::vector<int64_t> &slots, DevMem &stage_x, DevMem &stage_i,
                         hipStream_t st) {
  const int64_t n = (int64_t)slots.size();
  stage_x.ensure(sizeof(float) * std::max<int64_t>(n, 1) * s.dim);
  if (n == 0) return;
  stage_i.ensure(sizeof(int64_t) * n);
  HIPCHK(hipMemcpyAsync(stage_i.p, slots.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, st));
  launch_gather_blocked(s.rows.as<float>(), stage_i.as<int64_t>(), n, s.dim, stage_x.as<float>(), st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
}

// the live slots of a store in slot order (BruteForce _vectors / Dictionary enumeration order)
static std::vector<int64_t> live_slots(const RowStore &s, std::vector<int64_t> &labels) {
  std::vector<int64_t> slots;
  for (int64_t i = 0; i < s.n; i++)
    if (s.hlive[i]) {
      slots.push_back(i);
      labels.push_back(s.hlabels[i]);
    }
  return slots;
}

static void write_rows(ImageWriter &w, uint32_t tag_labels, uint32_t tag_rows, const RowStore &s,
                       const std::vector<int64_t> &slots, const std::vector<int64_t> &labels, DevMem &stage_x,
                       DevMem &stage_i, hipStream_t st) {
  w.host(tag_labels, labels.data(), sizeof(int64_t) * labels.size());
  gather_slots(s, slots, stage_x, stage_i, st);
  w.device(tag_rows, stage_x.p, sizeof(float) * slots.size() * s.dim, st);
}

// labels + host rows of a (labels, rows) section pair; absent sections = no rows
static int64_t read_rows(ImageReader &r, uint32_t tag_labels, uint32_t tag_rows, int dim, std::vector<int64_t> &labels,
                         std::vector<float> &rows) {
  labels = r.vec<int64_t>(tag_labels);
  const int64_t n = (int64_t)labels.size();
  rows.assign((size_t)n * dim, 0.0f);
  if (n) r.host(tag_rows, rows.data(), sizeof(float) * rows.size());
  return n;
}

// ---------------------------------------------------------------------------
// FLAT = BruteForceVectorIndex (BruteForceVectorIndex.cs)
// ---------------------------------------------------------------------------
static int build_ivf_items(Workspace &ws, int64_t nq, int nprobe, int nparts, int nlist, const DevMem &lbeg,
                           const DevMem &lend, int qchunk, IvfChunking ch, int phase = 0, bool balance = false,
                           bool zeroed = false);

struct FlatIndex : Index {
  RowStore st;
  int64_t key_label(uint32_t key) const override {
    return (int64_t)key < st.n && st.hlive[key] ? st.hlabels[key] : -1;
  }
  std::unordered_map<int64_t, int64_t> slot_of;  // _idMap (:15)
  // 8-bit search mode (EnableQuantization, :25-40; _quantizedVectors, :20-21): per slot
  // ScalarQuantizer codes + sums of squares, and whether the slot has codes at all
  bool quant = false;
  DevMem q8, q8s, q8ok;
  int64_t q8cap = 0;
  int dp;
  // VectorMath form of the exact scores: 4 = the *Unsafe forms of BruteForceVectorIndex; 1 = the safe
  // forms (ComputeScore of the IVF coarse step, when this store holds an index's centroids)
  int exact_v = 4;

  // Cosine on the filter path: an L2 FLAT index over the unit rows x / |x| of the same slots (its labels
  // are the slots), searched with the unit queries; its exact top-K2 are the candidates whose exact
  // Cosine (:354) cos_rerank_kernel ranks and certifies (filter.hip).  zflag: a zero-norm row was written
  std::unique_ptr<FlatIndex> unit;
  DevMem zflag;

  explicit FlatIndex(const pyr_index_desc &d) : Index(d) {
    st.dim = dim;
    st.cosine = metric == COS;  // norm cached at Add (:146)
    st.f16 = store16(dim, metric);
    st.dt = st.f16 ? store16_dt(dim) : 0;
    st.center16 = st.f16 && metric == L2;  // fp16 tiles of x - mean (engine.h RowStore)
    st.met16 = metric;
    dp = sq8_dp(dim);
    if (metric == COS && store16(dim, L2)) unit_reset();
  }
  void unit_reset() {
    pyr_index_desc u = desc;
    u.metric = L2;
    unit = std::make_unique<FlatIndex>(u);
    zflag.ensure(sizeof(uint32_t));
    HIPCHK(hipMemsetAsync(zflag.p, 0, sizeof(uint32_t), wst));
    HIPCHK(hipStreamSynchronize(wst));
  }
  // the unit rows of the slots just written (device norms: the reference's ComputeNorm and its 1e-6 rule)
  void unit_write(int64_t n, const std::vector<int64_t> &slots) {
    if (!unit || n <= 0) return;
    stage_b.ensure(sizeof(float) * n * dim);
    launch_unit_rows(st.rows.as<float>(), stage_i.as<int64_t>(), st.norms.as<float>(), n, dim, stage_b.as<float>(),
                     wst, zflag.as<uint32_t>());
    // straight from stage_b into the unit store at the same slots (labels = slots), all on wst (no host
    // hop; write() synchronizes wst at its end): a batch with a repeated id keeps its rows out of slot
    // order, so the unit index's own append order could differ
    FlatIndex &u = *unit;
    int64_t next = u.st.n;
    for (int64_t s : slots) next = std::max(next, s + 1);
    u.st.reserve(next, wst);
    u.st.hlabels.resize(next, -1);
    u.st.hlive.resize(next, 0);
    u.st.write(stage_b.as<float>(), slots.data(), slots.data(), n, wst, u.stage_x, u.stage_i, true);
    for (int64_t s : slots) {
      u.st.hlabels[s] = s;
      u.st.hlive[s] = 1;
      u.slot_of[s] = s;
    }
    u.st.n = next;
  }

  void set_quantization(bool on) override { quant = on; }
  // the stream scan's per-row terms for the rows just written, on the write stream (a search -- or a
  // hipGraph capture of one -- right after a write then finds them current; FlatIndex::stream_slice's
  // constants)
  void after_write() override {
    if (st.f16 && st.cap > 0 && st.sx > 0.0f && st.mub_gen != st.gen) {  // (small writes keep them current)
      StreamArgs sa{};
      const int dt = st.tdim();
      stream_ub_terms(dt, metric, filter_f16_cerr(dt, metric, FILTER_F16X1), filter_cerr(dt),
                      filter_f16_abs(dt, metric, st.sx, FILTER_F16X1), sa);
      st.row_terms(metric, sa.kr, sa.kx, wst);
    }
    if (unit) unit->after_write();
  }
  // BruteForceVectorIndex.Build is a no-op for the results; here the FLAT L2 tiles are re-centred on the
  // live rows (a Delta head is built after its compaction, DeltaVectorIndex.cs:124-158)
  void build() override {
    if (st.center16 && st.resid && !knob("PYR_FROZEN_CENTER")) st.recenter(wst);
  }
  void reserve(int64_t rows) override {
    st.reserve(st.n + rows, wst);
    slot_of.reserve(slot_of.size() + (size_t)rows);
    if (unit) unit->reserve(rows);
  }

  void q8_reserve() {
    if (q8cap >= st.cap) return;
    const int64_t nc = st.cap;
    q8.grow_keep((size_t)dp * nc, (size_t)dp * q8cap, wst);
    q8s.grow_keep(sizeof(int2) * nc, sizeof(int2) * q8cap, wst);
    q8ok.grow_keep(nc, q8cap, wst);
    HIPCHK(hipMemsetAsync(q8ok.as<uint8_t>() + q8cap, 0, nc - q8cap, wst));
    q8cap = nc;
  }

  void add(const float *x, int64_t n, const int64_t *labels, bool upsert) override {
    std::vector<int64_t> slots(n);
    int64_t next = st.n;
    if (n == 1) {  // VEC.ADD's granularity: no per-call maps
      auto f = slot_of.find(labels[0]);
      if (f != slot_of.end() && !upsert)
        throw Error(PYR_E_DUPLICATE, "Vector with id '" + std::to_string(labels[0]) + "' already exists.");
      slots[0] = f != slot_of.end() ? f->second : next++;
    } else {
      if (!upsert) {  // :141-144 duplicate id -> InvalidOperationException
        std::unordered_map<int64_t, int> seen;
        for (int64_t i = 0; i < n; i++)
          if (slot_of.count(labels[i]) || seen[labels[i]]++)
            throw Error(PYR_E_DUPLICATE, "Vector with id '" + std::to_string(labels[i]) + "' already exists.");
      }
      std::unordered_map<int64_t, int64_t> batch;
      for (int64_t i = 0; i < n; i++) {
        auto f = slot_of.find(labels[i]);
        if (f != slot_of.end()) slots[i] = f->second;        // :193-210 update in place
        else {
          auto b = batch.find(labels[i]);
          slots[i] = b != batch.end() ? b->second : next++;  // :151-179 append slot
          batch[labels[i]] = slots[i];
        }
      }
    }
    std::vector<float> xs;
    std::vector<int64_t> ls;
    keep_last_writes(x, labels, n, slots, dim, next, xs, ls);
    st.reserve(next, wst);
    st.hlabels.resize(next, -1);
    st.hlive.resize(next, 0);
    q8_reserve();
    // :166-178 / :200-211: codes when quantization is on, otherwise the slot loses them.  A few rows of a
    // plain store go through RowStore::write's small-batch path (the q8ok reset fused in, no sync)
    const bool small = !quant && !unit && st.write(x, slots.data(), labels, n, wst, stage_x, stage_i, false,
                                                   q8ok.as<uint8_t>());
    if (!small) {
      if (quant || unit) st.write(x, slots.data(), labels, n, wst, stage_x, stage_i, false, nullptr, true);
      // (stage_i holds the device copy of the slots)
      if (quant)
        launch_sq8_quantize(st.rows.as<float>(), stage_i.as<int64_t>(), 1, n, dim, dp, 1, q8.as<uint8_t>(),
                            q8s.as<int2>(), q8ok.as<uint8_t>(), wst);
      else
        launch_scatter_u8(q8ok.as<uint8_t>(), stage_i.as<int64_t>(), 0, n, wst);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(wst));
      unit_write(n, slots);  // (stage_i: the slots; the unit index appends new slots in the same order)
    }
    for (int64_t i = 0; i < n; i++) {
      st.hlabels[slots[i]] = labels[i];
      st.hlive[slots[i]] = 1;
      slot_of[labels[i]] = slots[i];
    }
    st.n = next;
    // the FLAT L2 tiles' center follows the rows: re-centred each time the store has doubled since
    if (st.center16 && st.resid && st.n >= 2 * st.center_rows && !knob("PYR_FROZEN_CENTER")) st.recenter(wst);
  }

  // BruteForceVectorIndex.Search with EnableQuantization (:296-336): quantize the queries,
  // exact integer scores over slots [0, cutoff) that have codes
  void search_sq8(const float *d_q, int64_t nq, int k, int64_t cutoff, float *d_s, int64_t *d_l, int32_t *d_c,
                  Workspace &ws) {
    if (!sq8_supported(dim, k)) throw Error(PYR_E_ARG, "quantized search supports dim <= 512 and topK <= 64");
    // exact int8 MFMA scores (sq8.hip); items of 128 queries x 8192-row chunks
    ws.q8q.ensure((size_t)dp * nq);
    ws.q8qs.ensure(sizeof(int2) * nq);
    launch_sq8_quantize(d_q, nullptr, 0, nq, dim, dp, 1, ws.q8q.as<uint8_t>(), ws.q8qs.as<int2>(), nullptr, ws.st);
    int64_t chunk = 8192;
    while ((cutoff + chunk - 1) / chunk > MAX_PARTS) chunk *= 2;
    const int nchunks = (int)((cutoff + chunk - 1) / chunk);
    const int64_t nqc = (nq + sq8_qgroup() - 1) / sq8_qgroup();
    if (nqc * nchunks > INT32_MAX) throw Error(PYR_E_ARG, "query batch too large for one launch");
    const size_t np = (size_t)nq * nchunks * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    ws.items.ensure(sizeof(ScanItem) * std::max<int64_t>(nqc * nchunks, 1));
    ws.nitems.ensure(sizeof(int32_t) * 16);  // the count + 9 queue bounds (ivf_scan_kernel)
    const int ni = make_flat_items(ws.items.as<ScanItem>(), ws.nitems.as<int32_t>(), cutoff, (int32_t)chunk, nq, 0,
                                   sq8_qgroup(), ws.st);
    Sq8Args a{};
    a.codes = q8.as<uint8_t>();
    a.sums = q8s.as<int2>();
    a.live = st.live.as<uint8_t>();
    a.ok = q8ok.as<uint8_t>();
    a.qcodes = ws.q8q.as<uint8_t>();
    a.qsums = ws.q8qs.as<int2>();
    a.items = ws.items.as<ScanItem>();
    a.n_items = ws.nitems.as<int32_t>();
    a.nparts = nchunks;
    a.k = k;
    a.dim = dim;
    a.dp = dp;
    a.row_limit = (uint32_t)cutoff;
    a.part_s = ws.part_s.as<float>();
    a.part_k = ws.part_k.as<uint32_t>();
    {
      PhaseTimer t(PH_FLAT_SCAN, ws.st, nq * cutoff);
      launch_sq8_scan(a, metric == L2 ? L2 : IP, ni, ws.st);  // Cosine scores with DotProduct8Bit (:329)
    }
    PhaseTimer t(PH_MERGE, ws.st);
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, nchunks, k, st.labels.as<int64_t>(),
                      nullptr, d_s, d_l, nullptr, d_c, ws.st);
  }

  void remove(const int64_t *labels, int64_t n, uint8_t *removed) override {  // :224-248
    std::vector<int64_t> dead;
    for (int64_t i = 0; i < n; i++) {
      auto f = slot_of.find(labels[i]);
      if (removed) removed[i] = f != slot_of.end();
      if (f == slot_of.end()) continue;
      dead.push_back(f->second);
      slot_of.erase(f);
    }
    st.set_live(dead, 0, wst, stage_b);
    if (unit && !dead.empty()) unit->remove(dead.data(), (int64_t)dead.size(), nullptr);
  }

  void search(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, float *d_s, int64_t *d_l,
              int32_t *d_c, Workspace &ws) override {
    if (k <= 0) throw Error(PYR_E_ARG, "topK must be positive.");  // :278
    int64_t count = st.n;
    int64_t cutoff = count;  // :288 scanLimit = min(MaxScans, count), counted over live slots in order
    if (prm.max_scans >= 0) {
      if (prm.max_scans == 0) cutoff = 0;
      else {
        int64_t seen = 0;
        cutoff = count;
        for (int64_t i = 0; i < count; i++)
          if (st.hlive[i] && ++seen == prm.max_scans) {
            cutoff = i + 1;
            break;
          }
      }
    }
    if (count == 0 || cutoff == 0 || nq == 0) {  // :285, :289
      fill_empty_results(d_s, d_l, d_c, nq, k, ws.st);
      return;
    }
    if (quant) {  // :296
      search_sq8(d_q, nq, k, cutoff, d_s, d_l, d_c, ws);
      return;
    }
    int k1 = filter_k1(k);
    // k > 60: depth 128 / 256 / 512 (deep_refine_kernel; Cosine on the unit store with the exact Cosine)
    if (k1 == 0 && deep_refine_on()) k1 = deep_k1(k);
    if (flat_stream_ok(k, k1, cutoff)) {
      search_stream(d_q, nq, k, k1, cutoff, d_s, d_l, d_c, ws);
      return;
    }
    if (unit && metric == COS && unit->flat_stream_ok(k, k1, cutoff)) {
      search_cosine_stream(d_q, nq, k, k1, cutoff, d_s, d_l, d_c, ws);
      return;
    }
    search_exact(d_q, nq, k, cutoff, d_s, d_l, d_c, ws);  // the one fallback: the reference's arithmetic
  }

  // FLAT on the stream scan (scan.hip, round 4): slots [0, cutoff) cut into chunks that play the IVF
  // path's lists (every query probes all of them, their centroid the store's center: mu for L2, 0 for IP),
  // so the sample, the emit scan, the merge and the certified refine (the *Unsafe form, V = 4) run as
  // for IVF_FLAT, and the exact re-run of certificate failures stays on the device: no host round trip.
  // Anything else (k > 60, dims past 768, an L2 store without its centre) takes the exact scan.
  bool flat_stream_ok(int k, int k1, int64_t cutoff) const {
    if (!filter_enabled()) return false;
    if (metric != L2 && metric != IP) return false;
    if (!st.f16 || (k > KMAX_FAST && k1 <= STREAM_KO) || k1 <= 0 || !scan_supported(dim, metric, k1)) return false;
    if (metric == L2 && !(st.resid && st.center16)) return false;
    return cutoff > 0 && cutoff < (int64_t)KEY_BUF;
  }

  // the chunking of [0, cutoff): at most MAX_PARTS chunks of whole tiles, 10,240 rows where the store is
  // large (the sample scores the first 512 rows of each: 5 % of the rows).  A query emits about
  // R / f = R c / 512 rows in all (R <= K1 sample rank, f = 512 / c the sampled fraction), R c^2 / (512
  // cutoff) per chunk; a small store therefore takes chunks of ~sqrt(512 cutoff) rows so that a chunk's
  // region (stream_cap, 256) does not fill -- a full region's floor sits among the best rows and fails
  // the certificate (20,000 rows, k = 20: 7 % of queries with 10,240-row chunks).
  static int64_t flat_chunk_rows(int64_t cutoff) {
    const int64_t small = round_up((int64_t)std::sqrt(512.0 * (double)std::max<int64_t>(cutoff, 1)), 32);
    int64_t c = std::max<int64_t>(1024, std::min<int64_t>(10240, small));
    while ((cutoff + c - 1) / c > MAX_PARTS) c *= 2;
    return c;
  }
  // Cosine (:339-354) on the stream scan: the unit index's scan of the unit queries over the unit rows'
  // fp16 tiles (L2 bounds of -|q^ - x^|^2), the exact Cosine -- DotProductUnsafe / (|q| |x|) with the zero
  // rule -- of the candidates on the raw rows, certified in cosine units (refine_kernel, cosine), and the
  // exact Cosine re-run of failures on the device: no host round trip, as for L2 / IP
  void search_cosine_stream(const float *d_q, int64_t nq, int k, int k1, int64_t cutoff, float *d_s, int64_t *d_l,
                            int32_t *d_c, Workspace &ws) {
    ws.qn.ensure(sizeof(float) * std::max<int64_t>(nq, 1));
    launch_norms(d_q, nq, dim, 0, ws.qn.as<float>(), ws.st);  // VectorMath.ComputeNorm (:339)
    ws.cq.ensure(sizeof(float) * std::max<int64_t>(nq, 1) * dim);
    launch_unit_rows(d_q, nullptr, ws.qn.as<float>(), nq, dim, ws.cq.as<float>(), ws.st);
    CosRefine cr{&st, d_q, ws.qn.as<float>(), zflag.as<uint32_t>(), nullptr};
    cr.exact = [&](const float *q2, int64_t n2, float *s2, int64_t *l2, int32_t *c2) {
      search_exact(q2, n2, k, cutoff, s2, l2, c2, ws.nested());  // BruteForceVectorIndex.cs:354 on the raw rows
    };
    std::shared_lock<std::shared_mutex> g(unit->mu);
    unit->search_stream(ws.cq.as<float>(), nq, k, k1, cutoff, d_s, d_l, d_c, ws, &cr);
    // (measurement: the unit store's keys are this store's slots)
    if (unit->dbg_ws) note_stream_slice(*unit->dbg_ws, unit->dbg_nq, unit->dbg_cap);
  }

  void search_stream(const float *d_q, int64_t nq, int k, int k1, int64_t cutoff, float *d_s, int64_t *d_l,
                     int32_t *d_c, Workspace &ws, const CosRefine *cr = nullptr) {
    const int64_t crow = flat_chunk_rows(cutoff);
    const int nch = (int)((cutoff + crow - 1) / crow);
    const int cap = k1 > STREAM_KO ? deep_cap(k1) : stream_cap();
    const int nparts = nch;  // one chunk per "list"
    const int64_t qs = stream_slice_queries(nq, nch, st.tdim(), cap, scan_sample_values());
    // the chunks as lists, on the device (no host work per search): bounds, the centroid copies (mu for
    // L2, 0 for IP) and the probe lists (every chunk, in order) of the largest slice
    ws.vlb.ensure(sizeof(int32_t) * nch);
    ws.vle.ensure(sizeof(int32_t) * nch);
    ws.vcents.ensure(sizeof(float) * nch * dim);
    launch_chunk_lists(ws.vlb.as<int32_t>(), ws.vle.as<int32_t>(), nch, crow, cutoff,
                       metric == L2 ? st.center.as<float>() : nullptr, dim, ws.vcents.as<float>(), ws.st);
    for (int64_t a0 = 0; a0 < nq; a0 += qs) {
      const int64_t n = std::min(qs, nq - a0);
      if (cr) {  // the slice's raw queries and norms
        CosRefine c2 = *cr;
        c2.queries = cr->queries + a0 * dim;
        c2.qnorm = cr->qnorm + a0;
        stream_slice(d_q + a0 * dim, n, k, k1, cutoff, nch, nparts, cap, d_s + a0 * k, d_l + a0 * k,
                     d_c ? d_c + a0 : nullptr, ws, &c2);
      } else {
        stream_slice(d_q + a0 * dim, n, k, k1, cutoff, nch, nparts, cap, d_s + a0 * k, d_l + a0 * k,
                     d_c ? d_c + a0 : nullptr, ws);
      }
    }
  }

  void stream_slice(const float *d_q, int64_t nq, int k, int k1, int64_t cutoff, int nch, int nparts, int cap,
                    float *d_s, int64_t *d_l, int32_t *d_c, Workspace &ws, const CosRefine *cr = nullptr) {
    const int probes = nch;
    const IvfChunking ch{(int32_t)flat_chunk_rows(cutoff), 1, 0};
    reset_stream_counters(ws, nq, nch);
    ws.probes.ensure(sizeof(int32_t) * nq * probes);
    launch_iota_rows(ws.probes.as<int32_t>(), nq, probes, ws.st);
    DevMem &lbd = ws.vlb, &led = ws.vle;
    int maxi;
    {
      PhaseTimer t(PH_ITEMS, ws.st);
      maxi = build_ivf_items(ws, nq, probes, nparts, nch, lbd, led, scan_qmax(st.tdim()), ch, 0, true, true);
    }
    const int64_t npos = nq * probes;
    const int sv = scan_sample_values();
    ws.sbq.ensure(sizeof(uint16_t) * std::max<int64_t>(npos, 1) * st.tdim());
    ws.sqsc.ensure(sizeof(float2) * std::max<int64_t>(npos, 1));
    ws.ssamp.ensure(sizeof(float) * std::max<int64_t>(npos, 1) * sv);
    ws.sthr.ensure(sizeof(float) * nq);
    ws.scand.ensure(sizeof(uint2) * (size_t)std::max<int64_t>(nq, 1) * cap);
    ws.scn.ensure(sizeof(int32_t) * std::max<int64_t>(nq, 1));
    ws.scf.ensure(sizeof(uint32_t) * std::max<int64_t>(nq, 1));
    ws.swork.ensure(sizeof(int32_t) * 2);
    StreamArgs sa{};
    sa.h16 = st.h16.p;
    sa.meta = st.meta.as<float>();
    sa.queries = d_q;
    sa.cents = ws.vcents.as<float>();
    sa.sx = st.sx;
    sa.items = ws.items.as<ScanItem>();
    sa.n_items = ws.nitems.as<int32_t>();
    sa.qlist = ws.qlist.as<int32_t>();
    sa.qpos = ws.qpos.as<int32_t>();  // (build_ivf_items: every probe of every query)
    sa.probes = ws.probes.as<int32_t>();
    sa.nq = nq;
    sa.nparts = nparts;
    sa.nprobe = probes;
    sa.cmax = 1;
    sa.dim = dim;
    sa.dt = st.tdim();
    sa.bq = ws.sbq.as<_Float16>();
    sa.qsc = ws.sqsc.as<float2>();
    sa.samp = ws.ssamp.as<float>();
    sa.thr = ws.sthr.as<float>();
    sa.cand = ws.scand.as<uint2>();
    sa.cand_n = ws.scn.as<int32_t>();
    sa.cand_f = ws.scf.as<uint32_t>();
    sa.cap = cap;
    sa.work = ws.swork.as<int32_t>();
    sa.key_base = 0;
    sa.row_limit = (uint32_t)cutoff;
    sa.ablate = filter_ablate();
    sa.rsq16 = metric == L2 ? st.rsq16.as<float>() : st.rsq.as<float>();
    sa.rsq = st.rsq.as<float>();
    // the scan's error terms at the tile dimension (the padded dims' products are exact zeros: the
    // larger D only widens the bound)
    const int dt = st.tdim();
    stream_ub_terms(dt, metric, filter_f16_cerr(dt, metric, FILTER_F16X1), filter_cerr(dt),
                    filter_f16_abs(dt, metric, st.sx, FILTER_F16X1), sa);
    sa.mub = st.row_terms(metric, sa.kr, sa.kx, ws.st);
    {
      PhaseTimer t(PH_SAMPLE, ws.st);
      stream_sample(sa, metric, maxi, ws.st);
      StreamSelectArgs sel{};
      sel.samp = ws.ssamp.as<float>();
      sel.nq = nq;
      sel.n = probes * sv;
      stream_rank(k1, sel.rmin, sel.rmax, sel.et);
      sel.probes = ws.probes.as<int32_t>();
      sel.nprobe = probes;
      sel.lb = lbd.as<int32_t>();
      sel.le = led.as<int32_t>();
      sel.thr = ws.sthr.as<float>();
      launch_stream_select(sel, ws.st);
    }
    sa.work = ws.swork.as<int32_t>() + 1;
    {
      PhaseTimer t(PH_FLAT_SCAN, ws.st, nq * cutoff);
      launch_scan_main(main_scan_args(sa), metric, maxi, ws.st);
    }
    note_stream_slice(ws, nq, cap);
    ws.ms.ensure(sizeof(float) * nq * STREAM_KO);
    ws.mk.ensure(sizeof(int32_t) * nq * STREAM_KO);
    const bool fused = merge_refine_fused();
    CandMergeArgs m{};
    m.cand = ws.scand.as<uint2>();
    m.cand_n = ws.scn.as<int32_t>();
    m.cand_f = ws.scf.as<uint32_t>();
    m.thr = ws.sthr.as<float>();
    m.nq = nq;
    m.cap = cap;
    m.out_s = ws.ms.as<float>();
    m.out_k = ws.mk.as<int32_t>();
    if (!fused) {
      PhaseTimer t(PH_MERGE, ws.st);
      launch_cand_merge(m, ws.st);
    }
    ws.fail.ensure(sizeof(int32_t) * nq);
    ws.fail2.ensure(sizeof(int32_t) * nq);
    ws.fail_cnt.ensure(sizeof(int32_t));
    ws.fail_cnt2.ensure(sizeof(int32_t));
    RefineArgs r{};
    r.rows = st.rows.as<float>();
    r.rows_rm = st.rrm.as<float>();
    r.row_labels = st.labels.as<int64_t>();
    r.queries = d_q;
    r.ms = ws.ms.as<float>();
    r.mk = ws.mk.as<int32_t>();
    r.ld = STREAM_KO;
    r.max_rsq = st.rmax.as<uint32_t>();
    r.nq = nq;
    r.k = k;
    r.dim = dim;
    r.c_err = filter_cerr(dim);
    r.c_bf = filter_f16_cerr(dim, metric, FILTER_F16X1);
    r.ub = 1;
    r.resid = 1;
    r.q16 = 1;
    r.c_abs = filter_f16_abs(dim, metric, st.sx, FILTER_F16X1);
    if (cr) {  // Cosine: the candidates' exact Cosine on the raw rows, certified in cosine units
      r.rows = cr->raw->rows.as<float>();
      r.rows_rm = cr->raw->f16 ? cr->raw->rrm.as<float>() : nullptr;
      r.row_labels = cr->raw->labels.as<int64_t>();
      r.queries = cr->queries;
      r.max_rsq = cr->raw->rmax.as<uint32_t>();
      r.cosine = 1;
      r.qnorm = cr->qnorm;
      r.rnorm = cr->raw->norms.as<float>();
      r.zflag = cr->zflag;
    }
    r.out_s = d_s;
    r.out_l = d_l;
    r.out_c = d_c;
    if (k1 > STREAM_KO) {  // k > 60 (L2 / IP): depth K1 in one block per query, what fails on the exact scan
      {
        PhaseTimer t(PH_REFINE, ws.st, nq * k1);
        r.k1 = k1;
        r.fail_list = ws.fail.as<int32_t>();
        r.fail_cnt = ws.fail_cnt.as<int32_t>();
        launch_deep_refine(m, r, metric, exact_v, ws.st);
        HIPCHK(hipGetLastError());
      }
      int32_t nf = 0;
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
      if (knob("PYR_STREAM_DEBUG"))
        fprintf(stderr, "[flat stream deep] nq %lld k %d: depth %d certificate failures %d\n", (long long)nq, k, k1,
                nf);
      // Cosine: the raw queries through the Cosine index's own exact scan
      filter_fallback(ws, nf, cr ? cr->queries : d_q, dim, k, d_s, d_l, d_c,
                      [&](const float *q2, int64_t n2, float *s2, int64_t *l2, int32_t *c2) {
                        if (cr) cr->exact(q2, n2, s2, l2, c2);
                        else search_exact(q2, n2, k, cutoff, s2, l2, c2, ws.nested());
                      });
      return;
    }
    if (fused) {  // merge, depth K1, depth 64 for the failures: one kernel
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.fail_list = ws.fail.as<int32_t>();
      r.fail_cnt = ws.fail_cnt.as<int32_t>();
      launch_merge_refine(m, r, metric, exact_v, ws.st);
      HIPCHK(hipGetLastError());
    } else {
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.fail_list = ws.fail2.as<int32_t>();
      r.fail_cnt = ws.fail_cnt2.as<int32_t>();
      launch_refine(r, metric, exact_v, ws.st);
      r.k1 = STREAM_KO;  // the failures at depth 64 from the same candidates
      r.qsel = ws.fail2.as<int32_t>();
      r.nsel = ws.fail_cnt2.as<int32_t>();
      r.fail_list = ws.fail.as<int32_t>();
      r.fail_cnt = ws.fail_cnt.as<int32_t>();
      launch_refine(r, metric, exact_v, ws.st);
      HIPCHK(hipGetLastError());
    }
    // measurement only (the profiler's re-run count, PYR_STREAM_DEBUG): read the failure counts back
    int32_t nf = 0;
    if (prof().on || knob("PYR_STREAM_DEBUG")) {
      int32_t n1 = 0;
      HIPCHK(hipMemcpyAsync(&n1, ws.fail_cnt2.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
      if (knob("PYR_STREAM_DEBUG"))
        fprintf(stderr, "[flat stream] nq %lld chunks %d: certificate failures depth %d %d, depth 64 %d\n",
                (long long)nq, nch, k1, n1, nf);
    }
    // what neither certificate covers: the exact *Unsafe scan of the failing queries over every chunk,
    // on the device from the device fail list (pyr_index_search_device stays asynchronous)
    IvfRerunArgs ra{};
    ra.rows = st.rows.as<float>();
    ra.live = st.live.as<uint8_t>();
    ra.labels = st.labels.as<int64_t>();
    ra.queries = d_q;
    ra.probes = ws.probes.as<int32_t>();
    ra.nprobe = probes;
    ra.lb = lbd.as<int32_t>();
    ra.le = led.as<int32_t>();
    ra.fail = ws.fail.as<int32_t>();
    ra.nfail = ws.fail_cnt.as<int32_t>();
    ra.dim = dim;
    ra.k = k;
    ra.v4 = exact_v == 4;
    if (cr) {  // the exact Cosine (:354) over the raw rows
      ra.rows = cr->raw->rows.as<float>();
      ra.labels = cr->raw->labels.as<int64_t>();
      ra.queries = cr->queries;
      ra.qnorm = cr->qnorm;
      ra.rnorm = cr->raw->norms.as<float>();
    }
    ra.out_s = d_s;
    ra.out_l = d_l;
    ra.out_c = d_c;
    if (!filter_ablate() && !knob("PYR_STREAM_THR_BIAS")) {
      PhaseTimer t(PH_FALLBACK, ws.st, nf);
      ra.nchunk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, (flat_chunk_rows(cutoff) + 1023) / 1024));
      ra.done = rerun_done(ws, nq);
      ws.rrpart.ensure(sizeof(uint64_t) * ivf_rerun_part_keys(nq, probes, k));
      launch_ivf_exact_rerun(ra, cr ? COS : metric, nq, ws.rrpart.as<uint64_t>(), ws.st);
    }
    HIPCHK(hipGetLastError());
  }

  // BruteForceVectorIndex.Search (:275-379) on the VALU, the reference's exact arithmetic
  void search_exact(const float *d_q, int64_t nq, int k, int64_t cutoff, float *d_s, int64_t *d_l, int32_t *d_c,
                    Workspace &ws) {
    prep_queries(d_q, nq, dim, metric, ws);
    ScanPlan p = plan_flat(cutoff, nq, dim, k, MAX_PARTS);
    const size_t np = (size_t)nq * p.nchunks * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    uint32_t *gthr = shared_bounds(ws, nq);
    {
      PhaseTimer t(PH_FLAT_SCAN, ws.st, nq * cutoff);
      flat_scan(st, cutoff, p, d_q, metric == COS ? ws.qn.as<float>() : nullptr, nq, k, exact_v, metric, p.nchunks, 0,
                0, ws, ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), false, gthr);
    }
    PhaseTimer t(PH_MERGE, ws.st);
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, p.nchunks, k, st.labels.as<int64_t>(),
                      nullptr, d_s, d_l, nullptr, d_c, ws.st);
  }

  void scan(int64_t *labels, float *x, int64_t *n) override {  // :250-273
    std::vector<int64_t> slots;
    slots.reserve(slot_of.size());
    for (int64_t i = 0; i < st.n; i++)
      if (st.hlive[i]) slots.push_back(i);
    *n = (int64_t)slots.size();
    if (labels)
      for (size_t j = 0; j < slots.size(); j++) labels[j] = st.hlabels[slots[j]];
    if (!x || slots.empty()) return;
    const int64_t cnt = (int64_t)slots.size();
    stage_i.ensure(sizeof(int64_t) * cnt);
    stage_x.ensure(sizeof(float) * cnt * dim);
    HIPCHK(hipMemcpyAsync(stage_i.p, slots.data(), sizeof(int64_t) * cnt, hipMemcpyHostToDevice, wst));
    launch_gather_blocked(st.rows.as<float>(), stage_i.as<int64_t>(), cnt, dim, stage_x.as<float>(), wst);
    HIPCHK(hipMemcpyAsync(x, stage_x.p, sizeof(float) * cnt * dim, hipMemcpyDeviceToHost, wst));
    HIPCHK(hipStreamSynchronize(wst));
  }

  int64_t count() const override { return (int64_t)slot_of.size(); }  // :115-126
  void all_labels(std::vector<int64_t> &out) const override { (void)live_slots(st, out); }

  void snapshot(const std::string &path) override {  // :58-82: the live (id, vector) pairs in slot order
    ImageWriter w(path, PYR_FLAT, dim, metric);
    std::vector<int64_t> labels;
    const std::vector<int64_t> slots = live_slots(st, labels);
    write_rows(w, T_FLABELS, T_FROWS, st, slots, labels, stage_x, stage_i, wst);
    w.commit();
  }

  void load(const std::string &path) override {  // :84-106: Clear(), then InternalAdd per entry
    ImageReader r(path);
    check_image(r, PYR_FLAT, *this);
    std::vector<int64_t> labels;
    std::vector<float> rows;
    const int64_t n = read_rows(r, T_FLABELS, T_FROWS, dim, labels, rows);
    if (st.cap) HIPCHK(hipMemsetAsync(st.live.p, 0, st.cap, wst));
    if (st.rmax.p) HIPCHK(hipMemsetAsync(st.rmax.p, 0, 2 * sizeof(uint32_t), wst));
    if (q8cap) HIPCHK(hipMemsetAsync(q8ok.p, 0, q8cap, wst));
    HIPCHK(hipStreamSynchronize(wst));
    st.clear();
    slot_of.clear();
    if (unit) unit_reset();
    if (n) add(rows.data(), n, labels.data(), false);  // codes iff EnableQuantization now (:166-178)
  }
};

// ---------------------------------------------------------------------------
// Pre-build buffer with .NET Dictionary<string, ...> slot semantics:
// enumeration = slot order; removal frees a slot; insertion reuses the most
// recently freed slot (LIFO free list).  (IvfFlatVectorIndex.cs:17, IvfPqVectorIndex.cs:19)
// ---------------------------------------------------------------------------
struct DictBuffer {
  RowStore st;
  std::unordered_map<int64_t, int64_t> slot_of;
  std::vector<int64_t> free_slots;
  void all_labels(std::vector<int64_t> &out) const {
    for (const auto &e : slot_of) out.push_back(e.first);
  }

  // returns slots for labels (overwrite existing, reuse freed, else append)
  std::vector<int64_t> place(const int64_t *labels, int64_t n) {
    std::vector<int64_t> slots(n);
    for (int64_t i = 0; i < n; i++) {
      auto f = slot_of.find(labels[i]);
      if (f != slot_of.end()) {
        slots[i] = f->second;
        continue;
      }
      int64_t s;
      if (!free_slots.empty()) {
        s = free_slots.back();
        free_slots.pop_back();
      } else {
        s = st.n++;
        st.hlabels.push_back(-1);
        st.hlive.push_back(0);
      }
      slot_of[labels[i]] = s;
      slots[i] = s;
    }
    return slots;
  }
  void write(const float *x, const int64_t *labels, int64_t n, hipStream_t wst, DevMem &sx, DevMem &si) {
    std::vector<int64_t> slots = place(labels, n);
    std::vector<float> xs;
    std::vector<int64_t> ls;
    keep_last_writes(x, labels, n, slots, st.dim, st.n, xs, ls);
    st.reserve(st.n, wst);
    st.write(x, slots.data(), labels, n, wst, sx, si);
    for (int64_t i = 0; i < n; i++) {
      st.hlabels[slots[i]] = labels[i];
      st.hlive[slots[i]] = 1;
    }
  }
  bool erase(int64_t label, std::vector<int64_t> &dead) {
    auto f = slot_of.find(label);
    if (f == slot_of.end()) return false;
    dead.push_back(f->second);
    free_slots.push_back(f->second);
    slot_of.erase(f);
    return true;
  }
  int64_t live_count() const { return (int64_t)slot_of.size(); }
  void reserve(int64_t rows, hipStream_t wst) {
    st.reserve(st.n + rows, wst);
    slot_of.reserve(slot_of.size() + (size_t)rows);
    st.hlabels.reserve(st.n + rows);
    st.hlive.reserve(st.n + rows);
  }
  // slot cutoff after the first `m` live slots (m < 0: all)
  int64_t cutoff(int64_t m) const {
    if (m < 0 || m >= live_count()) return st.n;
    if (m == 0) return 0;
    int64_t seen = 0;
    for (int64_t i = 0; i < st.n; i++)
      if (st.hlive[i] && ++seen == m) return i + 1;
    return st.n;
  }
  void clear(hipStream_t wst) {
    if (st.n) HIPCHK(hipMemsetAsync(st.live.p, 0, st.n, wst));
    HIPCHK(hipStreamSynchronize(wst));
    if (st.cap > 65536) {  // a bulk-loaded buffer was compacted into lists: give the HBM back
      st.rows.release();
      st.rrm.release();
      st.rsq.release();
      st.norms.release();
      st.live.release();
      st.labels.release();
      st.cap = 0;
    }
    st.clear();
    slot_of.clear();
    free_slots.clear();
  }
};

// coarse quantizer shared by IVF_FLAT and IVF_PQ: centroids blocked + row-major
// error-bound constant of the matrix-core coarse ranking (coarse.hip coarse_pick_kernel): 4 D + 64
// covers (2.2 D + 8) u (|q| + |c|)^2; PYR_COARSE_CERR overrides it for tests (huge: every query takes
// the dense exact fallback)
static double coarse_cerr(int dim) {
  if (const char *e = knob("PYR_COARSE_CERR")) return atof(e);
  return 4.0 * dim + 64.0;
}

struct Coarse {
  int nlist = 0;
  RowStore cs;
  DevMem rm;  // row-major centroids
  std::vector<float> host;
  // the matrix-core ranking (coarse.hip launch_coarse_mfma): |c|^2 per centroid, max |c|, and whether
  // every centroid value is finite (otherwise the dense exact ranking runs)
  DevMem c2;
  DevMem split;  // bf16 hi / lo planes in MFMA fragment order (launch_coarse_split)
  double cnmax = 0.0;
  bool cfinite = false;

  void set(const float *d_cents_rm, int k, int dim, int met, hipStream_t st) {
    nlist = k;
    cs.dim = dim;
    cs.cosine = met == COS;  // centroid norms cached (IvfFlatVectorIndex.cs:122)
    cs.clear();
    cs.reserve(round_up(k, 8), st);
    HIPCHK(hipMemsetAsync(cs.live.p, 0, cs.cap, st));
    launch_to_blocked(d_cents_rm, nullptr, k, dim, cs.rows.as<float>(), 0, st);
    fill_u8(cs.live.as<uint8_t>(), 1, k, st);
    if (cs.cosine) launch_norms(cs.rows.as<float>(), k, dim, 1, cs.norms.as<float>(), st);
    rm.ensure(sizeof(float) * k * dim);
    HIPCHK(hipMemcpyAsync(rm.p, d_cents_rm, sizeof(float) * k * dim, hipMemcpyDeviceToDevice, st));
    host.resize((size_t)k * dim);
    HIPCHK(hipMemcpyAsync(host.data(), d_cents_rm, sizeof(float) * k * dim, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    cs.n = k;
    {
      std::vector<float> n2((size_t)k);
      double mx = 0.0;
      cfinite = true;
      for (int i = 0; i < k; ++i) {
        double a = 0.0;
        for (int d = 0; d < dim; ++d) {
          const float v = host[(size_t)i * dim + d];
          cfinite = cfinite && std::isfinite(v);
          a += (double)v * v;
        }
        n2[i] = (float)a;
        mx = std::max(mx, std::sqrt(a));
      }
      cnmax = mx * (1.0 + 1e-6);
      c2.ensure(sizeof(float) * std::max(k, 1));
      HIPCHK(hipMemcpyAsync(c2.p, n2.data(), sizeof(float) * k, hipMemcpyHostToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    // the bf16 hi / lo split of the centroids for the matrix-core approximate scores (coarse.hip)
    if (dim % 16 == 0 && dim <= coarse_bf3_max_dim() && k >= 1) {
      split.ensure(coarse_split_bytes(k, dim));
      launch_coarse_split(rm.as<float>(), k, dim, split.p, st);
    } else {
      split.release();
    }
  }

  // score all centroids (ComputeScore, safe VectorMath), rank desc (ties by index), keep nprobe
  // IvfFlatVectorIndex.cs:186-198, IvfPqVectorIndex.cs:141-150
  void probe(const float *d_q, const float *d_qn, int64_t nq, int nprobe, int met, Workspace &ws) {
    if (ws.ext_probes) {  // ranked by the caller (pyr_index_search_probed_device)
      if (ws.ext_nprobe != nprobe) throw Error(PYR_E_ARG, "probe lists have the wrong width for this nprobe");
      ws.probes.ensure(sizeof(int32_t) * nq * nprobe);
      launch_copy_words(ws.probes.p, ws.ext_probes, nq * nprobe, ws.st);
      return;
    }
    // the matrix-core ranking (PYR_COARSE_MFMA=0: the dense exact ranking below; same probes)
    const char *cm = knob("PYR_COARSE_MFMA");
    if (!(cm && atoi(cm) == 0) && cfinite && coarse_mfma_supported(nlist, cs.dim, met, nprobe) &&
        coarse_dense_supported(nlist)) {
      ws.probes.ensure(sizeof(int32_t) * nq * nprobe);
      const int64_t qb = std::max<int64_t>(1, std::min<int64_t>(int64_t(1) << 21, (int64_t(1) << 26) / nlist));
      const int64_t nb = std::min<int64_t>(nq, qb);
      ws.cpart_s.ensure(sizeof(float) * (size_t)nb * nlist);
      ws.cfail.ensure(sizeof(int32_t) * (size_t)nb);
      ws.cnfail.ensure(sizeof(int32_t));
      for (int64_t a = 0; a < nq; a += qb) {
        const int64_t n = std::min<int64_t>(qb, nq - a);
        launch_coarse_mfma(d_q + a * cs.dim, rm.as<float>(), c2.as<float>(), n, nlist, cs.dim, met, nprobe, cnmax,
                           coarse_cerr(cs.dim), ws.cpart_s.as<float>(), ws.cfail.as<int32_t>(),
                           ws.cnfail.as<int32_t>(), ws.probes.as<int32_t>() + a * nprobe, ws.st,
                           ws.pz_set ? &ws.pz : nullptr, split.p);
        ws.pz_set = false;
      }
      return;
    }
    const char *ce = knob("PYR_COARSE_DENSE");  // 0: the top-k scan below (A/B only, same ranking)
    if (!(ce && atoi(ce) == 0) && coarse_dense_supported(nlist)) {
      ws.probes.ensure(sizeof(int32_t) * nq * nprobe);
      // <= 256 MB of scores and <= 2^21 queries (grid.y) per launch
      const int64_t qb = std::max<int64_t>(1, std::min<int64_t>(int64_t(1) << 21, (int64_t(1) << 26) / nlist));
      ws.cpart_s.ensure(sizeof(float) * (size_t)std::min<int64_t>(nq, qb) * nlist);
      for (int64_t a = 0; a < nq; a += qb) {
        const int64_t n = std::min<int64_t>(qb, nq - a);
        launch_coarse_dense(d_q + a * cs.dim, rm.as<float>(), d_qn ? d_qn + a : nullptr,
                            met == COS ? cs.norms.as<float>() : nullptr, n, nlist, cs.dim, met, nprobe,
                            ws.cpart_s.as<float>(), ws.probes.as<int32_t>() + a * nprobe, ws.st);
      }
      return;
    }
    const int qchunk = fast_path(cs.dim, nprobe) ? QCHUNK : QCHUNK_GENERIC;
    const int64_t nqc = (nq + qchunk - 1) / qchunk;
    int want = (int)std::max<int64_t>(1, std::min<int64_t>(16, (2048 + nqc - 1) / nqc));
    want = std::min(want, std::max(1, nlist / 32));
    if (const char *e = knob("PYR_COARSE_CHUNKS")) want = std::max(1, std::min(atoi(e), nlist));  // measurement
    ScanPlan p;
    p.qchunk = qchunk;
    p.chunk_rows = (int)round_up((nlist + want - 1) / want, 8);
    p.nchunks = (nlist + p.chunk_rows - 1) / p.chunk_rows;
    p.nitems = (int)(p.nchunks * nqc);
    const size_t np = (size_t)nq * p.nchunks * nprobe;
    ws.cpart_s.ensure(sizeof(float) * np);
    ws.cpart_k.ensure(sizeof(uint32_t) * np);
    flat_scan(cs, nlist, p, d_q, d_qn, nq, nprobe, 1, met, p.nchunks, 0, 0, ws, ws.cpart_s.as<float>(),
              ws.cpart_k.as<uint32_t>());
    ws.probes.ensure(sizeof(int32_t) * nq * nprobe);
    launch_merge_keys(ws.cpart_s.as<float>(), ws.cpart_k.as<uint32_t>(), nq, p.nchunks, nprobe, nullptr, nullptr,
                      nullptr, nullptr, ws.probes.as<int32_t>(), nullptr, ws.st);
  }
};

// (query, row) pairs a list scan scores: sum of probed list lengths (profiling only; syncs)
static int64_t probed_rows(Workspace &ws, int64_t nq, int probes, const std::vector<int32_t> &le,
                           const std::vector<int32_t> &lb) {
  std::vector<int32_t> pr((size_t)nq * probes);
  HIPCHK(hipMemcpyAsync(pr.data(), ws.probes.p, sizeof(int32_t) * pr.size(), hipMemcpyDeviceToHost, ws.st));
  HIPCHK(hipStreamSynchronize(ws.st));
  int64_t s = 0;
  for (int32_t l : pr) s += le[l] - lb[l];
  return s;
}

// list-major work items from ws.probes
// phase 0 -> ws.items / ws.nitems, phase 1 -> ws.items3 / ws.nitems3 (IvfChunking, kernels.h)
static int build_ivf_items(Workspace &ws, int64_t nq, int nprobe, int nparts, int nlist, const DevMem &lbeg,
                           const DevMem &lend, int qchunk, IvfChunking ch, int phase, bool balance, bool zeroed) {
  const int64_t maxi64 = ivf_max_items(nq, nprobe, nlist, qchunk, ch, phase);
  if (maxi64 > INT32_MAX) throw Error(PYR_E_ARG, "query batch too large for one launch");
  const int maxi = (int)maxi64;
  DevMem &items = phase == 0 ? ws.items : ws.items3;
  DevMem &nitems = phase == 0 ? ws.nitems : ws.nitems3;
  ws.ivf_cnt.ensure(sizeof(int32_t) * nlist);
  ws.ivf_fill.ensure(sizeof(int32_t) * nlist);
  ws.ivf_qoff.ensure(sizeof(int32_t) * (nlist + 1));
  ws.ivf_ioff.ensure(sizeof(int32_t) * (nlist + 1));
  ws.qlist.ensure(sizeof(int32_t) * std::max<int64_t>(nq * nprobe, 1));
  ws.qpos.ensure(sizeof(int32_t) * std::max<int64_t>(nq * nprobe, 1));
  items.ensure(sizeof(ScanItem) * std::max(maxi, 1));
  nitems.ensure(sizeof(int32_t) * 16);  // the count, then (IvfChunking::xcd) the 9 queue bounds
  IvfItemWs iw{ws.ivf_cnt.as<int32_t>(), ws.ivf_fill.as<int32_t>(), ws.ivf_qoff.as<int32_t>(),
               ws.ivf_ioff.as<int32_t>(), ws.qlist.as<int32_t>(), items.as<ScanItem>(), nitems.as<int32_t>(),
               ws.qpos.as<int32_t>()};
  launch_ivf_items(ws.probes.as<int32_t>(), nq, nprobe, nparts, nlist, lbeg.as<int32_t>(), lend.as<int32_t>(), qchunk,
                   ch, phase, iw, ws.st, 0, -1, balance, zeroed);
  return maxi;
}

// Items of probe ranks [pb, pe) only, into item set 0 (ws.items, ws.qlist, ...) or 1 (ws.items3,
// ws.qlist2, ...).  Partial slots keep the absolute probe rank.
static int build_ivf_items_range(Workspace &ws, int set, int64_t nq, int nprobe, int pb, int pe, int nparts,
                                 int nlist, const DevMem &lbeg, const DevMem &lend, int qchunk, IvfChunking ch,
                                 bool balance = false) {
  const int64_t maxi64 = ivf_max_items(nq, pe - pb, nlist, qchunk, ch, 0);
  if (maxi64 > INT32_MAX) throw Error(PYR_E_ARG, "query batch too large for one launch");
  const int maxi = (int)maxi64;
  DevMem &items = set == 0 ? ws.items : ws.items3;
  DevMem &nitems = set == 0 ? ws.nitems : ws.nitems3;
  DevMem &cnt = set == 0 ? ws.ivf_cnt : ws.ivf_cnt2, &fill = set == 0 ? ws.ivf_fill : ws.ivf_fill2;
  DevMem &qoff = set == 0 ? ws.ivf_qoff : ws.ivf_qoff2, &ioff = set == 0 ? ws.ivf_ioff : ws.ivf_ioff2;
  DevMem &qlist = set == 0 ? ws.qlist : ws.qlist2;
  cnt.ensure(sizeof(int32_t) * nlist);
  fill.ensure(sizeof(int32_t) * nlist);
  qoff.ensure(sizeof(int32_t) * (nlist + 1));
  ioff.ensure(sizeof(int32_t) * (nlist + 1));
  qlist.ensure(sizeof(int32_t) * std::max<int64_t>(nq * (pe - pb), 1));
  items.ensure(sizeof(ScanItem) * std::max(maxi, 1));
  nitems.ensure(sizeof(int32_t) * 16);  // the count + 9 queue bounds (ivf_scan_kernel)
  IvfItemWs iw{cnt.as<int32_t>(), fill.as<int32_t>(), qoff.as<int32_t>(), ioff.as<int32_t>(), qlist.as<int32_t>(),
               items.as<ScanItem>(), nitems.as<int32_t>()};
  launch_ivf_items(ws.probes.as<int32_t>(), nq, nprobe, nparts, nlist, lbeg.as<int32_t>(), lend.as<int32_t>(), qchunk,
                   ch, 0, iw, ws.st, pb, pe, balance);
  return maxi;
}

// Nearest-list seeding of the shared bounds (PYR_IVF_SEED=1; off by default, results
// identical): every query's first-ranked list is scanned by a first launch, so the main launch
// starts with each query's bound at the K1-th best of its nearest list instead of -inf.
// Measured at the bench config: candidates 16.3 M -> 9.4 M, insertion iterations -7 %, but the
// small first launch leaves the chip half idle: 9.84 -> 12.0 ms (profiles/r1_sweeps/sweep16-17).
static bool ivf_seed_enabled() {
  const char *e = knob("PYR_IVF_SEED");
  return e && atoi(e) != 0;
}

// Row chunking of the IVF list scan (IvfChunking, kernels.h): a `warm`-row chunk 0 per
// list scanned by an earlier launch to seed the shared per-query bounds, then chunks of
// <= `chunk` rows so that work items are uniform whatever the list-size skew of the
// trained quantizer.  Each (query, probe, chunk) gets its own partial top-k slot, within
// the MAX_PARTS budget left after `other_parts` and a cap on the partial buffer.
// PYR_IVF_CHUNK / PYR_IVF_WARM override the defaults for measurements.
static IvfChunking ivf_chunking(int64_t max_len, int probes, int other_parts, int64_t nq, int k, bool bounds) {
  // 5120 rows: 2048 -> 4096 -> 5120 gave 5.71 -> 5.27 -> ~5.2 ms at the bench config
  // (profiles/r1_sweeps/sweep21, sweep28, sweep29); warm-up launch measured neutral (profiles/)
  int64_t chunk = 5120, warm = 0;
  // a small batch (e.g. the re-run of certificate failures) has few (list, query group) items:
  // shorter chunks give it more of the chip
  if (nq * probes < 8192) chunk = 1024;
  if (const char *e = knob("PYR_IVF_CHUNK")) chunk = std::max<int64_t>(8, atoll(e));
  if (const char *e = knob("PYR_IVF_WARM")) warm = std::max<int64_t>(0, atoll(e));
  if (!bounds) warm = 0;  // the warm-up launch only pays with shared bounds
  chunk = round_up(chunk, 32);  // whole fp16 tiles (lists start on a 32-row boundary)
  warm = round_up(warm, 32);
  auto chunks = [&](int64_t c) {
    return (int64_t)ivf_list_chunks((int)max_len, IvfChunking{(int32_t)c, 1, (int32_t)warm});
  };
  int64_t cmax = chunks(chunk);
  int64_t budget = probes > 0 ? (MAX_PARTS - other_parts) / probes : 1;
  const int64_t buf_cap = (int64_t(4) << 30) / std::max<int64_t>(1, nq * (int64_t)k * 8);  // <= 4 GiB of partials
  budget = std::min(budget, std::max<int64_t>(1, buf_cap / std::max(probes, 1)));
  if (budget < 1) throw Error(PYR_E_ARG, "nprobe too large");
  if (cmax > budget) {
    if (budget < 2) warm = 0;
    const int64_t room = std::max<int64_t>(1, budget - (warm > 0 ? 1 : 0));
    chunk = round_up(std::max<int64_t>(32, (max_len - warm + room - 1) / room), 32);
    cmax = chunks(chunk);
  }
  return IvfChunking{(int32_t)chunk, (int32_t)cmax, (int32_t)warm};
}

// ---------------------------------------------------------------------------
// IVF_FLAT = IvfFlatVectorIndex (IvfFlatVectorIndex.cs)
// ---------------------------------------------------------------------------
struct IvfFlatIndex : Index {
  DictBuffer buf;                         // _buffer (:17)
  RowStore lists;                         // _invertedLists (:22), list-major, lists padded to 8 rows
  std::vector<uint8_t> lstate;            // 0 removed/pad, 1 visible, 2 shadowed by a buffer id (:210)
  std::unordered_map<int64_t, int64_t> pos_of;
  std::vector<int32_t> lb, le, llen, llive;
  int64_t max_len = 0;                    // longest list (rows incl. tombstones): row chunking
  DevMem dlb, dle, dllive;
  DevMem dlmax;                           // per-list max |x|^2 (score_key): refine certificate bound
  int64_t key_label(uint32_t key) const override {
    if (key & KEY_BUF) {
      const int64_t s = key & ~KEY_BUF;
      return s < buf.st.n && buf.st.hlive[s] ? buf.st.hlabels[s] : -1;
    }
    return (size_t)key < lstate.size() && lstate[key] == 1 ? lists.hlabels[key] : -1;
  }
  DevMem dlmax_r;                         // per-list max |x - c|^2 (residual fp16 tiles)
  // Cosine: the fp16 tiles hold unit residuals x/|x| - c/|c| (ucents: the unit centroids) scanned as L2
  // (on unit vectors the L2 order is the cosine order); zflag: a list row with a norm below 1e-6
  DevMem ucents, zflag;
  void reserve(int64_t rows) override { buf.reserve(rows, wst); }
  Coarse coarse;
  bool built = false;                     // _isBuilt (:20)
  int nprobe_default;
  std::vector<float> given;               // pyr_index_set_centroids
  int given_k = 0;

  void set_centroids(const float *c, int nl) override {
    if (nl <= 0) throw Error(PYR_E_ARG, "nlist must be positive");
    given.assign(c, c + (size_t)nl * dim);
    given_k = nl;
  }

  explicit IvfFlatIndex(const pyr_index_desc &d) : Index(d) {
    buf.st.dim = lists.dim = dim;
    buf.st.cosine = lists.cosine = metric == COS;  // CreateEntry norm (:343-349)
    nprobe_default = d.default_nprobe > 0 ? d.default_nprobe : 3;  // CombineNProbe (:14)
  }

  // per row slot its list (shard records): built with the list bounds, on the write stream, under the write
  // lock (no search can see it half built)
  DevMem row_list;
  const int32_t *row_lists(hipStream_t) { return row_list.as<int32_t>(); }

  void upload_list_meta() {
    const int nl = coarse.nlist;
    dlb.ensure(sizeof(int32_t) * std::max(nl, 1));
    dle.ensure(sizeof(int32_t) * std::max(nl, 1));
    dllive.ensure(sizeof(int32_t) * std::max(nl, 1));
    HIPCHK(hipMemcpyAsync(dlb.p, lb.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(dle.p, le.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(dllive.p, llive.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    if (row_list.n < sizeof(int32_t) * (size_t)std::max<int64_t>(lists.n, 1))
      row_list.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(lists.n, 1));
    launch_list_ids(dlb.as<int32_t>(), dle.as<int32_t>(), nl, row_list.as<int32_t>(), wst);
    HIPCHK(hipStreamSynchronize(wst));
  }
  int list_of_pos(int64_t pos) const {
    return (int)(std::upper_bound(lb.begin(), lb.end(), (int32_t)pos) - lb.begin()) - 1;
  }

  void add(const float *x, int64_t n, const int64_t *labels, bool) override {  // Add == Upsert (:39-59)
    buf.write(x, labels, n, wst, stage_x, stage_i);
    if (!built) return;
    std::vector<int64_t> shadow;
    for (int64_t i = 0; i < n; i++) {
      auto f = pos_of.find(labels[i]);
      if (f != pos_of.end() && lstate[f->second] == 1) {
        lstate[f->second] = 2;
        llive[list_of_pos(f->second)]--;
        shadow.push_back(f->second);
      }
    }
    if (!shadow.empty()) {
      lists.set_live(shadow, 0, wst, stage_b);
      upload_list_meta();
    }
  }

  void remove(const int64_t *labels, int64_t n, uint8_t *removed) override {  // :61-83
    std::vector<int64_t> dead_buf, dead_list;
    for (int64_t i = 0; i < n; i++) {
      bool r = buf.erase(labels[i], dead_buf);
      if (built) {
        auto f = pos_of.find(labels[i]);
        if (f != pos_of.end()) {
          if (lstate[f->second] == 1) llive[list_of_pos(f->second)]--;
          lstate[f->second] = 0;
          dead_list.push_back(f->second);
          pos_of.erase(f);
          r = true;
        }
      }
      if (removed) removed[i] = r;
    }
    buf.st.set_live(dead_buf, 0, wst, stage_b);
    if (!dead_list.empty()) {
      lists.set_live(dead_list, 0, wst, stage_b);
      for (int64_t p : dead_list) lists.hlabels[p] = -1;
      upload_list_meta();
    }
  }

  void build() override {  // :85-145
    // 1. uniqueData: existing list items in list order (buffer value wins), then new buffer ids
    std::vector<int64_t> src, labs;  // src >= 0: list position; < 0: buffer slot (-s-1)
    if (built)
      for (int l = 0; l < coarse.nlist; l++)
        for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++) {
          if (lstate[p] == 0) continue;
          const int64_t lab = lists.hlabels[p];
          src.push_back(lstate[p] == 2 ? -buf.slot_of.at(lab) - 1 : p);
          labs.push_back(lab);
        }
    for (int64_t s = 0; s < buf.st.n; s++) {
      if (!buf.st.hlive[s]) continue;
      const int64_t lab = buf.st.hlabels[s];
      if (built && pos_of.count(lab)) continue;  // already placed (overwritten in place)
      src.push_back(-s - 1);
      labs.push_back(lab);
    }
    const int64_t n = (int64_t)src.size();
    if (n == 0) return;  // :111
    DevMem X, dsrc;
    X.ensure(sizeof(float) * n * dim);
    dsrc.ensure(sizeof(int64_t) * n);
    HIPCHK(hipMemcpyAsync(dsrc.p, src.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, wst));
    launch_gather2(built ? lists.rows.as<float>() : buf.st.rows.as<float>(), buf.st.rows.as<float>(),
                   dsrc.as<int64_t>(), n, dim, X.as<float>(), wst);
    // 2. train (:116-119), or take the supplied quantizer
    int k = (int)std::min<int64_t>(desc.nlist, n);
    if (k <= 0) k = 1;
    DevMem C;
    if (given_k > 0) {
      k = given_k;
      C.ensure(sizeof(float) * k * dim);
      HIPCHK(hipMemcpyAsync(C.p, given.data(), sizeof(float) * k * dim, hipMemcpyHostToDevice, wst));
    } else {
      C.ensure(sizeof(float) * k * dim);
      k = kmeans_train_gpu(X.as<float>(), n, dim, k, metric, 10, 42, C.as<float>(), wst);
    }
    // 3. assign (:128-132)
    DevMem A;
    A.ensure(sizeof(int32_t) * n);
    assign_gpu(X.as<float>(), n, dim, C.as<float>(), k, metric, A.as<int32_t>(), wst);
    std::vector<int32_t> asg(n);
    HIPCHK(hipMemcpyAsync(asg.data(), A.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, wst));
    HIPCHK(hipStreamSynchronize(wst));
    commit_lists(X.as<float>(), n, asg, labs, C.as<float>(), k);
    buf.clear(wst);
    built = true;
  }

  // 4. commit (:135-139): rows X (device, row-major n x dim; row i has label labs[i]) into the
  // stable list-major layout by list asg[i] (lists keep X order, padded to 8 rows), quantizer C.
  void commit_lists(const float *X, int64_t n, const std::vector<int32_t> &asg, const std::vector<int64_t> &labs,
                    const float *C, int k) {
    // stable list-major layout, lists padded to 8 rows
    std::vector<int32_t> cnt(k, 0);
    for (int32_t a : asg) cnt[a]++;
    lb.assign(k, 0);
    le.assign(k, 0);
    llen = cnt;
    llive = cnt;
    int64_t tot = 0;
    max_len = 0;
    for (int l = 0; l < k; l++) {
      lb[l] = (int32_t)tot;
      le[l] = (int32_t)(tot + cnt[l]);
      tot += round_up(cnt[l], 32);  // lists start on a 32-row tile boundary
      max_len = std::max<int64_t>(max_len, cnt[l]);
    }
    if (tot >= (int64_t)KEY_BUF) throw Error(PYR_E_ARG, "IVF index larger than 2^31 rows");
    std::vector<int64_t> srcrow(tot, -1), newlab(tot, -1);
    std::vector<int32_t> fillp(lb);
    for (int64_t i = 0; i < n; i++) {
      const int32_t p = fillp[asg[i]]++;
      srcrow[p] = i;
      newlab[p] = labs[i];
    }
    // 4. commit (:135-139)
    RowStore nl;
    nl.dim = dim;
    nl.cosine = metric == COS;
    const bool unit = metric == COS && store16(dim, L2);
    nl.f16 = unit || store16(dim, metric);
    nl.dt = nl.f16 ? store16_dt(dim) : 0;
    nl.met16 = unit ? L2 : metric;
    nl.reserve(std::max<int64_t>(tot, 32), wst);
    DevMem dsr;
    dsr.ensure(sizeof(int64_t) * tot);
    HIPCHK(hipMemcpyAsync(dsr.p, srcrow.data(), sizeof(int64_t) * tot, hipMemcpyHostToDevice, wst));
    launch_to_blocked(X, dsr.as<int64_t>(), tot, dim, nl.rows.as<float>(), 0, wst);
    if (nl.f16) launch_to_rowmajor(X, dsr.as<int64_t>(), tot, dim, nl.rrm.as<float>(), wst);
    std::vector<uint8_t> lv(tot);
    for (int64_t p = 0; p < tot; p++) lv[p] = srcrow[p] >= 0;
    HIPCHK(hipMemcpyAsync(nl.live.p, lv.data(), tot, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(nl.labels.p, newlab.data(), sizeof(int64_t) * tot, hipMemcpyHostToDevice, wst));
    if (nl.cosine) launch_norms(nl.rows.as<float>(), tot, dim, 1, nl.norms.as<float>(), wst);
    launch_sqnorms(nl.rows.as<float>(), nullptr, tot, dim, nl.rsq.as<float>(), nl.rmax.as<uint32_t>(), wst);
    HIPCHK(hipGetLastError());
    DevMem dtl;
    if (nl.f16) {
      // the fp16 tiles hold residuals x - c[list] (filter16.hip residual mode): lists start on a
      // 32-row boundary, so every tile belongs to one list
      std::vector<int32_t> tl((size_t)(nl.cap / 32), 0);
      for (int l = 0; l < k; l++)
        for (int64_t t = lb[l] / 32; t < (lb[l] + round_up(cnt[l], 32)) / 32; t++) tl[t] = l;
      dtl.ensure(sizeof(int32_t) * tl.size());
      HIPCHK(hipMemcpyAsync(dtl.p, tl.data(), sizeof(int32_t) * tl.size(), hipMemcpyHostToDevice, wst));
      nl.resid = true;
      nl.rsq16.ensure(sizeof(float) * nl.cap);
      // Cosine: tiles of the unit rows x/|x| (0 below the 1e-6 norm rule) around the unit centroids
      const float *TR = nl.rows.as<float>(), *TC = C;
      DevMem urm, ublk, cn;
      if (unit) {
        zflag.ensure(sizeof(uint32_t));
        HIPCHK(hipMemsetAsync(zflag.p, 0, sizeof(uint32_t), wst));
        urm.ensure(sizeof(float) * nl.cap * dim);
        ublk.ensure(sizeof(float) * nl.cap * dim);
        launch_unit_rows(nl.rrm.as<float>(), nullptr, nl.norms.as<float>(), tot, dim, urm.as<float>(), wst,
                         zflag.as<uint32_t>(), nl.live.as<uint8_t>());
        HIPCHK(hipMemsetAsync(ublk.p, 0, sizeof(float) * nl.cap * dim, wst));
        launch_to_blocked(urm.as<float>(), nullptr, tot, dim, ublk.as<float>(), 0, wst);
        cn.ensure(sizeof(float) * k);
        launch_norms(C, k, dim, 0, cn.as<float>(), wst);
        ucents.ensure(sizeof(float) * k * dim);
        launch_unit_rows(C, nullptr, cn.as<float>(), k, dim, ucents.as<float>(), wst);
        TR = ublk.as<float>();
        TC = ucents.as<float>();
      }
      launch_resid_sq(TR, nl.cap, dim, TC, dtl.as<int32_t>(), nl.rsq16.as<float>(), wst);
      HIPCHK(hipMemsetAsync(nl.amaxd.p, 0, sizeof(uint32_t), wst));
      launch_absmax(TR, nullptr, nl.cap, dim, nl.amaxd.as<uint32_t>(), wst, TC, dtl.as<int32_t>());
      uint32_t bits = 0;
      HIPCHK(hipMemcpyAsync(&bits, nl.amaxd.p, sizeof(bits), hipMemcpyDeviceToHost, wst));
      HIPCHK(hipStreamSynchronize(wst));
      std::memcpy(&nl.amax, &bits, sizeof(bits));
      nl.sx = pow2_scale_host(nl.amax);
      launch_encode16(TR, nullptr, nl.cap, dim, nl.sx, nl.h16.p, wst, TC, dtl.as<int32_t>(), nl.rsq16.as<float>(),
                      nl.tdim());
      launch_meta16(nullptr, nl.cap, nl.met16, nl.rsq16.as<float>(), nl.live.as<uint8_t>(), nl.meta.as<float>(), wst);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(wst));  // urm / ublk / cn are freed at the end of this block
    }
    HIPCHK(hipStreamSynchronize(wst));
    nl.n = tot;
    nl.hlabels = newlab;
    nl.hlive = lv;
    std::swap(lists.rows.p, nl.rows.p);
    std::swap(lists.rows.n, nl.rows.n);
    std::swap(lists.live.p, nl.live.p);
    std::swap(lists.live.n, nl.live.n);
    std::swap(lists.labels.p, nl.labels.p);
    std::swap(lists.labels.n, nl.labels.n);
    std::swap(lists.norms.p, nl.norms.p);
    std::swap(lists.norms.n, nl.norms.n);
    std::swap(lists.rsq.p, nl.rsq.p);
    std::swap(lists.rsq.n, nl.rsq.n);
    std::swap(lists.rmax.p, nl.rmax.p);
    std::swap(lists.rmax.n, nl.rmax.n);
    std::swap(lists.h16.p, nl.h16.p);
    std::swap(lists.h16.n, nl.h16.n);
    std::swap(lists.meta.p, nl.meta.p);
    std::swap(lists.meta.n, nl.meta.n);
    std::swap(lists.amaxd.p, nl.amaxd.p);
    std::swap(lists.amaxd.n, nl.amaxd.n);
    std::swap(lists.rsq16.p, nl.rsq16.p);
    std::swap(lists.rsq16.n, nl.rsq16.n);
    std::swap(lists.rrm.p, nl.rrm.p);
    std::swap(lists.rrm.n, nl.rrm.n);
    lists.f16 = nl.f16;
    lists.dt = nl.dt;
    lists.met16 = nl.met16;
    lists.sx = nl.sx;
    lists.amax = nl.amax;
    lists.resid = nl.resid;
    lists.n = tot;
    lists.cap = nl.cap;
    lists.hlabels.swap(nl.hlabels);
    lists.hlive.swap(nl.hlive);
    ++lists.gen;
    lstate = lv;
    pos_of.clear();
    for (int64_t p = 0; p < tot; p++)
      if (newlab[p] >= 0) pos_of[newlab[p]] = p;
    coarse.set(C, k, dim, metric, wst);
    upload_list_meta();
    dlmax.ensure(sizeof(uint32_t) * k);
    launch_list_rmax(lists.rsq.as<float>(), dlb.as<int32_t>(), dle.as<int32_t>(), k, dlmax.as<uint32_t>(), wst);
    if (lists.resid) {
      dlmax_r.ensure(sizeof(uint32_t) * k);
      launch_list_rmax(lists.rsq16.as<float>(), dlb.as<int32_t>(), dle.as<int32_t>(), k, dlmax_r.as<uint32_t>(), wst);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(wst));
  }

  void search(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, float *d_s, int64_t *d_l,
              int32_t *d_c, Workspace &ws) override {  // :147-231
    if (k <= 0 || nq == 0) {
      fill_empty_results(d_s, d_l, d_c, nq, std::max(k, 0), ws.st);
      return;
    }
    // MFMA filter path: built lists only (empty pre-build buffer), L2 / IP / Cosine; a MaxScans budget bounds
    // each (query, list) pair's rows (stream_slice), MaxScans 0 scans nothing (the exact path's empty answer)
    const int nprobe = prm.nprobe < 0 ? nprobe_default : prm.nprobe;
    const int probes = (built && coarse.nlist > 0) ? std::max(0, std::min(nprobe, coarse.nlist)) : 0;
    int k1 = filter_k1(k);
    const bool budget_ok = prm.max_scans < 0 || (prm.max_scans > 0 && !ws.ext_probes && max_scans_stream());
    const bool nbuf = buf.live_count() > 0;
    // k > 60: depth 128 / 256 / 512 (deep_refine_kernel), a MaxScans budget too (a buffer: merged beside, below)
    const bool deep = k1 == 0 && !ws.ext_probes && deep_refine_on();
    if (deep) k1 = deep_k1(k);
    const bool fast = filter_enabled() && probes > 0 && (!nbuf || buffer_stream()) && budget_ok &&
                      (k <= KMAX_FAST || deep) && probes < MAX_PARTS && k1 > 0;
    // the stream scan (L2 / IP, and Cosine over the unit residual tiles with the exact Cosine in the refine)
    if (fast && stream_ok(k1)) {
      auto lists_stream = [&](int64_t budget, float *s, int64_t *l, int32_t *c) {
        ws.max_scans = budget;
        try {
          search_stream(d_q, nq, k, k1, probes, s, l, c, ws);
        } catch (...) {
          ws.max_scans = -1;
          throw;
        }
        ws.max_scans = -1;
      };
      if (!nbuf) {
        lists_stream(prm.max_scans, d_s, d_l, d_c);
        return;
      }
      // a non-empty buffer (:169-180): its exact top k over the slots the budget reaches, the lists on the
      // stream scan with what is left of it (their buffer-shadowed rows are not live, :210), the two answers
      // merged with a list entry first on equal scores (the exact path's key order)
      const int64_t maxs = prm.max_scans < 0 ? INT64_MAX : prm.max_scans;
      const int64_t bscanned = std::min<int64_t>(maxs, buf.live_count());
      ws.bx_s.ensure(sizeof(float) * nq * k);
      ws.bx_l.ensure(sizeof(int64_t) * nq * k);
      ws.bx_c.ensure(sizeof(int32_t) * nq);
      ws.lx_s.ensure(sizeof(float) * nq * k);
      ws.lx_l.ensure(sizeof(int64_t) * nq * k);
      ws.lx_c.ensure(sizeof(int32_t) * nq);
      buffer_topk(d_q, nq, k, buf.cutoff(bscanned), ws.bx_s.as<float>(), ws.bx_l.as<int64_t>(),
                  ws.bx_c.as<int32_t>(), ws);
      if (bscanned < maxs)  // :183
        lists_stream(prm.max_scans < 0 ? -1 : maxs - bscanned, ws.lx_s.as<float>(), ws.lx_l.as<int64_t>(),
                     ws.lx_c.as<int32_t>());
      else
        fill_empty_results(ws.lx_s.as<float>(), ws.lx_l.as<int64_t>(), ws.lx_c.as<int32_t>(), nq, k, ws.st);
      PhaseTimer tm(PH_MERGE, ws.st);
      launch_merge_two(ws.lx_s.as<float>(), ws.lx_l.as<int64_t>(), ws.lx_c.as<int32_t>(), ws.bx_s.as<float>(),
                       ws.bx_l.as<int64_t>(), ws.bx_c.as<int32_t>(), nq, k, d_s, d_l, d_c, ws.st);
      HIPCHK(hipGetLastError());
      return;
    }
    search_exact(d_q, nq, k, prm, d_s, d_l, d_c, ws);
  }

  // the buffer's exact top k over its first bcut slots (:169-180, ComputeScore) in (score desc, slot asc) order
  void buffer_topk(const float *d_q, int64_t nq, int k, int64_t bcut, float *d_s, int64_t *d_l, int32_t *d_c,
                   Workspace &ws) {
    if (bcut <= 0) {
      fill_empty_results(d_s, d_l, d_c, nq, k, ws.st);
      return;
    }
    const ScanPlan bp = plan_flat(bcut, nq, dim, k, MAX_PARTS);
    prep_queries(d_q, nq, dim, metric, ws);
    const float *qn = metric == COS ? ws.qn.as<float>() : nullptr;
    const size_t np = (size_t)nq * bp.nchunks * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    {
      PhaseTimer t(PH_BUF_SCAN, ws.st, nq * bcut);
      flat_scan(buf.st, bcut, bp, d_q, qn, nq, k, 1, metric, bp.nchunks, 0, KEY_BUF, ws, ws.part_s.as<float>(),
                ws.part_k.as<uint32_t>(), true);
    }
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, bp.nchunks, k, lists.labels.as<int64_t>(),
                      buf.st.labels.as<int64_t>(), d_s, d_l, nullptr, d_c, ws.st, nullptr);
  }

  // the lists' fp16 residual tiles serve this search's stream scan (scan.hip) at every tile dimension;
  // anything else (k > 60, MaxScans, dims past 768, an unbuilt index) takes the exact scan
  bool stream_ok(int k1) const {
    if (!lists.f16 || !lists.resid) return false;
    const int met = metric == COS ? L2 : metric;
    if (metric == COS && lists.met16 != L2) return false;
    return scan_supported(dim, met, k1);
  }

  // IvfFlatVectorIndex.Search (:147-231) as stream-and-emit (scan.hip): the coarse ranking, then per
  // (list chunk, <= 512 queries) item every row whose approximate score reaches the query's sampled
  // threshold T_q is emitted; the best 64 per query are re-scored exactly and certified (depth K1, then
  // depth 64 for the failures); what still fails is re-run by the exact scan.  Query batches are
  // sliced so that the candidate regions stay within 16 GiB.
  void search_stream(const float *d_q, int64_t nq, int k, int k1, int probes, float *d_s, int64_t *d_l, int32_t *d_c,
                     Workspace &ws, const ShardCtx *sh = nullptr) {
    const int cap = k1 > STREAM_KO ? deep_cap(k1) : stream_cap();
    int64_t chunk = stream_chunk();
    // a list-sharded rank's lists it does not own are empty: their (query, list) pairs get no item.  Not
    // otherwise: the sample pass writes the (empty) sample of an empty list's pairs through its item
    IvfChunking ch{(int32_t)chunk, 1, 0, sh ? 1 : 0};
    ch.cmax = std::max(1, ivf_list_chunks((int)max_len, ch));
    if ((int64_t)probes * ch.cmax > MAX_PARTS) {  // fewer, longer chunks
      const int64_t room = std::max<int64_t>(1, MAX_PARTS / std::max(probes, 1));
      chunk = round_up(std::max<int64_t>(32, (max_len + room - 1) / room), 32);
      ch.chunk = (int32_t)chunk;
      ch.cmax = std::max(1, ivf_list_chunks((int)max_len, ch));
    }
    const int nparts = probes * ch.cmax;
    if (nparts > MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    const int64_t qs = stream_slice_queries(nq, probes, lists.tdim(), cap, scan_sample_values());
    for (int64_t a0 = 0; a0 < nq; a0 += qs) {
      const int64_t n = std::min(qs, nq - a0);
      const int32_t *ext = ws.ext_probes;
      if (ext) ws.ext_probes = ext + a0 * ws.ext_nprobe;
      ShardCtx s2{};
      if (sh)
        s2 = ShardCtx{sh->thr + a0, sh->rec + a0 * shard_record_bytes(k), sh->rem ? sh->rem + a0 * sh->rstride : nullptr,
                      sh->rstride};
      try {
        stream_slice(d_q + a0 * dim, n, k, k1, probes, ch, nparts, cap, d_s ? d_s + a0 * k : nullptr,
                     d_l ? d_l + a0 * k : nullptr, d_c ? d_c + a0 : nullptr, ws, sh ? &s2 : nullptr);
      } catch (...) {
        ws.ext_probes = ext;
        throw;
      }
      ws.ext_probes = ext;
    }
  }

  // measurement only (PYR_STREAM_DEBUG): candidate pool and certificate statistics of one slice, to stderr
  void stream_debug(int64_t nq, int k, int k1, int nparts, int cap, int32_t nf, const float *d_s, Workspace &ws) {
    (void)nparts;
    const size_t nslot = (size_t)nq;  // per query: rows emitted (may exceed cap) and floor
    std::vector<float> ms((size_t)nq * STREAM_KO), thr(nq), res((size_t)nq * k);
    std::vector<int32_t> mk((size_t)nq * STREAM_KO), f1(nq);
    std::vector<uint32_t> cf(nslot);
    int32_t n1 = 0;
    HIPCHK(hipMemcpyAsync(ms.data(), ws.ms.p, sizeof(float) * ms.size(), hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(mk.data(), ws.mk.p, sizeof(int32_t) * mk.size(), hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(thr.data(), ws.sthr.p, sizeof(float) * nq, hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(res.data(), d_s, sizeof(float) * res.size(), hipMemcpyDeviceToHost, ws.st));
    std::vector<int32_t> cn(nslot);
    HIPCHK(hipMemcpyAsync(cn.data(), ws.scn.p, sizeof(int32_t) * nslot, hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(cf.data(), ws.scf.p, sizeof(uint32_t) * nslot, hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(&n1, ws.fail_cnt2.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipMemcpyAsync(f1.data(), ws.fail.p, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ws.st));
    HIPCHK(hipStreamSynchronize(ws.st));
    int64_t emitted = 0, full = 0, shallow = 0;
    for (size_t i = 0; i < nslot; ++i) {
      emitted += cn[i];
      full += cn[i] > cap || cf[i] != 0u;
    }
    for (int64_t q = 0; q < nq; ++q) {
      int real = 0;
      for (int i = 0; i < STREAM_KO; ++i) real += mk[q * STREAM_KO + i] >= 0;
      shallow += real < STREAM_KO;
    }
    fprintf(stderr, "[stream] nq %lld: emitted %lld (%.1f per query), full buffers %lld, queries with < %d real "
            "candidates %lld; certificate failures: depth %d %d, depth %d %d\n", (long long)nq, (long long)emitted,
            (double)emitted / std::max<int64_t>(nq, 1), (long long)full, STREAM_KO, (long long)shallow, k1, n1,
            STREAM_KO, nf);
    for (int i = 0; i < std::min(nf, 6); ++i) {
      const int64_t q = f1[i];
      int real = 0, floors = 0;
      for (int j = 0; j < STREAM_KO; ++j) {
        real += mk[q * STREAM_KO + j] >= 0;
        floors += mk[q * STREAM_KO + j] == -2;
      }
      fprintf(stderr, "[stream]   failed q %lld: T %.6g, k-th exact %.6g, approx K1-th %.6g, 64th %.6g, real %d, "
              "floors %d\n", (long long)q, thr[q], res[q * k + k - 1], ms[q * STREAM_KO + k1 - 1],
              ms[q * STREAM_KO + STREAM_KO - 1], real, floors);
    }
  }

  void stream_slice(const float *d_q, int64_t nq, int k, int k1, int probes, IvfChunking ch, int nparts, int cap,
                    float *d_s, int64_t *d_l, int32_t *d_c, Workspace &ws, const ShardCtx *sh = nullptr) {
    const bool cosine = metric == COS;
    const int met = cosine ? L2 : metric;  // Cosine: L2 over the unit vectors (commit_lists)
    defer_stream_counters(ws, nq, coarse.nlist);
    DeferredCounters dc{ws};
    if (cosine) {
      ws.qn.ensure(sizeof(float) * std::max<int64_t>(nq, 1));
      launch_norms(d_q, nq, dim, 0, ws.qn.as<float>(), ws.st);  // VectorMath.ComputeNorm (:167)
    }
    {
      PhaseTimer t(PH_COARSE, ws.st, nq * coarse.nlist);
      // exact coarse ranking (ComputeScore, :186-198)
      coarse.probe(d_q, cosine ? ws.qn.as<float>() : nullptr, nq, probes, metric, ws);
      flush_stream_counters(ws);
    }
    const float *d_qs = d_q;  // the queries the scan scores: the unit queries for Cosine
    if (cosine) {
      ws.cq.ensure(sizeof(float) * nq * dim);
      launch_unit_rows(d_q, nullptr, ws.qn.as<float>(), nq, dim, ws.cq.as<float>(), ws.st);
      d_qs = ws.cq.as<float>();
    }
    const int qmax = scan_qmax(lists.tdim());
    int maxi;
    {
      PhaseTimer t(PH_ITEMS, ws.st);
      maxi = build_ivf_items(ws, nq, probes, nparts, coarse.nlist, dlb, dle, qmax, ch, 0, true, true);
    }
    const int64_t npos = nq * probes;
    // MaxScans (:202-212; the buffer is empty here): every pair's exclusive row bound, in probe order over the
    // live rows (ivf_limits_kernel, one chunk per probe), then at its qlist position for the scan kernel; a
    // list-sharded rank takes each pair's remaining budget from the home rank's plan
    const bool budget = sh ? sh->rem != nullptr : ws.max_scans > 0;
    if (budget) {
      ws.limits.ensure(sizeof(uint32_t) * std::max<int64_t>(npos, 1));
      ws.plim.ensure(sizeof(uint32_t) * std::max<int64_t>(npos, 1));
      IvfChunking c1{1, 1, 0};
      launch_ivf_limits(ws.probes.as<int32_t>(), nq, probes, probes, sh ? 0 : ws.max_scans, dlb.as<int32_t>(),
                        dle.as<int32_t>(), dllive.as<int32_t>(), lists.live.as<uint8_t>(), c1,
                        ws.limits.as<uint32_t>(), ws.st, sh ? sh->rem : nullptr, sh ? sh->rstride : 0);
      launch_pos_limits(ws.qpos.as<int32_t>(), ws.limits.as<uint32_t>(), npos, ws.plim.as<uint32_t>(), ws.st);
    }
    const int sv = scan_sample_values();
    ws.sbq.ensure(sizeof(uint16_t) * std::max<int64_t>(npos, 1) * lists.tdim());
    ws.sqsc.ensure(sizeof(float2) * std::max<int64_t>(npos, 1));
    ws.ssamp.ensure(sizeof(float) * std::max<int64_t>(npos, 1) * sv);
    ws.sthr.ensure(sizeof(float) * nq);
    ws.scand.ensure(sizeof(uint2) * (size_t)std::max<int64_t>(nq, 1) * cap);
    ws.scn.ensure(sizeof(int32_t) * std::max<int64_t>(nq, 1));
    ws.scf.ensure(sizeof(uint32_t) * std::max<int64_t>(nq, 1));
    ws.swork.ensure(sizeof(int32_t) * 2);
    StreamArgs sa{};
    sa.h16 = lists.h16.p;
    sa.meta = lists.meta.as<float>();
    sa.queries = d_qs;
    sa.cents = cosine ? ucents.as<float>() : coarse.rm.as<float>();
    sa.sx = lists.sx;
    sa.items = ws.items.as<ScanItem>();
    sa.n_items = ws.nitems.as<int32_t>();
    sa.qlist = ws.qlist.as<int32_t>();
    // query-major operands (build_ivf_items: every probe of every query) -- not on a list-sharded rank: its batch
    // is N x the queries, most of whose pairs fall on lists it does not hold (-1 positions); the list-major pass
    // visits only its items' pairs (80,000 queries at the N = 8 shape: 46 us vs ~100 us query-major)
    sa.qpos = sh ? nullptr : ws.qpos.as<int32_t>();
    sa.plim = budget ? ws.plim.as<uint32_t>() : nullptr;
    sa.probes = ws.probes.as<int32_t>();
    sa.nq = nq;
    sa.nparts = nparts;
    sa.nprobe = probes;
    sa.cmax = ch.cmax;
    sa.dim = dim;
    sa.dt = lists.tdim();
    sa.bq = ws.sbq.as<_Float16>();
    sa.qsc = ws.sqsc.as<float2>();
    sa.samp = ws.ssamp.as<float>();
    sa.thr = ws.sthr.as<float>();
    sa.cand = ws.scand.as<uint2>();
    sa.cand_n = ws.scn.as<int32_t>();
    sa.cand_f = ws.scf.as<uint32_t>();
    sa.cap = cap;
    sa.work = ws.swork.as<int32_t>();
    sa.key_base = 0;
    sa.row_limit = 0xFFFFFFFFu;
    sa.ablate = filter_ablate();
    sa.thr_bias = knob("PYR_STREAM_THR_BIAS") ? (float)atof(knob("PYR_STREAM_THR_BIAS")) : 0.0f;
    const int prec = FILTER_F16X1;
    sa.rsq16 = lists.rsq16.as<float>();
    sa.rsq = lists.rsq.as<float>();
    const int dt = lists.tdim();  // the scan's error terms at the tile dimension (FlatIndex::stream_slice)
    stream_ub_terms(dt, met, filter_f16_cerr(dt, met, prec), filter_cerr(dt), filter_f16_abs(dt, met, lists.sx, prec),
                    sa);
    sa.mub = lists.row_terms(met, sa.kr, sa.kx, ws.st);
    sa.lioff = ws.ivf_ioff.as<int32_t>();  // the sample pass by list (scan.hip SMP)
    sa.lcnt = ws.ivf_cnt.as<int32_t>();
    sa.nlist = coarse.nlist;
    sa.lqchunk = qmax;
    const bool timing = knob("PYR_STREAM_TIMING") != nullptr;  // measurement only (syncs)
    if (timing) {
      ws.tdbg.ensure(sizeof(unsigned long long) * 8);
      WordFill z;
      z.add(ws.tdbg.p, 16, 0);
      launch_fill_words(z, ws.st);
    }
    {
      PhaseTimer t(PH_SAMPLE, ws.st);
      // list-sharded: T_q comes from the home rank's plan (its sample of every list); only the operands here
      stream_sample(sa, met, maxi, ws.st, sh != nullptr);
      if (sh) {
        sa.thr = sh->thr;
      } else {
        StreamSelectArgs sel{};
        sel.samp = ws.ssamp.as<float>();
        sel.nq = nq;
        sel.n = probes * sv;
        stream_rank(k1, sel.rmin, sel.rmax, sel.et);
        sel.probes = ws.probes.as<int32_t>();
        sel.nprobe = probes;
        sel.lb = dlb.as<int32_t>();
        sel.le = dle.as<int32_t>();
        sel.thr = ws.sthr.as<float>();
        launch_stream_select(sel, ws.st);
      }
    }
    sa.work = ws.swork.as<int32_t>() + 1;
    {
      PhaseTimer t(PH_LIST_SCAN, ws.st, prof().on && !sh ? probed_rows(ws, nq, probes, le, lb) : 0);
      if (timing) sa.tdbg = ws.tdbg.as<unsigned long long>();
      launch_scan_main(main_scan_args(sa), met, maxi, ws.st);
      sa.tdbg = nullptr;
    }
    note_stream_slice(ws, nq, cap);
    if (timing) {
      unsigned long long c[8];
      HIPCHK(hipMemcpyAsync(c, ws.tdbg.p, sizeof(c), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
      const double tot = (double)(c[0] + c[1] + c[2] + c[3]);
      fprintf(stderr, "[stream timing] wave-cycles %.3g: prologue %.1f%%, tiles %.1f%%, end barrier %.1f%%, flush "
              "%.1f%%; wave-items %llu, cycles per wave-item %.0f\n", tot, 100 * c[0] / tot, 100 * c[1] / tot,
              100 * c[2] / tot, 100 * c[3] / tot, c[4], c[4] ? tot / c[4] : 0.0);
    }
    HIPCHK(hipGetLastError());
    ws.ms.ensure(sizeof(float) * nq * STREAM_KO);
    ws.mk.ensure(sizeof(int32_t) * nq * STREAM_KO);
    const bool fused = merge_refine_fused();
    CandMergeArgs m{};
    m.cand = ws.scand.as<uint2>();
    m.cand_n = ws.scn.as<int32_t>();
    m.cand_f = ws.scf.as<uint32_t>();
    m.thr = sa.thr;
    m.nq = nq;
    m.cap = cap;
    m.out_s = ws.ms.as<float>();
    m.out_k = ws.mk.as<int32_t>();
    if (!fused) {
      PhaseTimer t(PH_MERGE, ws.st);
      launch_cand_merge(m, ws.st);
    }
    // certificate at depth K1, then the failures at depth 64 from the same candidates
    ws.fail.ensure(sizeof(int32_t) * nq);
    ws.fail2.ensure(sizeof(int32_t) * nq);
    ws.fail_cnt.ensure(sizeof(int32_t));
    ws.fail_cnt2.ensure(sizeof(int32_t));
    RefineArgs r{};
    r.rows = lists.rows.as<float>();
    r.rows_rm = lists.f16 ? lists.rrm.as<float>() : nullptr;
    r.row_labels = lists.labels.as<int64_t>();
    r.queries = d_q;
    r.ms = ws.ms.as<float>();
    r.mk = ws.mk.as<int32_t>();
    r.ld = STREAM_KO;
    r.max_rsq = lists.rmax.as<uint32_t>();
    r.tri = 1;
    r.list_rmax = dlmax.as<uint32_t>();
    r.probes = ws.probes.as<int32_t>();
    r.nprobe = probes;
    r.nq = nq;
    r.k = k;
    r.dim = dim;
    r.c_err = filter_cerr(dim);
    r.c_bf = filter_f16_cerr(dim, met, prec);
    r.ub = 1;
    r.c_abs = filter_f16_abs(dim, met, lists.sx, prec);
    r.q16 = 1;
    r.resid = 1;
    r.cents = cosine ? ucents.as<float>() : coarse.rm.as<float>();
    r.list_rmax_r = dlmax_r.as<uint32_t>();
    if (cosine) {
      r.cosine = 1;
      r.qnorm = ws.qn.as<float>();
      r.rnorm = lists.norms.as<float>();
      r.zflag = zflag.as<uint32_t>();
    }
    r.out_s = d_s;
    r.out_l = d_l;
    r.out_c = d_c;
    int32_t nf = 0;
    if (k1 > STREAM_KO) {  // k > 60: depth K1 = 128 / 256 in one block per query, what fails on the exact scan
      {
        PhaseTimer t(PH_REFINE, ws.st, nq * k1);
        r.k1 = k1;
        r.fail_list = ws.fail.as<int32_t>();
        r.fail_cnt = ws.fail_cnt.as<int32_t>();
        launch_deep_refine(m, r, met, 1, ws.st);
        HIPCHK(hipGetLastError());
      }
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
      if (knob("PYR_STREAM_DEBUG"))
        fprintf(stderr, "[stream deep] nq %lld k %d: depth %d certificate failures %d\n", (long long)nq, k, k1, nf);
      // the failures' own probe lists (gathered by the fail list) on the exact VALU scan, same arithmetic
      filter_fallback(ws, nf, d_q, dim, k, d_s, d_l, d_c,
                      [&](const float *q2, int64_t n2, float *s2, int64_t *l2, int32_t *c2) {
                        ws.fprobes.ensure(sizeof(int32_t) * n2 * probes);
                        launch_gather_words(ws.probes.as<uint32_t>(), ws.fail.as<int32_t>(), n2, probes,
                                            ws.fprobes.as<uint32_t>(), ws.st);
                        Workspace &nw = ws.nested();
                        nw.ext_probes = ws.fprobes.as<int32_t>();
                        nw.ext_nprobe = probes;
                        // the lists only (a buffer is merged by search()), with what the buffer left of the budget
                        nw.skip_buffer = true;
                        pyr_search_params p2{};
                        p2.nprobe = probes;
                        p2.max_scans = ws.max_scans;
                        try {
                          search_exact(q2, n2, k, p2, s2, l2, c2, nw);
                        } catch (...) {
                          nw.ext_probes = nullptr;
                          nw.skip_buffer = false;
                          throw;
                        }
                        nw.ext_probes = nullptr;
                        nw.skip_buffer = false;
                      });
      return;
    }
    if (sh) {  // list-sharded: the records (exact local top-k + bound); the home rank's merge certifies
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.rec = sh->rec;
      r.rec_lb = dlb.as<int32_t>();
      r.rec_nlist = coarse.nlist;
      r.rec_row_list = row_lists(ws.st);
      if (fused) launch_merge_refine(m, r, met, 1, ws.st);
      else launch_refine(r, met, 1, ws.st);
      HIPCHK(hipGetLastError());
      return;
    }
    if (fused) {  // merge, depth K1, depth 64 for the failures: one kernel
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.fail_list = ws.fail.as<int32_t>();
      r.fail_cnt = ws.fail_cnt.as<int32_t>();
      launch_merge_refine(m, r, met, 1, ws.st);
      HIPCHK(hipGetLastError());
    } else {
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.fail_list = ws.fail2.as<int32_t>();
      r.fail_cnt = ws.fail_cnt2.as<int32_t>();
      launch_refine(r, met, 1, ws.st);
      if (k1 < STREAM_KO && k + 4 <= STREAM_KO) {
        r.k1 = STREAM_KO;
        r.qsel = ws.fail2.as<int32_t>();
        r.nsel = ws.fail_cnt2.as<int32_t>();
        r.fail_list = ws.fail.as<int32_t>();
        r.fail_cnt = ws.fail_cnt.as<int32_t>();
        launch_refine(r, met, 1, ws.st);
      } else {
        launch_copy_words(ws.fail.p, ws.fail2.p, nq, ws.st);
        launch_copy_words(ws.fail_cnt.p, ws.fail_cnt2.p, 1, ws.st);
      }
      HIPCHK(hipGetLastError());
    }
    // measurement only (the profiler's re-run count, PYR_STREAM_DEBUG): read the failure count back
    const bool dbg = knob("PYR_STREAM_DEBUG") != nullptr;
    if (prof().on || dbg) {
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
      if (dbg) stream_debug(nq, k, k1, nparts, cap, nf, d_s, ws);
    }
    // what neither certificate covers: the exact scan of the failing queries' own probe lists, driven by
    // the device-side fail list (no host round trip: pyr_index_search_device stays asynchronous)
    IvfRerunArgs ra{};
    ra.rows = lists.rows.as<float>();
    ra.live = lists.live.as<uint8_t>();
    ra.labels = lists.labels.as<int64_t>();
    ra.queries = d_q;
    ra.probes = ws.probes.as<int32_t>();
    ra.nprobe = probes;
    ra.lb = dlb.as<int32_t>();
    ra.le = dle.as<int32_t>();
    ra.fail = ws.fail.as<int32_t>();
    ra.nfail = ws.fail_cnt.as<int32_t>();
    ra.dim = dim;
    ra.k = k;
    if (cosine) {
      ra.qnorm = ws.qn.as<float>();
      ra.rnorm = lists.norms.as<float>();
    }
    ra.out_s = d_s;
    ra.out_l = d_l;
    ra.out_c = d_c;
    ra.qlim = budget ? ws.limits.as<uint32_t>() : nullptr;
    // (measurement-only knobs that change the candidates skip the re-run: PYR_FILTER_ABLATE,
    // PYR_STREAM_THR_BIAS)
    if (!filter_ablate() && !knob("PYR_STREAM_THR_BIAS")) {
      PhaseTimer t(PH_FALLBACK, ws.st, nf);
      ra.nchunk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, (max_len + 1023) / 1024));
      ra.done = rerun_done(ws, nq);
      ws.rrpart.ensure(sizeof(uint64_t) * ivf_rerun_part_keys(nq, probes, k));
      launch_ivf_exact_rerun(ra, metric, nq, ws.rrpart.as<uint64_t>(), ws.st);
    }
    HIPCHK(hipGetLastError());
  }

  int probe_only(const float *d_q, int64_t nq, int nprobe, int32_t *d_out, Workspace &ws) override {
    if (!built || coarse.nlist <= 0) throw Error(PYR_E_STATE, "index is not built");
    const int probes = std::max(0, std::min(nprobe < 0 ? nprobe_default : nprobe, coarse.nlist));
    if (probes == 0 || nq == 0) return probes;
    prep_queries(d_q, nq, dim, metric, ws);
    coarse.probe(d_q, metric == COS ? ws.qn.as<float>() : nullptr, nq, probes, metric, ws);
    launch_copy_words(d_out, ws.probes.p, nq * probes, ws.st);
    return probes;
  }

  // ---- list-sharded multi-GPU search (shard.hip) ----
  // The rank holds whole lists (the others are empty here) with the shared quantizer, plus a replicated
  // sample of EVERY list: its first <= 512 rows in list order as fp16 residual tiles (the rows the
  // unsharded index's sample pass scores), so that a query's home rank computes the unsharded T_q.
  std::unique_ptr<RowStore> ssamp;
  DevMem sslb, ssle, sglb, sgle;
  std::vector<int64_t> sglen;  // host copy of every list's length given with the samples (MaxScans accounting)

  void set_list_samples(const float *rows, const int64_t *counts, const int64_t *glen, int nl) override {
    if (!built || coarse.nlist <= 0) throw Error(PYR_E_STATE, "index is not built");
    if (nl != coarse.nlist) throw Error(PYR_E_ARG, "the samples do not cover the quantizer's lists");
    if (metric == COS || !store16(dim, metric)) throw Error(PYR_E_STATE, "list-sharded search serves L2 / IP");
    std::vector<int32_t> slb(nl), sle(nl), z(nl, 0), gl(nl);
    int64_t tot = 0, nrows = 0;
    for (int l = 0; l < nl; ++l) {
      if (counts[l] < 0 || counts[l] > 512 || counts[l] > glen[l])
        throw Error(PYR_E_ARG, "a list sample holds more rows than 512 or than its list");
      if (glen[l] > INT32_MAX) throw Error(PYR_E_ARG, "list longer than 2^31 rows");
      slb[l] = (int32_t)tot;
      sle[l] = (int32_t)(tot + counts[l]);
      gl[l] = (int32_t)glen[l];
      tot += round_up(counts[l], 32);
      nrows += counts[l];
    }
    std::vector<int64_t> src((size_t)std::max<int64_t>(tot, 1), -1);
    std::vector<uint8_t> lv((size_t)std::max<int64_t>(tot, 1), 0);
    for (int l = 0, off = 0; l < nl; off += (int)counts[l], ++l)
      for (int64_t j = 0; j < counts[l]; ++j) {
        src[slb[l] + j] = off + j;
        lv[slb[l] + j] = 1;
      }
    auto ss = std::make_unique<RowStore>();
    RowStore &s = *ss;
    s.dim = dim;
    s.f16 = true;
    s.dt = store16_dt(dim);
    s.met16 = metric;
    s.reserve(std::max<int64_t>(tot, 32), wst);
    DevMem X, dsr, dtl;
    X.ensure(sizeof(float) * std::max<int64_t>(nrows, 1) * dim);
    if (nrows) HIPCHK(hipMemcpyAsync(X.p, rows, sizeof(float) * nrows * dim, hipMemcpyHostToDevice, wst));
    dsr.ensure(sizeof(int64_t) * src.size());
    HIPCHK(hipMemcpyAsync(dsr.p, src.data(), sizeof(int64_t) * src.size(), hipMemcpyHostToDevice, wst));
    launch_to_blocked(X.as<float>(), dsr.as<int64_t>(), tot, dim, s.rows.as<float>(), 0, wst);
    HIPCHK(hipMemcpyAsync(s.live.p, lv.data(), (size_t)tot, hipMemcpyHostToDevice, wst));
    launch_sqnorms(s.rows.as<float>(), nullptr, tot, dim, s.rsq.as<float>(), s.rmax.as<uint32_t>(), wst);
    std::vector<int32_t> tl((size_t)(s.cap / 32), 0);  // the list of every 32-row tile (residual tiles)
    for (int l = 0; l < nl; ++l)
      for (int64_t t = slb[l] / 32; t < (slb[l] + round_up(sle[l] - slb[l], 32)) / 32; ++t) tl[t] = l;
    dtl.ensure(sizeof(int32_t) * tl.size());
    HIPCHK(hipMemcpyAsync(dtl.p, tl.data(), sizeof(int32_t) * tl.size(), hipMemcpyHostToDevice, wst));
    s.resid = true;
    s.rsq16.ensure(sizeof(float) * s.cap);
    const float *C = coarse.rm.as<float>();
    launch_resid_sq(s.rows.as<float>(), s.cap, dim, C, dtl.as<int32_t>(), s.rsq16.as<float>(), wst);
    HIPCHK(hipMemsetAsync(s.amaxd.p, 0, sizeof(uint32_t), wst));
    launch_absmax(s.rows.as<float>(), nullptr, s.cap, dim, s.amaxd.as<uint32_t>(), wst, C, dtl.as<int32_t>());
    uint32_t bits = 0;
    HIPCHK(hipMemcpyAsync(&bits, s.amaxd.p, sizeof(bits), hipMemcpyDeviceToHost, wst));
    HIPCHK(hipStreamSynchronize(wst));
    std::memcpy(&s.amax, &bits, sizeof(bits));
    s.sx = pow2_scale_host(s.amax);
    launch_encode16(s.rows.as<float>(), nullptr, s.cap, dim, s.sx, s.h16.p, wst, C, dtl.as<int32_t>(),
                    s.rsq16.as<float>(), s.tdim());
    launch_meta16(nullptr, s.cap, s.met16, s.rsq16.as<float>(), s.live.as<uint8_t>(), s.meta.as<float>(), wst);
    s.n = tot;
    for (DevMem *d : {&sslb, &ssle, &sglb, &sgle}) d->ensure(sizeof(int32_t) * nl);
    HIPCHK(hipMemcpyAsync(sslb.p, slb.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(ssle.p, sle.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(sglb.p, z.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));  // [0, glen): the
    HIPCHK(hipMemcpyAsync(sgle.p, gl.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));  // true lengths
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(wst));
    ssamp = std::move(ss);
    sglen.assign(glen, glen + nl);
  }

  // MaxScans on a list-sharded rank: the home ran the budget down every rank's lists with the lengths given to
  // set_list_samples, so the lists this rank owns must still hold exactly that many live rows (a Delete since
  // would shift every later pair's budget on the other ranks)
  void check_shard_budget_lengths() const {
    for (size_t l = 0; l < llen.size() && l < sglen.size(); ++l)
      if (llen[l] > 0 && (int64_t)llive[l] != sglen[l])
        throw Error(PYR_E_STATE, "list-sharded MaxScans: a list's live rows changed since set_list_samples (call it "
                                 "again with the new lengths)");
  }

  // ---- the multi-device index's hooks (multi.cpp; engine.h "the multi-device index") ----
  bool ms_lists(MsLists &out) const override {
    if (!built || coarse.nlist <= 0) return false;
    out.nlist = coarse.nlist;
    out.nprobe_default = nprobe_default;
    out.lb = lb;
    out.llen = llen;
    out.llive = llive;
    out.state = lstate;
    out.cents.resize((size_t)coarse.nlist * dim);
    int32_t nl = 0;
    centroids(out.cents.data(), &nl);
    return true;
  }
  void ms_gather_rows(const int64_t *d_pos, int64_t n, float *d_out, hipStream_t st) const override {
    if (n > 0) launch_gather_blocked(lists.rows.as<float>(), d_pos, n, dim, d_out, st);
  }
  void ms_commit(const float *d_x, int64_t n, const std::vector<int32_t> &asg, const std::vector<int64_t> &labs,
                 const float *c, int k) override {
    DevMem C;
    C.ensure(sizeof(float) * (size_t)k * dim);
    HIPCHK(hipMemcpyAsync(C.p, c, sizeof(float) * (size_t)k * dim, hipMemcpyHostToDevice, wst));
    commit_lists(d_x, n, asg, labs, C.as<float>(), k);
    buf.clear(wst);
    built = true;
    HIPCHK(hipStreamSynchronize(wst));
  }
  void ms_set_list_lengths(const int64_t *glen, int nl) override {
    if (!ssamp || nl != coarse.nlist) throw Error(PYR_E_STATE, "no list samples (pyr_index_set_list_samples)");
    std::vector<int32_t> g(nl);
    for (int l = 0; l < nl; ++l) g[l] = (int32_t)glen[l];
    HIPCHK(hipMemcpyAsync(sgle.p, g.data(), sizeof(int32_t) * nl, hipMemcpyHostToDevice, wst));
    HIPCHK(hipStreamSynchronize(wst));
    sglen.assign(glen, glen + nl);
  }
  int64_t ms_position(int64_t label) const override {
    auto f = pos_of.find(label);
    return f == pos_of.end() ? -1 : f->second;
  }
  bool ms_shardable(int k, const pyr_search_params &prm, int *P) const override {
    if (!built || coarse.nlist <= 0 || metric == COS || buf.live_count() > 0 || !filter_enabled()) return false;
    const int k1 = filter_k1(k);
    if (k <= 0 || k > KMAX_FAST || k1 <= 0 || !stream_ok(k1)) return false;
    const int nprobe = prm.nprobe < 0 ? nprobe_default : prm.nprobe;
    *P = std::max(0, std::min(nprobe, coarse.nlist));
    return *P > 0 && *P < MAX_PARTS;
  }
  const int64_t *ms_position_labels() const override { return lists.labels.as<int64_t>(); }

  int shard_prepare(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, int32_t *d_plan,
                    Workspace &ws) override {
    if (!ssamp) throw Error(PYR_E_STATE, "no list samples (pyr_index_set_list_samples)");
    const int k1 = filter_k1(k);
    if (k <= 0 || k > KMAX_FAST || k1 <= 0) throw Error(PYR_E_ARG, "topK out of the list-sharded search's range");
    const int nprobe = prm.nprobe < 0 ? nprobe_default : prm.nprobe;
    const int P = std::max(0, std::min(nprobe, coarse.nlist));
    if (P == 0 || nq == 0) return P;
    if (P >= MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    const bool budget = prm.max_scans >= 0;  // plan rows carry the remaining budget per probe (S = 2P + 1)
    const int S = shard_plan_stride(P, budget);
    RowStore &s = *ssamp;
    const int dt = s.tdim(), sv = scan_sample_values();
    // slices of <= 1 GiB of operands and samples
    const int64_t per_q = (int64_t)P * (2 * dt + 8 + 4 * sv) + 64;
    const int64_t qs = std::max<int64_t>(1, std::min<int64_t>(nq, (int64_t(1) << 30) / per_q));
    for (int64_t a0 = 0; a0 < nq; a0 += qs) {
      const int64_t n = std::min(qs, nq - a0);
      const float *q = d_q + a0 * dim;
      defer_stream_counters(ws, n, coarse.nlist);
      DeferredCounters dc{ws};
      {
        PhaseTimer t(PH_COARSE, ws.st, n * coarse.nlist);
        coarse.probe(q, nullptr, n, P, metric, ws);
        flush_stream_counters(ws);
      }
      const IvfChunking ch{512, 1, 0};  // a sample list is one chunk (an empty one too: its sample is empty)
      const int maxi = build_ivf_items(ws, n, P, P, coarse.nlist, sslb, ssle, scan_qmax(dt), ch, 0, true, true);
      const int64_t npos = n * P;
      ws.sbq.ensure(sizeof(uint16_t) * npos * dt);
      ws.sqsc.ensure(sizeof(float2) * npos);
      ws.ssamp.ensure(sizeof(float) * npos * sv);
      ws.sthr.ensure(sizeof(float) * n);
      StreamArgs sa{};
      sa.h16 = s.h16.p;
      sa.meta = s.meta.as<float>();
      sa.queries = q;
      sa.cents = coarse.rm.as<float>();
      sa.sx = s.sx;
      sa.items = ws.items.as<ScanItem>();
      sa.n_items = ws.nitems.as<int32_t>();
      sa.qlist = ws.qlist.as<int32_t>();
      sa.qpos = ws.qpos.as<int32_t>();  // query-major operands (build_ivf_items: every probe of every query)
      sa.probes = ws.probes.as<int32_t>();
      sa.nq = n;
      sa.nparts = P;
      sa.nprobe = P;
      sa.cmax = 1;
      sa.dim = dim;
      sa.dt = dt;
      sa.bq = ws.sbq.as<_Float16>();
      sa.qsc = ws.sqsc.as<float2>();
      sa.samp = ws.ssamp.as<float>();
      sa.work = ws.swork.as<int32_t>();
      sa.row_limit = 0xFFFFFFFFu;
      sa.rsq16 = s.rsq16.as<float>();
      sa.rsq = s.rsq.as<float>();
      stream_ub_terms(dt, metric, filter_f16_cerr(dt, metric, FILTER_F16X1), filter_cerr(dt),
                      filter_f16_abs(dt, metric, s.sx, FILTER_F16X1), sa);
      sa.mub = s.row_terms(metric, sa.kr, sa.kx, ws.st);
      sa.lioff = ws.ivf_ioff.as<int32_t>();  // the sample pass by list (scan.hip SMP)
      sa.lcnt = ws.ivf_cnt.as<int32_t>();
      sa.nlist = coarse.nlist;
      sa.lqchunk = scan_qmax(dt);
      if (budget) {  // the pairs' budgets, and the sample pass bounded as the unsharded LIM sample is
        ws.shp.ensure(sizeof(int32_t) * npos);
        ws.limits.ensure(sizeof(uint32_t) * npos);
        ws.plim.ensure(sizeof(uint32_t) * npos);
        launch_shard_budget(ws.probes.as<int32_t>(), n, P, prm.max_scans, sgle.as<int32_t>(), sslb.as<int32_t>(),
                            ssle.as<int32_t>(), ws.shp.as<int32_t>(), ws.limits.as<uint32_t>(), ws.st);
        launch_pos_limits(ws.qpos.as<int32_t>(), ws.limits.as<uint32_t>(), npos, ws.plim.as<uint32_t>(), ws.st);
        sa.plim = ws.plim.as<uint32_t>();
      }
      {
        PhaseTimer t(PH_SAMPLE, ws.st);
        stream_sample(sa, metric, maxi, ws.st);
        StreamSelectArgs sel{};
        sel.samp = ws.ssamp.as<float>();
        sel.nq = n;
        sel.n = P * sv;
        stream_rank(k1, sel.rmin, sel.rmax, sel.et);
        sel.probes = ws.probes.as<int32_t>();
        sel.nprobe = P;
        sel.lb = sglb.as<int32_t>();  // the lists' true lengths: the sampled fraction of the unsharded scan
        sel.le = sgle.as<int32_t>();
        sel.thr = ws.sthr.as<float>();
        launch_stream_select(sel, ws.st);
      }
      launch_pack_plan(ws.probes.as<int32_t>(), ws.sthr.as<float>(), budget ? ws.shp.as<int32_t>() : nullptr, n, P,
                       d_plan + a0 * S, ws.st);
      HIPCHK(hipGetLastError());
    }
    return P;
  }

  void shard_search(const float *d_q, int64_t nq, int k, const int32_t *d_plan, int P, bool budget, void *d_rec,
                    Workspace &ws) override {
    if (!built || coarse.nlist <= 0) throw Error(PYR_E_STATE, "index is not built");
    if (metric == COS) throw Error(PYR_E_STATE, "list-sharded search serves L2 / IP");
    if (buf.live_count() > 0) throw Error(PYR_E_STATE, "list-sharded search needs every row in the lists (Build)");
    const int k1 = filter_k1(k);
    if (k <= 0 || k > KMAX_FAST || k1 <= 0 || !stream_ok(k1))
      throw Error(PYR_E_ARG, "topK out of the list-sharded search's range");
    if (P <= 0 || P > coarse.nlist || P >= MAX_PARTS) throw Error(PYR_E_ARG, "plan width does not fit the index");
    if (nq == 0) return;
    if (budget) check_shard_budget_lengths();
    const int S = shard_plan_stride(P, budget);
    ws.shp.ensure(sizeof(int32_t) * nq * P);
    ws.shthr.ensure(sizeof(float) * nq);
    launch_unpack_plan(d_plan, nq, P, S, ws.shp.as<int32_t>(), ws.shthr.as<float>(), ws.st);
    const ShardCtx sh{ws.shthr.as<float>(), static_cast<uint8_t *>(d_rec), budget ? d_plan + P + 1 : nullptr,
                      budget ? S : 0};
    ws.ext_probes = ws.shp.as<int32_t>();
    ws.ext_nprobe = P;
    try {
      search_stream(d_q, nq, k, k1, P, nullptr, nullptr, nullptr, ws, &sh);
    } catch (...) {
      ws.ext_probes = nullptr;
      throw;
    }
    ws.ext_probes = nullptr;
  }

  void shard_rerun(const float *d_q, int64_t nq, int k, const int32_t *d_plan, int P, bool budget,
                   const int32_t *d_fails, int nranks, int fcap, int64_t nq_home, void *d_rec, Workspace &ws) override {
    if (!built || coarse.nlist <= 0) throw Error(PYR_E_STATE, "index is not built");
    if (k <= 0 || k > 64) throw Error(PYR_E_ARG, "topK out of the list-sharded search's range");
    if (fcap <= 0 || nranks <= 0) return;
    const int S = shard_plan_stride(P, budget);
    if (budget) {  // every pair's row bound on this rank's lists, as shard_search bounds the scan
      check_shard_budget_lengths();
      ws.shp.ensure(sizeof(int32_t) * std::max<int64_t>(nq, 1) * P);
      ws.shthr.ensure(sizeof(float) * std::max<int64_t>(nq, 1));
      ws.limits.ensure(sizeof(uint32_t) * std::max<int64_t>(nq, 1) * P);
      launch_unpack_plan(d_plan, nq, P, S, ws.shp.as<int32_t>(), ws.shthr.as<float>(), ws.st);
      IvfChunking c1{1, 1, 0};
      launch_ivf_limits(ws.shp.as<int32_t>(), nq, P, P, 0, dlb.as<int32_t>(), dle.as<int32_t>(), dllive.as<int32_t>(),
                        lists.live.as<uint8_t>(), c1, ws.limits.as<uint32_t>(), ws.st, d_plan + P + 1, S);
    }
    const int64_t mf = (int64_t)nranks * fcap;
    ws.fail.ensure(sizeof(int32_t) * mf);
    ws.rpos.ensure(sizeof(int32_t) * mf);
    ws.fail_cnt.ensure(sizeof(int32_t));
    launch_shard_fail_compact(d_fails, nranks, fcap, nq_home, ws.fail.as<int32_t>(), ws.rpos.as<int32_t>(),
                              ws.fail_cnt.as<int32_t>(), ws.st);
    IvfRerunArgs ra{};
    ra.rows = lists.rows.as<float>();
    ra.live = lists.live.as<uint8_t>();
    ra.labels = lists.labels.as<int64_t>();
    ra.queries = d_q;
    ra.probes = d_plan;
    ra.nprobe = P;
    ra.pstride = S;
    ra.qlim = budget ? ws.limits.as<uint32_t>() : nullptr;
    ra.lb = dlb.as<int32_t>();
    ra.le = dle.as<int32_t>();
    ra.fail = ws.fail.as<int32_t>();
    ra.nfail = ws.fail_cnt.as<int32_t>();
    ra.dim = dim;
    ra.k = k;
    // a rank re-runs a handful of queries over the few of their lists it holds: 4,096-row chunks (1,024 would
    // cut each probed list 10-18 ways and leave one wave ~6k partial keys to merge per query)
    ra.nchunk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, (max_len + 4095) / 4096));
    ra.rec = d_rec;
    ra.rec_pos = ws.rpos.as<int32_t>();
    ra.rec_lb = dlb.as<int32_t>();
    ra.rec_nlist = coarse.nlist;
    PhaseTimer t(PH_FALLBACK, ws.st);
    // (no fused merge here: a rank's re-run list is rarely empty, and the fused merge's agent-scope fences --
    // L2 write-back / invalidate across the XCDs -- cost more than the launch they save: 0.085 vs 0.077 ms at
    // the N = 8 rank shape, profiles/r5_i1/rank8_rerun_fused_ab.log)
    ws.rrpart.ensure(sizeof(uint64_t) * ivf_rerun_part_keys(mf, P, k));
    launch_ivf_exact_rerun(ra, metric, mf, ws.rrpart.as<uint64_t>(), ws.st);
    HIPCHK(hipGetLastError());
  }

  // IvfFlatVectorIndex.Search (:147-231) with the list scan on the VALU, the reference's exact arithmetic
  void search_exact(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, float *d_s, int64_t *d_l,
                    int32_t *d_c, Workspace &ws) {
    const int nprobe = prm.nprobe < 0 ? nprobe_default : prm.nprobe;                  // :151-158
    const int64_t maxs = prm.max_scans < 0 ? (int64_t)INT32_MAX : prm.max_scans;       // :152
    // (ws.skip_buffer: the lists alone -- a stream search's re-run, whose buffer search() merges itself)
    const int64_t blive = ws.skip_buffer ? 0 : buf.live_count();
    const int64_t bcut = buf.cutoff(std::min<int64_t>(maxs, blive));
    const int64_t bscanned = std::min<int64_t>(maxs, blive);
    const bool index_on = built && coarse.nlist > 0 && bscanned < maxs;                // :183
    const int probes = index_on ? std::max(0, std::min(nprobe, coarse.nlist)) : 0;    // :198
    if (probes >= MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    ScanPlan bp;
    if (bcut > 0) bp = plan_flat(bcut, nq, dim, k, std::max(1, std::min(64, MAX_PARTS - probes)));
    const IvfChunking ch =
        probes > 0 ? ivf_chunking(max_len, probes, bp.nchunks, nq, k, bounds_enabled()) : IvfChunking{8, 1, 0};
    const int nparts = probes * ch.cmax + bp.nchunks;
    if (nparts > MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    if (nparts == 0) {
      fill_empty_results(d_s, d_l, d_c, nq, k, ws.st);
      return;
    }
    prep_queries(d_q, nq, dim, metric, ws);
    const float *qn = metric == COS ? ws.qn.as<float>() : nullptr;
    const size_t np = (size_t)nq * nparts * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    uint32_t *gthr = shared_bounds(ws, nq);
    if (probes > 0) {
      {
        PhaseTimer t(PH_COARSE, ws.st, nq * coarse.nlist);
        coarse.probe(d_q, qn, nq, probes, metric, ws);
      }
      const int qchunk = fast_path(dim, k) ? QCHUNK : QCHUNK_GENERIC;
      int maxi, maxi_main = 0;
      {
        PhaseTimer t(PH_ITEMS, ws.st);
        maxi = build_ivf_items(ws, nq, probes, nparts, coarse.nlist, dlb, dle, qchunk, ch, 0);
        if (ch.warm > 0) maxi_main = build_ivf_items(ws, nq, probes, nparts, coarse.nlist, dlb, dle, qchunk, ch, 1);
      }
      const uint32_t *lim = nullptr;
      if (prm.max_scans >= 0) {  // :202-212
        ws.limits.ensure(sizeof(uint32_t) * nq * nparts);
        launch_ivf_limits(ws.probes.as<int32_t>(), nq, probes, nparts, maxs - bscanned, dlb.as<int32_t>(),
                          dle.as<int32_t>(), dllive.as<int32_t>(), lists.live.as<uint8_t>(), ch,
                          ws.limits.as<uint32_t>(), ws.st);
        lim = ws.limits.as<uint32_t>();
      }
      ScanArgs a{};
      a.rows = lists.rows.as<float>();
      a.live = lists.live.as<uint8_t>();
      a.rnorm = lists.cosine ? lists.norms.as<float>() : nullptr;
      a.queries = d_q;
      a.queries_t = ws.qt.as<float>();
      a.qnorm = qn;
      a.items = ws.items.as<ScanItem>();
      a.n_items = ws.nitems.as<int32_t>();
      a.qlist = ws.qlist.as<int32_t>();
      a.limits = lim;
      a.nparts = nparts;
      a.k = k;
      a.key_base = 0;
      a.dim = dim;
      a.part_s = ws.part_s.as<float>();
      a.part_k = ws.part_k.as<uint32_t>();
      a.gthr = gthr;
      PhaseTimer t(PH_LIST_SCAN, ws.st, prof().on ? probed_rows(ws, nq, probes, le, lb) : 0);
      launch_scan(a, metric, 1, maxi, ws.st);  // chunk 0 of every list (all chunks when ch.warm == 0)
      if (ch.warm > 0) {                       // the rest, behind the bounds the first launch published
        a.items = ws.items3.as<ScanItem>();
        a.n_items = ws.nitems3.as<int32_t>();
        launch_scan(a, metric, 1, maxi_main, ws.st);
      }
    }
    if (bcut > 0) {  // :170-180 exact buffer scan, keys KEY_BUF | slot
      PhaseTimer t(PH_BUF_SCAN, ws.st, nq * bcut);
      flat_scan(buf.st, bcut, bp, d_q, qn, nq, k, 1, metric, nparts, probes * ch.cmax, KEY_BUF, ws,
                ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), true, gthr);
    }
    PhaseTimer tm(PH_MERGE, ws.st);
    MergeIvf mi;
    if (probes > 0) {
      mi.probes = ws.probes.as<int32_t>();
      mi.lb = dlb.as<int32_t>();
      mi.le = dle.as<int32_t>();
      mi.nprobe = probes;
      mi.ch = ch;
    }
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, nparts, k, lists.labels.as<int64_t>(),
                      buf.st.labels.as<int64_t>(), d_s, d_l, nullptr, d_c, ws.st, &mi);
  }

  void snapshot(const std::string &path) override {  // :233-257 IvfStateDto
    ImageWriter w(path, PYR_IVF_FLAT, dim, metric);
    const uint8_t b = built ? 1 : 0;
    w.host(T_BUILT, &b, 1);
    if (built) {
      w.host(T_CENTS, coarse.host.data(), sizeof(float) * coarse.host.size());
      // _invertedLists in order: visible and buffer-shadowed entries (removed ones are gone, :61-83)
      std::vector<int32_t> cnt(coarse.nlist, 0);
      std::vector<int64_t> slots, labels;
      for (int l = 0; l < coarse.nlist; l++)
        for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++)
          if (lstate[p]) {
            cnt[l]++;
            slots.push_back(p);
            labels.push_back(lists.hlabels[p]);
          }
      w.host(T_LCOUNT, cnt.data(), sizeof(int32_t) * cnt.size());
      write_rows(w, T_LLABELS, T_LROWS, lists, slots, labels, stage_x, stage_i, wst);
    }
    std::vector<int64_t> blabels;
    const std::vector<int64_t> bslots = live_slots(buf.st, blabels);
    write_rows(w, T_BLABELS, T_BROWS, buf.st, bslots, blabels, stage_x, stage_i, wst);
    w.commit();
  }

  void load(const std::string &path) override {  // :259-298
    ImageReader r(path);
    check_image(r, PYR_IVF_FLAT, *this);
    buf.clear(wst);
    built = false;
    lists.clear();
    lstate.clear();
    pos_of.clear();
    lb.clear();
    le.clear();
    llen.clear();
    llive.clear();
    max_len = 0;
    uint8_t b = 0;
    if (r.has(T_BUILT)) r.host(T_BUILT, &b, 1);
    const std::vector<float> cents = r.vec<float>(T_CENTS);
    if (cents.size() % (size_t)dim != 0) ImageReader::throw_format("centroids are not whole rows");
    const int k = (int)(cents.size() / dim);
    if (b && k > 0) {
      const std::vector<int32_t> cnt = r.vec<int32_t>(T_LCOUNT);
      if ((int)cnt.size() != k) ImageReader::throw_format("list counts do not match the centroids");
      const std::vector<int64_t> labels = r.vec<int64_t>(T_LLABELS);
      std::vector<int32_t> asg;
      asg.reserve(labels.size());
      for (int l = 0; l < k; l++) asg.insert(asg.end(), (size_t)cnt[l], l);
      if (asg.size() != labels.size()) ImageReader::throw_format("list counts do not match the labels");
      const int64_t n = (int64_t)labels.size();
      DevMem X, C;
      X.ensure(sizeof(float) * std::max<int64_t>(n, 1) * dim);
      if (n) r.device(T_LROWS, X.p, sizeof(float) * n * dim, wst);
      C.ensure(sizeof(float) * k * dim);
      HIPCHK(hipMemcpyAsync(C.p, cents.data(), sizeof(float) * k * dim, hipMemcpyHostToDevice, wst));
      commit_lists(X.as<float>(), n, asg, labels, C.as<float>(), k);
      built = true;
    }
    std::vector<int64_t> blabels;
    std::vector<float> brows;
    const int64_t nb = read_rows(r, T_BLABELS, T_BROWS, dim, blabels, brows);
    if (nb) add(brows.data(), nb, blabels.data(), true);  // buffer ids shadow their list entries (:210)
  }

  int64_t count() const override {  // :305 buffer + all list entries (shadowed ones too)
    int64_t c = buf.live_count();
    for (uint8_t s : lstate) c += s != 0;
    return c;
  }
  void all_labels(std::vector<int64_t> &out) const override {
    buf.all_labels(out);
    for (size_t p = 0; p < lstate.size(); p++)
      if (lstate[p] != 0) out.push_back(lists.hlabels[p]);
  }

  void centroids(float *out, int32_t *nl) const override {  // :314-325
    *nl = built ? coarse.nlist : 0;
    if (out && built) std::memcpy(out, coarse.host.data(), sizeof(float) * coarse.host.size());
  }

  void ivf_layout(int64_t *off, int64_t *labels, uint8_t *live, int64_t *total) const override {
    int64_t t = 0;
    for (int l = 0; l < coarse.nlist && built; l++) {
      if (off) off[l] = t;
      for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++, t++) {
        if (labels) labels[t] = lstate[p] ? lists.hlabels[p] : -1;
        if (live) live[t] = lstate[p] == 1;
      }
    }
    if (off && built) off[coarse.nlist] = t;
    *total = t;
  }
};

// ---------------------------------------------------------------------------
// IVF_PQ = IvfPqVectorIndex + ProductQuantizer
// ---------------------------------------------------------------------------
struct IvfPqIndex : Index {
  DictBuffer buf;                    // _buffer (:19)
  int M, K, sub;
  DevMem codes, clive, clabels;      // blocked codes, per code-row visibility, labels
  std::vector<int64_t> hlabels;      // per code row (-1 pad)
  std::vector<uint8_t> hlive;
  int64_t key_label(uint32_t key) const override {
    return (size_t)key < hlive.size() && hlive[key] ? hlabels[key] : -1;
  }
  std::unordered_map<int64_t, int64_t> pos_of;
  std::vector<int32_t> lb, le, llen;
  DevMem dlb, dle;
  Coarse coarse;
  DevMem cb;                         // [M][ksub][sub]
  int ksub = 0;
  int64_t ncode_rows = 0;
  // the matrix-core list scan (pq32.hip): tile code layout, |x^|^2 per position, fp16 codebook and its
  // power-of-two scale, the per-position row terms (cached for (pq_gen, kr)); pq_gen advances with clive
  bool pq32_ready = false;
  DevMem cpack, nrm, cb16, pmeta, pmub;
  float cbsx = 1.0f;
  uint64_t pq_gen = 1, pmub_gen = 0;
  float pmub_kr = 0.0f;
  int64_t pq_max_len = 0;
  bool built = false;
  int nprobe_default;
  std::vector<float> given;
  int given_k = 0;

  void set_centroids(const float *c, int nl) override {
    if (nl <= 0) throw Error(PYR_E_ARG, "nlist must be positive");
    given.assign(c, c + (size_t)nl * dim);
    given_k = nl;
  }
  std::vector<float> given_cb;  // pyr_index_set_codebooks: [M][ksub][sub]
  int given_ksub = 0;
  void set_codebooks(const float *c, int m, int ks) override {
    if (m != M) throw Error(PYR_E_ARG, "codebooks have " + std::to_string(m) + " subspaces, the index " + std::to_string(M));
    if (ks <= 0 || ks > 256) throw Error(PYR_E_ARG, "K must be <= 256 for byte encoding");
    given_cb.assign(c, c + (size_t)m * ks * sub);
    given_ksub = ks;
  }
  void reserve(int64_t rows) override { buf.reserve(rows, wst); }

  explicit IvfPqIndex(const pyr_index_desc &d) : Index(d) {
    M = d.pq_m;
    K = d.pq_k;
    if (M <= 0 || dim % M != 0) throw Error(PYR_E_ARG, "Dimension must be divisible by M");  // PQ.cs:18
    if (K > 256 || K <= 0) throw Error(PYR_E_ARG, "K must be <= 256 for byte encoding");    // PQ.cs:19
    sub = dim / M;
    buf.st.dim = dim;
    buf.st.cosine = metric == COS;
    nprobe_default = d.default_nprobe > 0 ? d.default_nprobe : 1;  // :125
  }

  void set_shadow(int64_t label, uint8_t visible, std::vector<int64_t> &on, std::vector<int64_t> &off) {
    auto f = pos_of.find(label);
    if (f == pos_of.end()) return;
    if (hlive[f->second] == visible) return;
    hlive[f->second] = visible;
    (visible ? on : off).push_back(f->second);
  }
  void push_live(const std::vector<int64_t> &slots, uint8_t v) {
    if (slots.empty()) return;
    stage_b.ensure(sizeof(int64_t) * slots.size());
    HIPCHK(hipMemcpyAsync(stage_b.p, slots.data(), sizeof(int64_t) * slots.size(), hipMemcpyHostToDevice, wst));
    launch_scatter_u8(clive.as<uint8_t>(), stage_b.as<int64_t>(), v, (int64_t)slots.size(), wst);
    HIPCHK(hipStreamSynchronize(wst));
    ++pq_gen;
  }

  void add(const float *x, int64_t n, const int64_t *labels, bool) override {  // :37-47
    buf.write(x, labels, n, wst, stage_x, stage_i);
    std::vector<int64_t> on, off;
    for (int64_t i = 0; i < n; i++) set_shadow(labels[i], 0, on, off);  // seen (:134,170)
    push_live(off, 0);
  }

  void remove(const int64_t *labels, int64_t n, uint8_t *removed) override {  // :48-53 buffer only
    std::vector<int64_t> dead, on, off;
    for (int64_t i = 0; i < n; i++) {
      const bool r = buf.erase(labels[i], dead);
      if (removed) removed[i] = r;
      if (r) set_shadow(labels[i], 1, on, off);  // no longer "seen": list entry visible again
    }
    buf.st.set_live(dead, 0, wst, stage_b);
    push_live(on, 1);
  }

  void build() override {  // :55-116
    if (buf.live_count() == 0 && !built) return;      // :60
    std::vector<int64_t> slots, labs;                 // allVectors = _buffer.Values (:64)
    for (int64_t s = 0; s < buf.st.n; s++)
      if (buf.st.hlive[s]) {
        slots.push_back(s);
        labs.push_back(buf.st.hlabels[s]);
      }
    const int64_t n = (int64_t)slots.size();
    if (n == 0) return;                               // :65
    if (given_k > 0 && given_ksub > 0) {
      build_given(slots, labs);
      return;
    }
    DevMem X, ds;
    X.ensure(sizeof(float) * n * dim);
    ds.ensure(sizeof(int64_t) * n);
    HIPCHK(hipMemcpyAsync(ds.p, slots.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, wst));
    launch_gather_blocked(buf.st.rows.as<float>(), ds.as<int64_t>(), n, dim, X.as<float>(), wst);
    int nc = (int)std::min<int64_t>(desc.nlist, n);   // :68
    if (nc <= 0) nc = 1;
    DevMem C;
    if (given_k > 0) {
      nc = given_k;
      C.ensure(sizeof(float) * nc * dim);
      HIPCHK(hipMemcpyAsync(C.p, given.data(), sizeof(float) * nc * dim, hipMemcpyHostToDevice, wst));
    } else {
      C.ensure(sizeof(float) * nc * dim);
      nc = kmeans_train_gpu(X.as<float>(), n, dim, nc, metric, 10, 123, C.as<float>(), wst);  // :69
    }
    DevMem A, R, S;
    A.ensure(sizeof(int32_t) * n);
    assign_gpu(X.as<float>(), n, dim, C.as<float>(), nc, metric, A.as<int32_t>(), wst);   // :79
    R.ensure(sizeof(float) * n * dim);
    launch_residuals(X.as<float>(), A.as<int32_t>(), C.as<float>(), n, dim, R.as<float>(), wst);  // :82-85
    // PQ train (ProductQuantizer.cs:28-58): per subspace k-means, L2, seed 42+m
    ksub = (int)std::min<int64_t>(K, n);
    if (ksub <= 0) ksub = 1;
    cb.ensure(sizeof(float) * (size_t)M * ksub * sub);
    S.ensure(sizeof(float) * n * sub);
    for (int m = 0; m < M; m++) {
      launch_extract_sub(R.as<float>(), n, dim, m * sub, sub, S.as<float>(), wst);
      kmeans_train_gpu(S.as<float>(), n, sub, K, L2, 10, 42 + m, cb.as<float>() + (size_t)m * ksub * sub, wst);
    }
    // Encode (:99-107)
    DevMem codes_rm;
    codes_rm.ensure((size_t)n * M);
    launch_pq_encode(X.as<float>(), A.as<int32_t>(), C.as<float>(), n, dim, M, ksub, cb.as<float>(),
                     codes_rm.as<uint8_t>(), wst);
    std::vector<int32_t> asg(n);
    HIPCHK(hipMemcpyAsync(asg.data(), A.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, wst));
    HIPCHK(hipStreamSynchronize(wst));
    commit_codes(codes_rm.as<uint8_t>(), n, asg, labs, C.as<float>(), nc);
    buf.clear(wst);                                    // :109
    built = true;
  }

  // Build with a supplied quantizer and codebooks (pyr_index_set_centroids + set_codebooks): the
  // assignment (:79, FindNearestCentroid) and Encode (:99-107) of every buffer row, in chunks of
  // ~1 GiB of gathered rows, so a buffer of 10^8 rows needs no second full copy (nor residuals).
  void build_given(const std::vector<int64_t> &slots, const std::vector<int64_t> &labs) {
    const int64_t n = (int64_t)slots.size();
    const int nc = given_k;
    DevMem C;
    C.ensure(sizeof(float) * nc * dim);
    HIPCHK(hipMemcpyAsync(C.p, given.data(), sizeof(float) * nc * dim, hipMemcpyHostToDevice, wst));
    ksub = given_ksub;
    cb.ensure(sizeof(float) * (size_t)M * ksub * sub);
    HIPCHK(hipMemcpyAsync(cb.p, given_cb.data(), sizeof(float) * given_cb.size(), hipMemcpyHostToDevice, wst));
    DevMem codes_rm, A, X, ds;
    codes_rm.ensure((size_t)n * M);
    A.ensure(sizeof(int32_t) * n);
    int64_t chunk = std::max<int64_t>(1024, (int64_t(1) << 30) / ((int64_t)dim * 4));
    if (const char *e = knob("PYR_PQ_BUILD_CHUNK")) chunk = std::max<int64_t>(1, atoll(e));  // tests
    X.ensure(sizeof(float) * std::min(chunk, n) * dim);
    ds.ensure(sizeof(int64_t) * std::min(chunk, n));
    const bool progress = getenv("PYR_PROGRESS") && atoi(getenv("PYR_PROGRESS")) != 0;  // long bulk builds
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t off = 0; off < n; off += chunk) {
      if (progress && (off / chunk) % 8 == 0) {
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[pyrope] IVF_PQ build: %lld / %lld rows assigned + encoded (%.1fs)\n", (long long)off,
                (long long)n, s);
        fflush(stderr);
      }
      const int64_t cn = std::min(chunk, n - off);
      HIPCHK(hipMemcpyAsync(ds.p, slots.data() + off, sizeof(int64_t) * cn, hipMemcpyHostToDevice, wst));
      launch_gather_blocked(buf.st.rows.as<float>(), ds.as<int64_t>(), cn, dim, X.as<float>(), wst);
      assign_gpu(X.as<float>(), cn, dim, C.as<float>(), nc, metric, A.as<int32_t>() + off, wst);
      launch_pq_encode(X.as<float>(), A.as<int32_t>() + off, C.as<float>(), cn, dim, M, ksub, cb.as<float>(),
                       codes_rm.as<uint8_t>() + (size_t)off * M, wst);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(wst));
    }
    X.release();
    std::vector<int32_t> asg(n);
    HIPCHK(hipMemcpyAsync(asg.data(), A.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, wst));
    HIPCHK(hipStreamSynchronize(wst));
    commit_codes(codes_rm.as<uint8_t>(), n, asg, labs, C.as<float>(), nc);
    buf.clear(wst);
    built = true;
  }

  // codes (device, row-major n x M; row i has label labs[i]) into the list-major blocked layout by
  // list asg[i] (lists keep code order, padded to 64 rows), with quantizer C (nc x dim, device)
  void commit_codes(const uint8_t *codes_rm, int64_t n, const std::vector<int32_t> &asg,
                    const std::vector<int64_t> &labs, const float *C, int nc) {
    std::vector<int32_t> cnt(nc, 0);
    for (int32_t a : asg) cnt[a]++;
    lb.assign(nc, 0);
    le.assign(nc, 0);
    llen = cnt;
    int64_t tot = 0;
    for (int l = 0; l < nc; l++) {
      lb[l] = (int32_t)tot;
      le[l] = (int32_t)(tot + cnt[l]);
      tot += round_up(cnt[l], 64);
    }
    std::vector<int64_t> src(tot, -1);
    hlabels.assign(tot, -1);
    std::vector<int32_t> fillp(lb);
    for (int64_t i = 0; i < n; i++) {
      const int32_t p = fillp[asg[i]]++;
      src[p] = i;
      hlabels[p] = labs[i];
    }
    const int nch = (M + 15) / 16;
    codes.ensure((size_t)std::max<int64_t>(tot, 64) * nch * 16);
    DevMem dsrc;
    dsrc.ensure(sizeof(int64_t) * std::max<int64_t>(tot, 1));
    HIPCHK(hipMemcpyAsync(dsrc.p, src.data(), sizeof(int64_t) * tot, hipMemcpyHostToDevice, wst));
    launch_pack_codes(codes_rm, dsrc.as<int64_t>(), tot, M, codes.as<uint8_t>(), wst);
    pq32_ready = false;
    if (pq32_supported(dim, M, ksub, 10)) {
      // tile code layout + |x^|^2 per position; fp16 codebook with a power-of-two scale keeping max |C| < 2^14
      const int64_t tiles = (tot + 31) / 32;
      const size_t cbytes = (size_t)std::max<int64_t>(tiles, 1) * 64 * 16 * pq32_lane_words(dim, M);
      cpack.ensure(cbytes);
      HIPCHK(hipMemsetAsync(cpack.p, 0, cbytes, wst));
      nrm.ensure(sizeof(float) * (size_t)std::max<int64_t>(tiles * 32, 1));
      HIPCHK(hipMemsetAsync(nrm.p, 0, sizeof(float) * (size_t)std::max<int64_t>(tiles * 32, 1), wst));
      launch_pq32_pack(codes_rm, dsrc.as<int64_t>(), tot, M, sub, cb.as<float>(), ksub, cpack.as<uint8_t>(),
                       nrm.as<float>(), wst);
      std::vector<float> hcb((size_t)M * ksub * sub);
      HIPCHK(hipMemcpyAsync(hcb.data(), cb.p, sizeof(float) * hcb.size(), hipMemcpyDeviceToHost, wst));
      HIPCHK(hipStreamSynchronize(wst));
      float am = 0.0f;
      bool fin = true;
      for (float v : hcb) {
        fin = fin && std::isfinite(v);
        am = std::max(am, std::fabs(v));
      }
      cbsx = pow2_scale_host(am);
      cb16.ensure(sizeof(uint16_t) * (size_t)M * 256 * sub);
      launch_pq32_cb16(cb.as<float>(), M, ksub, sub, cbsx, cb16.as<_Float16>(), wst);
      HIPCHK(hipGetLastError());
      pq32_ready = fin;
      ++pq_gen;
    }
    hlive.assign(tot, 0);
    for (int64_t p = 0; p < tot; p++) hlive[p] = src[p] >= 0;
    clive.ensure(std::max<int64_t>(tot, 1));
    clabels.ensure(sizeof(int64_t) * std::max<int64_t>(tot, 1));
    HIPCHK(hipMemcpyAsync(clive.p, hlive.data(), tot, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(clabels.p, hlabels.data(), sizeof(int64_t) * tot, hipMemcpyHostToDevice, wst));
    ncode_rows = tot;
    pq_max_len = 0;
    for (int32_t v : cnt) pq_max_len = std::max<int64_t>(pq_max_len, v);
    pos_of.clear();
    for (int64_t p = 0; p < tot; p++)
      if (hlabels[p] >= 0) pos_of[hlabels[p]] = p;
    coarse.set(C, nc, dim, metric, wst);
    dlb.ensure(sizeof(int32_t) * nc);
    dle.ensure(sizeof(int32_t) * nc);
    HIPCHK(hipMemcpyAsync(dlb.p, lb.data(), sizeof(int32_t) * nc, hipMemcpyHostToDevice, wst));
    HIPCHK(hipMemcpyAsync(dle.p, le.data(), sizeof(int32_t) * nc, hipMemcpyHostToDevice, wst));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(wst));
  }

  void search(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, float *d_s, int64_t *d_l,
              int32_t *d_c, Workspace &ws) override {  // :118-212 (MaxScans ignored)
    if (k <= 0 || nq == 0) {
      fill_empty_results(d_s, d_l, d_c, nq, std::max(k, 0), ws.st);
      return;
    }
    const int nprobe = prm.nprobe < 0 ? nprobe_default : prm.nprobe;
    const int probes = (built && coarse.nlist > 0) ? std::max(0, std::min(nprobe, coarse.nlist)) : 0;
    // the matrix-core scan: built lists only (no buffer rows), the P1 geometry (pq32_supported)
    const char *pm = knob("PYR_PQ_MFMA");  // 0: the LUT scan below (A/B and the re-run path)
    if (!(pm && atoi(pm) == 0) && pq32_ready && probes > 0 && filter_enabled() && pq32_supported(dim, M, ksub, k) &&
        pq32_depth(k, ws) > 0) {
      if (buf.live_count() == 0) {
        search_pq32(d_q, nq, k, probes, d_s, d_l, d_c, ws);
        return;
      }
      // a non-empty buffer (:130-136): the lists on the matrix cores, the buffer exactly beside them, the two
      // answers merged (a list entry first on equal scores, as the LUT path's keys order them)
      ws.bx_s.ensure(sizeof(float) * nq * k);
      ws.bx_l.ensure(sizeof(int64_t) * nq * k);
      ws.bx_c.ensure(sizeof(int32_t) * nq);
      ws.lx_s.ensure(sizeof(float) * nq * k);
      ws.lx_l.ensure(sizeof(int64_t) * nq * k);
      ws.lx_c.ensure(sizeof(int32_t) * nq);
      search_pq32(d_q, nq, k, probes, ws.lx_s.as<float>(), ws.lx_l.as<int64_t>(), ws.lx_c.as<int32_t>(), ws);
      buffer_topk(d_q, nq, k, ws.bx_s.as<float>(), ws.bx_l.as<int64_t>(), ws.bx_c.as<int32_t>(), ws);
      PhaseTimer tm(PH_MERGE, ws.st);
      launch_merge_two(ws.lx_s.as<float>(), ws.lx_l.as<int64_t>(), ws.lx_c.as<int32_t>(), ws.bx_s.as<float>(),
                       ws.bx_l.as<int64_t>(), ws.bx_c.as<int32_t>(), nq, k, d_s, d_l, d_c, ws.st);
      HIPCHK(hipGetLastError());
      return;
    }
    search_lut(d_q, nq, k, probes, d_s, d_l, d_c, ws);
  }

  // the buffer's exact top k (:130-136, ComputeScore) in (score desc, slot asc) order
  void buffer_topk(const float *d_q, int64_t nq, int k, float *d_s, int64_t *d_l, int32_t *d_c, Workspace &ws) {
    const int64_t bcut = buf.st.n;
    const ScanPlan bp = plan_flat(bcut, nq, dim, k, MAX_PARTS);
    prep_queries(d_q, nq, dim, metric, ws);
    const float *qn = metric == COS ? ws.qn.as<float>() : nullptr;
    const size_t np = (size_t)nq * bp.nchunks * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    {
      PhaseTimer t(PH_BUF_SCAN, ws.st, nq * bcut);
      flat_scan(buf.st, bcut, bp, d_q, qn, nq, k, 1, metric, bp.nchunks, 0, KEY_BUF, ws, ws.part_s.as<float>(),
                ws.part_k.as<uint32_t>(), true);
    }
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, bp.nchunks, k, clabels.as<int64_t>(),
                      buf.st.labels.as<int64_t>(), d_s, d_l, nullptr, d_c, ws.st, nullptr);
  }

  // the per-position row terms of the fp16 filter: -|x^|^2 (or -inf when not visible) + kr |x^|^2
  const float *pq_row_terms(float kr, Workspace &ws) {
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const int64_t tot = (ncode_rows + 31) / 32 * 32;
    if (pmub_gen == pq_gen && pmub_kr == kr && pmub.n >= sizeof(float) * tot) return pmub.as<float>();
    if (capturing(ws.st))
      throw Error(PYR_E_STATE, "the index changed since its last search and its per-row terms must be "
                               "refreshed: run one search outside the stream capture first");
    pmeta.ensure(sizeof(float) * std::max<int64_t>(tot, 1));
    pmub.ensure(sizeof(float) * std::max<int64_t>(tot, 1));
    WordFill z;
    z.add(pmeta.p, tot, 0xFF800000u);  // -inf: not a row
    launch_fill_words(z, ws.st);
    launch_pq32_meta(nrm.as<float>(), clive.as<uint8_t>(), ncode_rows, pmeta.as<float>(), ws.st);
    launch_row_terms(pmeta.as<float>(), nrm.as<float>(), nullptr, tot, L2, kr, 0.0f, pmub.as<float>(), ws.st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ws.st));
    pmub_gen = pq_gen;
    pmub_kr = kr;
    return pmub.as<float>();
  }

  // IvfPqVectorIndex.Search (:118-212) on the matrix cores (pq32.hip): coarse ranking, per (list chunk,
  // <= 64 queries) item the decoded rows' approximate ADC bounds -> rows reaching the query's sampled
  // threshold -> the reference's ADC sum of the best 64, certified; what fails re-runs on the LUT scan.
  // the refine depth K1 of the matrix-core scan: filter_k1 (k <= 60), else the deep refine's 128 / 256 / 512
  // (deep_k1; not for caller-ranked probe lists, as the IVF_FLAT stream's); 0: the LUT scan
  static int pq32_depth(int k, const Workspace &ws) {
    const int k1 = filter_k1(k);
    if (k1 > 0) return k1;
    return !ws.ext_probes && deep_refine_on() ? deep_k1(k, true) : 0;
  }

  void search_pq32(const float *d_q, int64_t nq, int k, int probes, float *d_s, int64_t *d_l, int32_t *d_c,
                   Workspace &ws) {
    const int k1 = pq32_depth(k, ws);
    if (k1 <= 0) throw Error(PYR_E_STATE, "pq32: no refine depth for this k");
    const int cap = k1 > STREAM_KO ? deep_cap(k1) : stream_cap();
    IvfChunking ch{(int32_t)stream_chunk(), 1, 0};
    // a list's items on one XCD (pq32.hip: its code chunks leave HBM once per L2); PYR_PQ_XCD=0: one queue (A/B)
    ch.xcd = knob("PYR_PQ_XCD") && atoi(knob("PYR_PQ_XCD")) == 0 ? 0 : 1;
    ch.cmax = std::max(1, ivf_list_chunks((int)pq_max_len, ch));
    if ((int64_t)probes * ch.cmax > MAX_PARTS) {
      const int64_t room = std::max<int64_t>(1, MAX_PARTS / std::max(probes, 1));
      ch.chunk = (int32_t)round_up(std::max<int64_t>(32, (pq_max_len + room - 1) / room), 32);
      ch.cmax = ivf_list_chunks((int)pq_max_len, ch);
    }
    const int nparts = probes * ch.cmax;
    if (nparts > MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    const int64_t qs = stream_slice_queries(nq, probes, dim, cap, pq32_sample_values());
    const int32_t *ext = ws.ext_probes;  // caller-ranked probe lists: each slice takes its own rows
    for (int64_t a0 = 0; a0 < nq; a0 += qs) {
      const int64_t n = std::min(qs, nq - a0);
      if (ext) ws.ext_probes = ext + a0 * ws.ext_nprobe;
      try {
        pq32_slice(d_q + a0 * dim, n, k, k1, probes, ch, nparts, cap, d_s + a0 * k, d_l + a0 * k,
                   d_c ? d_c + a0 : nullptr, ws);
      } catch (...) {
        ws.ext_probes = ext;
        throw;
      }
      ws.ext_probes = ext;
    }
  }

  void pq32_slice(const float *d_q, int64_t nq, int k, int k1, int probes, IvfChunking ch, int nparts, int cap,
                  float *d_s, int64_t *d_l, int32_t *d_c, Workspace &ws) {
    reset_stream_counters(ws, nq, coarse.nlist);
    {
      PhaseTimer t(PH_COARSE, ws.st, nq * coarse.nlist);
      prep_queries(d_q, nq, dim, metric, ws);
      coarse.probe(d_q, metric == COS ? ws.qn.as<float>() : nullptr, nq, probes, metric, ws);
    }
    int maxi;
    {
      PhaseTimer t(PH_ITEMS, ws.st);
      maxi = build_ivf_items(ws, nq, probes, nparts, coarse.nlist, dlb, dle, pq32_qmax(dim, M), ch, 0, true, true);
    }
    const int64_t npos = nq * probes;
    const int sv = pq32_sample_values();
    ws.sbq.ensure(sizeof(uint16_t) * std::max<int64_t>(npos, 1) * dim);
    ws.sqsc.ensure(sizeof(float2) * std::max<int64_t>(npos, 1));
    ws.ssamp.ensure(sizeof(float) * std::max<int64_t>(npos, 1) * sv);
    ws.sthr.ensure(sizeof(float) * nq);
    ws.scand.ensure(sizeof(uint2) * (size_t)std::max<int64_t>(nq, 1) * cap);
    ws.scn.ensure(sizeof(int32_t) * std::max<int64_t>(nq, 1));
    ws.scf.ensure(sizeof(uint32_t) * std::max<int64_t>(nq, 1));
    ws.swork.ensure(sizeof(int32_t) * 2);
    StreamArgs sa{};
    sa.h16 = cpack.p;
    sa.queries = d_q;
    sa.cents = coarse.rm.as<float>();
    sa.probes = ws.probes.as<int32_t>();
    sa.sx = cbsx;
    sa.items = ws.items.as<ScanItem>();
    sa.n_items = ws.nitems.as<int32_t>();
    sa.qlist = ws.qlist.as<int32_t>();
    sa.nparts = nparts;
    sa.nprobe = probes;
    sa.cmax = ch.cmax;
    sa.dim = dim;
    sa.bq = ws.sbq.as<_Float16>();
    sa.qsc = ws.sqsc.as<float2>();
    sa.samp = ws.ssamp.as<float>();
    sa.thr = ws.sthr.as<float>();
    sa.cand = ws.scand.as<uint2>();
    sa.cand_n = ws.scn.as<int32_t>();
    sa.cand_f = ws.scf.as<uint32_t>();
    sa.cap = cap;
    sa.work = ws.swork.as<int32_t>();
    sa.key_base = 0;
    sa.row_limit = 0xFFFFFFFFu;
    sa.ablate = filter_ablate();
    // the fp16 filter's bound with x^ in the role of x - c: X = |x^| (nrm), A = |r|
    stream_ub_terms(dim, L2, filter_f16_cerr(dim, L2, FILTER_F16X1), filter_cerr(dim),
                    filter_f16_abs(dim, L2, cbsx, FILTER_F16X1), sa);
    sa.mub = pq_row_terms(sa.kr, ws);
    {
      PhaseTimer t(PH_SAMPLE, ws.st);
      launch_pq32_prep(sa, npos, ws.st);
      launch_pq32_scan(sa, cb16.as<_Float16>(), M, maxi, true, ws.st);
      StreamSelectArgs sel{};
      sel.samp = ws.ssamp.as<float>();
      sel.nq = nq;
      sel.n = probes * sv;
      stream_rank(k1, sel.rmin, sel.rmax, sel.et);
      sel.probes = ws.probes.as<int32_t>();
      sel.nprobe = probes;
      sel.lb = dlb.as<int32_t>();
      sel.le = dle.as<int32_t>();
      sel.thr = ws.sthr.as<float>();
      launch_stream_select(sel, ws.st);
    }
    sa.work = ws.swork.as<int32_t>() + 8;  // the main pass's 8 queue counters
    {
      PhaseTimer t(PH_PQ_SCAN, ws.st, prof().on ? probed_rows(ws, nq, probes, le, lb) : 0);
      launch_pq32_scan(main_scan_args(sa), cb16.as<_Float16>(), M, maxi, false, ws.st);
    }
    note_stream_slice(ws, nq, cap);
    const bool deep = k1 > STREAM_KO;
    CandMergeArgs m{};
    m.cand = ws.scand.as<uint2>();
    m.cand_n = ws.scn.as<int32_t>();
    m.cand_f = ws.scf.as<uint32_t>();
    m.thr = ws.sthr.as<float>();
    m.nq = nq;
    m.cap = cap;
    if (!deep) {
      PhaseTimer t(PH_MERGE, ws.st);
      ws.ms.ensure(sizeof(float) * nq * STREAM_KO);
      ws.mk.ensure(sizeof(int32_t) * nq * STREAM_KO);
      m.out_s = ws.ms.as<float>();
      m.out_k = ws.mk.as<int32_t>();
      launch_cand_merge(m, ws.st);
    }
    ws.fail.ensure(sizeof(int32_t) * nq);
    ws.fail2.ensure(sizeof(int32_t) * nq);
    ws.fail_cnt.ensure(sizeof(int32_t));
    ws.fail_cnt2.ensure(sizeof(int32_t));
    PqRefineArgs r{};
    r.queries = d_q;
    r.cents = coarse.rm.as<float>();
    r.codebooks = cb.as<float>();
    r.cpack = cpack.as<uint8_t>();
    r.labels = clabels.as<int64_t>();
    r.lb = dlb.as<int32_t>();
    r.ms = ws.ms.as<float>();
    r.mk = ws.mk.as<int32_t>();
    r.nq = nq;
    r.ld = STREAM_KO;
    r.k = k;
    r.dim = dim;
    r.M = M;
    r.ksub = ksub;
    r.lw = pq32_lane_words(dim, M);
    r.dsub = sub;
    r.nlist = coarse.nlist;
    r.out_s = d_s;
    r.out_l = d_l;
    r.out_c = d_c;
    int32_t nf = 0;
    if (deep) {  // depth K1 over the emitted rows, the failures again at 2 K1 (<= 512); what fails re-runs on the LUT scan
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      const int k2 = std::min(2 * k1, 512);
      r.k1 = k1;
      r.fail_list = k2 > k1 ? ws.fail2.as<int32_t>() : ws.fail.as<int32_t>();
      r.fail_cnt = k2 > k1 ? ws.fail_cnt2.as<int32_t>() : ws.fail_cnt.as<int32_t>();
      launch_pq32_deep_refine(m, r, ws.st);
      if (k2 > k1) {
        r.k1 = k2;
        r.qsel = ws.fail2.as<int32_t>();
        r.nsel = ws.fail_cnt2.as<int32_t>();
        r.fail_list = ws.fail.as<int32_t>();
        r.fail_cnt = ws.fail_cnt.as<int32_t>();
        launch_pq32_deep_refine(m, r, ws.st);
      }
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
    } else {
      PhaseTimer t(PH_REFINE, ws.st, nq * k1);
      r.k1 = k1;
      r.fail_list = ws.fail2.as<int32_t>();
      r.fail_cnt = ws.fail_cnt2.as<int32_t>();
      launch_pq32_refine(r, nq, ws.st);
      r.k1 = STREAM_KO;  // the failures again at depth 64, from the same candidates
      r.qsel = ws.fail2.as<int32_t>();
      r.nsel = ws.fail_cnt2.as<int32_t>();
      r.fail_list = ws.fail.as<int32_t>();
      r.fail_cnt = ws.fail_cnt.as<int32_t>();
      launch_pq32_refine(r, nq, ws.st);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(&nf, ws.fail_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, ws.st));
      HIPCHK(hipStreamSynchronize(ws.st));
    }
    if (knob("PYR_STREAM_DEBUG")) {
      int32_t n1 = 0;
      HIPCHK(hipMemcpy(&n1, ws.fail_cnt2.p, sizeof(int32_t), hipMemcpyDeviceToHost));
      fprintf(stderr, "[pq32] nq %lld: certificate failures depth %d %d, depth %d %d\n", (long long)nq, k1, n1,
              deep ? std::min(2 * k1, 512) : STREAM_KO, nf);
    }
    // what neither depth certifies: the LUT scan of those queries over the same probe lists (the slice's
    // ranking or the caller's, gathered by the fail list), same arithmetic
    filter_fallback(ws, nf, d_q, dim, k, d_s, d_l, d_c,
                    [&](const float *q2, int64_t n2, float *s2, int64_t *l2, int32_t *c2) {
                      ws.fprobes.ensure(sizeof(int32_t) * n2 * probes);
                      launch_gather_words(ws.probes.as<uint32_t>(), ws.fail.as<int32_t>(), n2, probes,
                                          ws.fprobes.as<uint32_t>(), ws.st);
                      Workspace &nw = ws.nested();
                      nw.ext_probes = ws.fprobes.as<int32_t>();
                      nw.ext_nprobe = probes;
                      nw.skip_buffer = true;  // the lists only: a non-empty buffer is merged by search()
                      try {
                        search_lut(q2, n2, k, probes, s2, l2, c2, nw);
                      } catch (...) {
                        nw.ext_probes = nullptr;
                        nw.skip_buffer = false;
                        throw;
                      }
                      nw.ext_probes = nullptr;
                      nw.skip_buffer = false;
                    });
  }

  // the reference's per-row LUT sum on the LDS (pq_adc4 / pq_scan)
  void search_lut(const float *d_q, int64_t nq, int k, int probes, float *d_s, int64_t *d_l, int32_t *d_c,
                  Workspace &ws) {
    const int64_t bcut = buf.st.n;
    // list-scan kernel: pq_adc4 (4 queries per LDS gather; lists split into PQ4_ROWS-row chunks), else
    // the first-cut pq_scan; PYR_PQ_ADC=0 forces the latter (A/B only)
    const int mode = pq_adc_mode();
    IvfChunking ch{1 << 30, 1, 0};
    int kern = 0;
    if (mode >= 2 && pq_adc4_supported(dim, M, ksub, k)) {
      ch.chunk = pq_adc4_rows();
      int32_t mx = 0;
      for (int32_t v : llen) mx = std::max(mx, v);
      ch.cmax = ivf_list_chunks(mx, ch);
      if ((int64_t)probes * ch.cmax < MAX_PARTS) kern = 2;
      else ch = IvfChunking{1 << 30, 1, 0};
    }
    const int lparts = probes * ch.cmax;
    ScanPlan bp;
    if (buf.live_count() > 0 && !ws.skip_buffer) bp = plan_flat(bcut, nq, dim, k, MAX_PARTS - lparts);
    const int nparts = lparts + bp.nchunks;
    if (nparts > MAX_PARTS) throw Error(PYR_E_ARG, "nprobe too large");
    if (nparts == 0) {
      fill_empty_results(d_s, d_l, d_c, nq, k, ws.st);
      return;
    }
    prep_queries(d_q, nq, dim, metric, ws);
    const float *qn = metric == COS ? ws.qn.as<float>() : nullptr;
    const size_t np = (size_t)nq * nparts * k;
    ws.part_s.ensure(sizeof(float) * np);
    ws.part_k.ensure(sizeof(uint32_t) * np);
    if (probes > 0) {
      {
        PhaseTimer t(PH_COARSE, ws.st, nq * coarse.nlist);
        coarse.probe(d_q, qn, nq, probes, metric, ws);
      }
      const int qchunk = 32;
      const int maxi = build_ivf_items(ws, nq, probes, nparts, coarse.nlist, dlb, dle, qchunk, ch);
      PqArgs a{};
      a.codes = codes.as<uint8_t>();
      a.live = clive.as<uint8_t>();
      a.queries = d_q;
      a.cents = coarse.rm.as<float>();
      a.codebooks = cb.as<float>();
      a.probes = ws.probes.as<int32_t>();
      a.list_begin = dlb.as<int32_t>();
      a.list_end = dle.as<int32_t>();
      a.items = ws.items.as<ScanItem>();
      a.n_items = ws.nitems.as<int32_t>();
      a.qlist = ws.qlist.as<int32_t>();
      a.nparts = nparts;
      a.nprobe = probes;
      a.k = k;
      a.dim = dim;
      a.M = M;
      a.ksub = ksub;
      a.part_s = ws.part_s.as<float>();
      a.part_k = ws.part_k.as<uint32_t>();
      a.gthr = kern > 0 && bounds_enabled() ? shared_bounds(ws, nq) : nullptr;
      if (const char *e = knob("PYR_PQ_ABLATE")) a.ablate = atoi(e);  // measurement only
      if (kern == 0 && pq_scan_lds_bytes(dim, M, ksub, k) > 160 * 1024)
        throw Error(PYR_E_ARG, "PQ lookup table exceeds LDS");
      PhaseTimer t(PH_PQ_SCAN, ws.st, prof().on ? probed_rows(ws, nq, probes, le, lb) : 0);
      if (kern == 2) launch_pq_adc4(a, maxi, ws.st);
      else launch_pq_scan(a, maxi, ws.st);
    }
    if (bp.nchunks > 0) {  // :130-136 exact buffer scan
      PhaseTimer t(PH_BUF_SCAN, ws.st, nq * bcut);
      flat_scan(buf.st, bcut, bp, d_q, qn, nq, k, 1, metric, nparts, lparts, KEY_BUF, ws, ws.part_s.as<float>(),
                ws.part_k.as<uint32_t>(), true);
    }
    PhaseTimer tm(PH_MERGE, ws.st);
    MergeIvf mi;  // chunk slots p * cmax + c exist only for the chunks a probed list has
    mi.probes = ws.probes.as<int32_t>();
    mi.lb = dlb.as<int32_t>();
    mi.le = dle.as<int32_t>();
    mi.nprobe = probes;
    mi.ch = ch;
    launch_merge_keys(ws.part_s.as<float>(), ws.part_k.as<uint32_t>(), nq, nparts, k, clabels.as<int64_t>(),
                      buf.st.labels.as<int64_t>(), d_s, d_l, nullptr, d_c, ws.st, ch.cmax > 1 ? &mi : nullptr);
  }

  int64_t count() const override { return 0; }  // :230 GetStats quirk
  void all_labels(std::vector<int64_t> &out) const override {
    buf.all_labels(out);
    for (int64_t lab : hlabels)
      if (lab >= 0) out.push_back(lab);
  }

  // The reference's IvfPq Snapshot / Load are no-ops (:228-229); the image persists the trained
  // state (quantizer, codebooks, codes in list order) and the buffer like IVF_FLAT's.
  void snapshot(const std::string &path) override {
    ImageWriter w(path, PYR_IVF_PQ, dim, metric);
    const uint8_t b = built ? 1 : 0;
    w.host(T_BUILT, &b, 1);
    if (built) {
      w.host(T_CENTS, coarse.host.data(), sizeof(float) * coarse.host.size());
      const int32_t ks = ksub;
      w.host(T_KSUB, &ks, sizeof(ks));
      w.device(T_CODEBOOKS, cb.p, sizeof(float) * (size_t)M * ksub * sub, wst);
      w.host(T_LCOUNT, llen.data(), sizeof(int32_t) * llen.size());
      std::vector<int64_t> labels;
      for (int l = 0; l < coarse.nlist; l++)
        for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++) labels.push_back(hlabels[p]);
      w.host(T_LLABELS, labels.data(), sizeof(int64_t) * labels.size());
      std::vector<uint8_t> codes_rm(labels.size() * (size_t)M);
      pq_state(nullptr, nullptr, codes_rm.data());  // list-major rows of M codes
      w.host(T_LCODES, codes_rm.data(), codes_rm.size());
    }
    std::vector<int64_t> blabels;
    const std::vector<int64_t> bslots = live_slots(buf.st, blabels);
    write_rows(w, T_BLABELS, T_BROWS, buf.st, bslots, blabels, stage_x, stage_i, wst);
    w.commit();
  }

  void load(const std::string &path) override {
    ImageReader r(path);
    check_image(r, PYR_IVF_PQ, *this);
    buf.clear(wst);
    built = false;
    hlabels.clear();
    hlive.clear();
    pos_of.clear();
    lb.clear();
    le.clear();
    llen.clear();
    ncode_rows = 0;
    uint8_t b = 0;
    if (r.has(T_BUILT)) r.host(T_BUILT, &b, 1);
    const std::vector<float> cents = r.vec<float>(T_CENTS);
    if (cents.size() % (size_t)dim != 0) ImageReader::throw_format("centroids are not whole rows");
    const int k = (int)(cents.size() / dim);
    if (b && k > 0) {
      int32_t ks = 0;
      r.host(T_KSUB, &ks, sizeof(ks));
      if (ks <= 0 || ks > K) ImageReader::throw_format("codebook size out of range");
      ksub = ks;
      cb.ensure(sizeof(float) * (size_t)M * ksub * sub);
      r.device(T_CODEBOOKS, cb.p, sizeof(float) * (size_t)M * ksub * sub, wst);
      const std::vector<int32_t> cnt = r.vec<int32_t>(T_LCOUNT);
      if ((int)cnt.size() != k) ImageReader::throw_format("list counts do not match the centroids");
      const std::vector<int64_t> labels = r.vec<int64_t>(T_LLABELS);
      std::vector<int32_t> asg;
      for (int l = 0; l < k; l++) asg.insert(asg.end(), (size_t)cnt[l], l);
      if (asg.size() != labels.size()) ImageReader::throw_format("list counts do not match the labels");
      const int64_t n = (int64_t)labels.size();
      DevMem codes_rm, C;
      codes_rm.ensure((size_t)std::max<int64_t>(n, 1) * M);
      if (n) r.device(T_LCODES, codes_rm.p, (size_t)n * M, wst);
      C.ensure(sizeof(float) * k * dim);
      HIPCHK(hipMemcpyAsync(C.p, cents.data(), sizeof(float) * k * dim, hipMemcpyHostToDevice, wst));
      commit_codes(codes_rm.as<uint8_t>(), n, asg, labels, C.as<float>(), k);
      built = true;
    }
    std::vector<int64_t> blabels;
    std::vector<float> brows;
    const int64_t nb = read_rows(r, T_BLABELS, T_BROWS, dim, blabels, brows);
    if (nb) add(brows.data(), nb, blabels.data(), true);  // buffer ids hide their list entries (:134,170)
  }

  void ivf_layout(int64_t *off, int64_t *labels, uint8_t *live, int64_t *total) const override {
    int64_t t = 0;
    for (int l = 0; l < coarse.nlist && built; l++) {
      if (off) off[l] = t;
      for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++, t++) {
        if (labels) labels[t] = hlabels[p];
        if (live) live[t] = hlive[p];
      }
    }
    if (off && built) off[coarse.nlist] = t;
    *total = t;
  }

  void pq_state(float *out_cb, int32_t *out_ksub, uint8_t *out_codes) const override {
    if (out_ksub) *out_ksub = built ? ksub : 0;
    if (!built) return;
    if (out_cb) HIPCHK(hipMemcpy(out_cb, cb.p, sizeof(float) * (size_t)M * ksub * sub, hipMemcpyDeviceToHost));
    if (out_codes) {
      const int nch = (M + 15) / 16;
      std::vector<uint8_t> blk((size_t)ncode_rows * nch * 16);
      HIPCHK(hipMemcpy(blk.data(), codes.p, blk.size(), hipMemcpyDeviceToHost));
      int64_t t = 0;
      for (int l = 0; l < coarse.nlist; l++)
        for (int32_t p = lb[l]; p < lb[l] + llen[l]; p++, t++)
          for (int m = 0; m < M; m++)
            out_codes[t * M + m] = blk[(((size_t)(p >> 6) * nch + (m >> 4)) * 64 + (p & 63)) * 16 + (m & 15)];
    }
  }

  void centroids(float *out, int32_t *nl) const override {
    *nl = built ? coarse.nlist : 0;
    if (out && built) std::memcpy(out, coarse.host.data(), sizeof(float) * coarse.host.size());
  }
};

Index *create_index(const pyr_index_desc &d) {
  if (d.dim <= 0) throw Error(PYR_E_ARG, "Dimension must be positive.");  // BruteForceVectorIndex.cs:43-46
  if (d.metric < 0 || d.metric > 2) throw Error(PYR_E_ARG, "unknown metric");
  if (d.device_mask != 0) return create_multi_index(d);  // (pyr_index_create clears a one-GPU mask)
  switch (d.kind) {
    case PYR_FLAT: return new FlatIndex(d);
    case PYR_IVF_FLAT: return new IvfFlatIndex(d);
    case PYR_IVF_PQ: return new IvfPqIndex(d);
    default: throw Error(PYR_E_ARG, "unknown index kind");
  }
}

}  // namespace pyr
