// capi.cpp -- the extern "C" boundary of libpyrope_hip.so (include/pyrope_ann.h).
// No C++ exception crosses it: every entry point catches, records a thread-local
// message (pyr_last_error) and returns a pyr_status.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <tuple>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "persist.h"

namespace {
// Request coalescer (pyr_index_set_coalescing).  The reference serves one query per VEC.SEARCH
// call (VectorCommandSet.cs:457-459), one call per Garnet session thread; the scan reaches its
// throughput only on batches.  Concurrent pyr_index_search calls with the same (k, SearchOptions)
// join an open batch.  The first caller (the leader) dispatches it as soon as fewer than
// max_inflight (1) coalesced searches of this index are in flight (an idle device never waits: a lone
// caller pays no added latency), else when a running search finishes, when the batch holds max_batch queries,
// or at the latest max_wait_us after it opened; it runs ONE device search for all of them and
// copies every caller's rows into that caller's buffers.  The other callers (followers) block until
// then.  Each query's result is the same as a search of it alone (the engine is per query exact).
struct Batch {
  int32_t k = 0;
  pyr_search_params prm{};
  std::vector<float> q;  // queries in arrival order
  struct Part {
    int64_t off, n;
    float *s;
    int64_t *l;
    int32_t *c;
  };
  std::vector<Part> parts;
  int64_t nq = 0;
  bool closed = false, done = false;
  pyr_status status = PYR_OK;
  std::string err;
  std::chrono::steady_clock::time_point deadline;
};
struct Coalescer {
  std::mutex m;
  std::condition_variable cv;
  int32_t max_batch = 0, max_wait_us = 0;
  int32_t inflight = 0;  // coalesced device searches running
  // batches that may run at once (each on its own stream and workspace).  PYR_COALESCE_INFLIGHT
  // (measurement knob), default 1: two in flight measured no better (profiles/r3_serve/serve_if*.log)
  int32_t max_inflight = [] {
    const char *e = std::getenv("PYR_COALESCE_INFLIGHT");
    return e ? std::max(1, std::atoi(e)) : 1;
  }();
  std::map<std::tuple<int32_t, int32_t, int64_t>, std::shared_ptr<Batch>> open;  // (k, nprobe, max_scans)
};
}  // namespace

struct pyr_index {
  std::unique_ptr<pyr::Index> impl;
  Coalescer co;
};

namespace {
thread_local std::string g_err;

pyr_status fail(pyr_status s, const std::string &m) {
  g_err = m;
  return s;
}

template <class F>
pyr_status guard(F &&f) {
  try {
    f();
    return PYR_OK;
  } catch (const pyr::Error &e) {
    return fail(e.status, e.what());
  } catch (const std::bad_alloc &) {
    return fail(PYR_E_OOM, "host allocation failed");
  } catch (const std::exception &e) {
    return fail(PYR_E_ARG, e.what());
  }
}

void check_device(int dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw pyr::Error(PYR_E_DEVICE, "no HIP device available");
  if (dev < 0 || dev >= n) throw pyr::Error(PYR_E_DEVICE, "device ordinal out of range");
  hipDeviceProp_t p;
  HIPCHK(hipGetDeviceProperties(&p, dev));
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    throw pyr::Error(PYR_E_DEVICE, std::string("libpyrope_hip is built for gfx950, device is ") + p.gcnArchName);
}

pyr_search_params defaults(const pyr_search_params *p) {
  pyr_search_params d{-1, 0, -1};
  return p ? *p : d;
}
}  // namespace

extern "C" {

pyr_status pyr_index_create(const pyr_index_desc *desc, pyr_index **out) {
  if (!desc || !out) return fail(PYR_E_ARG, "null argument");
  *out = nullptr;
  return guard([&] {
    pyr_index_desc d = *desc;
    if (d.shards < 0) throw pyr::Error(PYR_E_ARG, "shards must be >= 0");
    if (d.device_mask != 0) {
      for (int b = 0; b < 64; ++b)
        if (d.device_mask >> b & 1) check_device(b);
      d.device = __builtin_ctzll(d.device_mask);  // the first device: the multi-GPU index's stage
      if (__builtin_popcountll(d.device_mask) == 1 && d.shards == 0) d.device_mask = 0;  // one GPU: the plain index
    } else {
      check_device(d.device);
      if (d.shards > 0) d.device_mask = 1ull << d.device;
    }
    if (d.device_mask == 0) d.shards = 0;
    auto *h = new pyr_index;
    try {
      h->impl.reset(pyr::create_index(d));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

void pyr_index_destroy(pyr_index *index) {
  if (!index) return;
  try {
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    g.unlock();
    delete index;
  } catch (...) {
  }
}

static pyr_status write_op(pyr_index *index, const float *x, int64_t n, const int64_t *labels, bool upsert) {
  if (!index || (n > 0 && (!x || !labels)) || n < 0) return fail(PYR_E_ARG, "null argument");
  for (int64_t i = 0; i < n; i++)
    if (labels[i] < 0) return fail(PYR_E_ARG, "Id cannot be empty.");  // ValidateId
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    const bool prof = pyr::wprof_on();
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](int sec) {
      if (!prof) return;
      const auto t1 = std::chrono::steady_clock::now();
      pyr::wprof_add(sec, std::chrono::duration<double>(t1 - t0).count());
      t0 = t1;
    };
    if (n > 0) index->impl->add(x, n, labels, upsert);
    lap(5);
    index->impl->after_write();
    lap(6);
    index->impl->note_write();
    lap(7);
    pyr::note_write_call();
  });
}

pyr_status pyr_index_add(pyr_index *index, const float *x, int64_t n, const int64_t *labels) {
  return write_op(index, x, n, labels, false);
}

pyr_status pyr_index_upsert(pyr_index *index, const float *x, int64_t n, const int64_t *labels) {
  return write_op(index, x, n, labels, true);
}

pyr_status pyr_index_remove(pyr_index *index, const int64_t *labels, int64_t n, uint8_t *removed) {
  if (!index || (n > 0 && !labels) || n < 0) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->remove(labels, n, removed);
  });
}

pyr_status pyr_index_build(pyr_index *index) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->build();
  });
}

pyr_status pyr_index_set_centroids(pyr_index *index, const float *centroids, int32_t nlist) {
  if (!index || !centroids) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->set_centroids(centroids, nlist);
  });
}

pyr_status pyr_index_set_codebooks(pyr_index *index, const float *codebooks, int32_t m, int32_t ksub) {
  if (!index || !codebooks) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->set_codebooks(codebooks, m, ksub);
  });
}

pyr_status pyr_index_reserve(pyr_index *index, int64_t rows) {
  if (!index || rows < 0) return fail(PYR_E_ARG, "bad argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->reserve(rows);
  });
}

pyr_status pyr_kmeans_train(int32_t device, const float *data, int64_t n, int32_t dim, int32_t k, int32_t metric,
                            int32_t max_iter, int32_t seed, float *out, int32_t *k_out) {
  if (!data || !out || n < 0 || dim <= 0) return fail(PYR_E_ARG, "bad argument");
  return guard([&] {
    check_device(device);
    HIPCHK(hipSetDevice(device));
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    try {
      pyr::DevMem X, C;
      X.ensure(sizeof(float) * (size_t)std::max<int64_t>(n, 1) * dim);
      const int kk = (int)std::max<int64_t>(1, std::min<int64_t>(k <= 0 ? 1 : k, std::max<int64_t>(n, 1)));
      C.ensure(sizeof(float) * (size_t)kk * dim);
      HIPCHK(hipMemcpyAsync(X.p, data, sizeof(float) * n * dim, hipMemcpyHostToDevice, st));
      const int used = pyr::kmeans_train_gpu(X.as<float>(), n, dim, k, metric, max_iter, seed, C.as<float>(), st);
      if (used > 0) HIPCHK(hipMemcpyAsync(out, C.p, sizeof(float) * (size_t)used * dim, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (k_out) *k_out = used;
    } catch (...) {
      (void)hipStreamDestroy(st);
      throw;
    }
    (void)hipStreamDestroy(st);
  });
}

pyr_status pyr_assign(int32_t device, const float *centroids, int32_t nlist, const float *x, int64_t n, int32_t dim,
                      int32_t metric, int32_t *assign) {
  if (!centroids || (n > 0 && (!x || !assign)) || n < 0 || dim <= 0 || nlist <= 0) return fail(PYR_E_ARG, "bad argument");
  return guard([&] {
    check_device(device);
    HIPCHK(hipSetDevice(device));
    if (n == 0) return;
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    try {
      pyr::DevMem X, C, A;
      X.ensure(sizeof(float) * (size_t)n * dim);
      C.ensure(sizeof(float) * (size_t)nlist * dim);
      A.ensure(sizeof(int32_t) * (size_t)n);
      HIPCHK(hipMemcpyAsync(X.p, x, sizeof(float) * n * dim, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(C.p, centroids, sizeof(float) * (size_t)nlist * dim, hipMemcpyHostToDevice, st));
      pyr::assign_gpu(X.as<float>(), n, dim, C.as<float>(), nlist, metric, A.as<int32_t>(), st);
      HIPCHK(hipMemcpyAsync(assign, A.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    } catch (...) {
      (void)hipStreamDestroy(st);
      throw;
    }
    (void)hipStreamDestroy(st);
  });
}

void pyr_profile_enable(int32_t on) {
  std::lock_guard<std::mutex> g(pyr::prof().m);
  pyr::prof().on = on != 0;
}

void pyr_profile_reset(void) {
  std::lock_guard<std::mutex> g(pyr::prof().m);
  pyr::prof().reset();
}

pyr_status pyr_profile_get(int32_t phase, double *total_ms, int64_t *calls, int64_t *work) {
  if (phase < 0 || phase >= pyr::PH_N) return fail(PYR_E_ARG, "bad phase");
  std::lock_guard<std::mutex> g(pyr::prof().m);
  pyr::prof().drain();
  if (total_ms) *total_ms = pyr::prof().ms[phase];
  if (calls) *calls = pyr::prof().calls[phase];
  if (work) *work = pyr::prof().work[phase];
  return PYR_OK;
}

pyr_status pyr_index_debug_candidates(pyr_index *index, int64_t nq, int32_t cap, float *h_ub, int64_t *h_label,
                                      int32_t *h_cnt) {
  if (!index || nq < 0 || cap <= 0 || (nq > 0 && (!h_ub || !h_label || !h_cnt))) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    ix.debug_candidates(nq, cap, h_ub, h_label, h_cnt);
  });
}

static pyr_status search_host(pyr_index *index, const float *q, int64_t nq, int32_t k, const pyr_search_params *params,
                              float *out_scores, int64_t *out_labels, int32_t *out_counts) {
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    auto ws = ix.take_ws();
    try {
      const int kk = k > 0 ? k : 0;
      const size_t qb = sizeof(float) * (size_t)nq * ix.dim;
      ws->q.ensure(qb);
      ws->out_s.ensure(sizeof(float) * (size_t)nq * kk);
      ws->out_l.ensure(sizeof(int64_t) * (size_t)nq * kk);
      ws->out_c.ensure(sizeof(int32_t) * (size_t)nq);
      if (nq > 0) HIPCHK(hipMemcpyAsync(ws->q.p, q, qb, hipMemcpyHostToDevice, ws->st));
      ix.search(ws->q.as<float>(), nq, k, defaults(params), ws->out_s.as<float>(), ws->out_l.as<int64_t>(),
                ws->out_c.as<int32_t>(), *ws);
      HIPCHK(hipGetLastError());
      if (nq > 0 && kk > 0) {
        if (out_scores)
          HIPCHK(hipMemcpyAsync(out_scores, ws->out_s.p, sizeof(float) * nq * kk, hipMemcpyDeviceToHost, ws->st));
        if (out_labels)
          HIPCHK(hipMemcpyAsync(out_labels, ws->out_l.p, sizeof(int64_t) * nq * kk, hipMemcpyDeviceToHost, ws->st));
      }
      if (out_counts && nq > 0)
        HIPCHK(hipMemcpyAsync(out_counts, ws->out_c.p, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ws->st));
      HIPCHK(hipStreamSynchronize(ws->st));
    } catch (...) {
      (void)hipStreamSynchronize(ws->st);
      ix.give_ws(std::move(ws));
      throw;
    }
    ix.give_ws(std::move(ws));
  });
}

static pyr_status search_coalesced(pyr_index *index, const float *q, int64_t nq, int32_t k,
                                   const pyr_search_params &prm, float *out_scores, int64_t *out_labels,
                                   int32_t *out_counts) {
  Coalescer &co = index->co;
  const int dim = index->impl->dim;
  std::unique_lock<std::mutex> lk(co.m);
  const auto key = std::make_tuple(k, prm.nprobe, prm.max_scans);
  std::shared_ptr<Batch> b;
  bool leader = false;
  size_t q0 = 0;  // b->q's size before this caller's rows
  try {  // no allocation failure may cross the C ABI or leave followers waiting
    auto it = co.open.find(key);
    if (it == co.open.end() || it->second->closed || it->second->nq + nq > co.max_batch) {
      b = std::make_shared<Batch>();
      b->k = k;
      b->prm = prm;
      b->deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(co.max_wait_us);
      co.open[key] = b;
      leader = true;
    } else {
      b = it->second;
    }
    q0 = b->q.size();
    b->q.insert(b->q.end(), q, q + nq * dim);
    b->parts.push_back({b->nq, nq, out_scores, out_labels, out_counts});
  } catch (...) {
    // leader or follower: the batch keeps exactly the rows of the callers in b->parts
    if (b && b->q.size() > q0) b->q.resize(q0);
    if (leader) {  // nobody else joined yet (the lock is held): withdraw the batch
      auto f = co.open.find(key);
      if (f != co.open.end() && f->second == b) co.open.erase(f);
    }
    return fail(PYR_E_OOM, "coalescer: host allocation failed");
  }
  b->nq += nq;
  if (b->nq >= co.max_batch) {  // full: the leader runs it now
    b->closed = true;
    if (co.open[key] == b) co.open.erase(key);
    co.cv.notify_all();
  }
  if (!leader) {
    co.cv.wait(lk, [&] { return b->done; });
    if (b->status != PYR_OK) return fail(b->status, b->err);
    return PYR_OK;
  }
  // dispatch when full, when no coalesced search is running (an idle device starts at once; a busy
  // one gathers every caller that arrives while it works), or at the deadline
  co.cv.wait_until(lk, b->deadline, [&] { return b->closed || co.inflight < co.max_inflight; });
  if (!b->closed) {
    b->closed = true;
    auto f = co.open.find(key);
    if (f != co.open.end() && f->second == b) co.open.erase(f);
  }
  ++co.inflight;
  lk.unlock();
  // one device search for the whole batch, then every caller's rows into its own buffers
  pyr_status st = PYR_OK;
  std::string err;
  try {
    const int kk = k > 0 ? k : 0;
    std::vector<float> s((size_t)b->nq * kk);
    std::vector<int64_t> l((size_t)b->nq * kk);
    std::vector<int32_t> c((size_t)b->nq);
    st = search_host(index, b->q.data(), b->nq, k, &b->prm, s.data(), l.data(), c.data());
    if (st == PYR_OK)
      for (const Batch::Part &p : b->parts) {
        if (p.s) std::memcpy(p.s, s.data() + p.off * kk, sizeof(float) * p.n * kk);
        if (p.l) std::memcpy(p.l, l.data() + p.off * kk, sizeof(int64_t) * p.n * kk);
        if (p.c) std::memcpy(p.c, c.data() + p.off, sizeof(int32_t) * p.n);
      }
    else
      err = pyr_last_error();
  } catch (...) {
    st = PYR_E_OOM;
    err = "coalescer: host allocation failed";
  }
  lk.lock();
  --co.inflight;
  b->status = st;
  b->err = err;
  b->done = true;
  co.cv.notify_all();
  lk.unlock();
  return st == PYR_OK ? PYR_OK : fail(st, err);
}

pyr_status pyr_index_search(pyr_index *index, const float *q, int64_t nq, int32_t k, const pyr_search_params *params,
                            float *out_scores, int64_t *out_labels, int32_t *out_counts) {
  if (!index || nq < 0 || (nq > 0 && !q)) return fail(PYR_E_ARG, "null argument");
  if (k > pyr::KMAX) return fail(PYR_E_ARG, "topK larger than 256 is not supported");
  int32_t mb, mw;
  {
    std::lock_guard<std::mutex> g(index->co.m);
    mb = index->co.max_batch;
    mw = index->co.max_wait_us;
  }
  if (mw > 0 && nq > 0 && k > 0 && nq < mb)
    return search_coalesced(index, q, nq, k, defaults(params), out_scores, out_labels, out_counts);
  return search_host(index, q, nq, k, params, out_scores, out_labels, out_counts);
}

pyr_status pyr_index_set_coalescing(pyr_index *index, int32_t max_batch, int32_t max_wait_us) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  if (max_wait_us > 0 && max_batch < 2) return fail(PYR_E_ARG, "max_batch must be at least 2");
  std::lock_guard<std::mutex> g(index->co.m);
  index->co.max_batch = max_batch;
  index->co.max_wait_us = max_wait_us > 0 ? max_wait_us : 0;
  return PYR_OK;
}

pyr_status pyr_index_search_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                   const pyr_search_params *params, float *d_scores, int64_t *d_labels,
                                   int32_t *d_counts, void *stream) {
  if (!index || nq < 0 || (nq > 0 && !d_q)) return fail(PYR_E_ARG, "null argument");
  if (k > pyr::KMAX) return fail(PYR_E_ARG, "topK larger than 256 is not supported");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    ix.search(d_q, nq, k, defaults(params), d_scores, d_labels, d_counts, ws);
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_probe_device(pyr_index *index, const float *d_q, int64_t nq, int32_t nprobe, int32_t *d_probes,
                                  int32_t *probes_out, void *stream) {
  if (!index || nq < 0 || (nq > 0 && (!d_q || !d_probes))) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    const int p = ix.probe_only(d_q, nq, nprobe, d_probes, ws);
    if (probes_out) *probes_out = p;
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_search_probed_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                          const pyr_search_params *params, const int32_t *d_probes, int32_t nprobe,
                                          float *d_scores, int64_t *d_labels, int32_t *d_counts, void *stream) {
  if (!index || nq < 0 || (nq > 0 && (!d_q || !d_probes))) return fail(PYR_E_ARG, "null argument");
  if (k > pyr::KMAX) return fail(PYR_E_ARG, "topK larger than 256 is not supported");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    ws.ext_probes = d_probes;
    ws.ext_nprobe = nprobe;
    try {
      ix.search(d_q, nq, k, defaults(params), d_scores, d_labels, d_counts, ws);
    } catch (...) {
      ws.ext_probes = nullptr;
      throw;
    }
    ws.ext_probes = nullptr;
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_snapshot(pyr_index *index, const char *path) {
  if (!index || !path) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    // the reference snapshots under its read lock; the image reuses the write stream and
    // staging buffers, so snapshots serialize among themselves (wmu) but not with searches
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    std::lock_guard<std::mutex> w(index->impl->wmu);
    HIPCHK(hipStreamSynchronize(index->impl->wst));  // writes the small-batch path left in flight
    index->impl->snapshot(path);
  });
}

pyr_status pyr_index_load(pyr_index *index, const char *path) {
  if (!index || !path) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->load(path);
  });
}

pyr_status pyr_image_nonce(const char *path, uint8_t *nonce) {
  if (!path || !nonce) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    pyr::ImageReader r(path);
    std::memset(nonce, 0, pyr::NONCE_BYTES);
    if (r.size(pyr::T_NONCE) == pyr::NONCE_BYTES) r.host(pyr::T_NONCE, nonce, pyr::NONCE_BYTES);
  });
}

pyr_status pyr_index_stats(const pyr_index *index, int64_t *count, int32_t *dim, int32_t *metric) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    if (count) *count = index->impl->count();
    if (dim) *dim = index->impl->dim;
    if (metric) *metric = index->impl->metric;
  });
}

pyr_status pyr_index_get_centroids(const pyr_index *index, float *out, int32_t *nlist) {
  if (!index || !nlist) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->centroids(out, nlist);
  });
}

pyr_status pyr_index_ivf_layout(const pyr_index *index, int64_t *list_off, int64_t *labels, uint8_t *live,
                                int64_t *total) {
  if (!index || !total) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->ivf_layout(list_off, labels, live, total);
  });
}

pyr_status pyr_index_pq_state(const pyr_index *index, float *codebooks, int32_t *ksub, uint8_t *codes) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    HIPCHK(hipStreamSynchronize(index->impl->wst));
    index->impl->pq_state(codebooks, ksub, codes);
  });
}

pyr_status pyr_index_labels(const pyr_index *index, int64_t *labels, int64_t *n) {
  if (!index || !n) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::shared_lock<std::shared_mutex> g(index->impl->mu);
    std::vector<int64_t> all;
    index->impl->all_labels(all);
    if (labels) {
      if (*n < (int64_t)all.size()) throw pyr::Error(PYR_E_ARG, "labels buffer too small");
      std::copy(all.begin(), all.end(), labels);
    }
    *n = (int64_t)all.size();
  });
}

pyr_status pyr_index_scan(pyr_index *index, int64_t *labels, float *x, int64_t *n) {
  if (!index || !n) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    HIPCHK(hipStreamSynchronize(index->impl->wst));  // writes the small-batch path left in flight
    index->impl->scan(labels, x, n);
  });
}

pyr_status pyr_index_set_quantization(pyr_index *index, int32_t enable) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->set_quantization(enable != 0);
  });
}

pyr_status pyr_scalar_quantize_minmax(int32_t device, const float *x, int64_t n, int32_t dim, uint8_t *codes,
                                      float *mins, float *maxs) {
  if (!x || !codes || n < 0 || dim <= 0) return fail(PYR_E_ARG, "bad arguments");
  return guard([&] {
    if (n == 0) return;
    check_device(device);
    HIPCHK(hipSetDevice(device));
    const int dp = pyr::sq8_dp(dim);
    pyr::DevMem dx, dc, ds, dm;
    dx.ensure(sizeof(float) * n * dim);
    dc.ensure((size_t)dp * n);
    ds.ensure(sizeof(int2) * n);
    dm.ensure(sizeof(float2) * n);
    HIPCHK(hipMemcpy(dx.p, x, sizeof(float) * n * dim, hipMemcpyHostToDevice));
    pyr::launch_sq8_quantize(dx.as<float>(), nullptr, 0, n, dim, dp, 0, dc.as<uint8_t>(), ds.as<int2>(), nullptr, nullptr,
                             dm.as<float2>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy2D(codes, dim, dc.p, dp, dim, n, hipMemcpyDeviceToHost));
    if (mins || maxs) {
      std::vector<float2> mm((size_t)n);
      HIPCHK(hipMemcpy(mm.data(), dm.p, sizeof(float2) * n, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < n; i++) {
        if (mins) mins[i] = mm[i].x;
        if (maxs) maxs[i] = mm[i].y;
      }
    }
  });
}

pyr_status pyr_scalar_quantize(int32_t device, const float *x, int64_t n, int32_t dim, uint8_t *codes) {
  return pyr_scalar_quantize_minmax(device, x, n, dim, codes, nullptr, nullptr);
}

pyr_status pyr_scalar_dequantize(int32_t device, const uint8_t *codes, int64_t n, int32_t dim, const float *mins,
                                 const float *maxs, float *out) {
  if (!codes || !mins || !maxs || !out || n < 0 || dim < 0) return fail(PYR_E_ARG, "bad arguments");
  return guard([&] {
    if (n == 0 || dim == 0) return;
    check_device(device);
    HIPCHK(hipSetDevice(device));
    pyr::DevMem dc, dmn, dmx, dout;
    dc.ensure((size_t)n * dim);
    dmn.ensure(sizeof(float) * n);
    dmx.ensure(sizeof(float) * n);
    dout.ensure(sizeof(float) * n * dim);
    HIPCHK(hipMemcpy(dc.p, codes, (size_t)n * dim, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dmn.p, mins, sizeof(float) * n, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dmx.p, maxs, sizeof(float) * n, hipMemcpyHostToDevice));
    pyr::launch_sq8_dequantize(dc.as<uint8_t>(), n, dim, dmn.as<float>(), dmx.as<float>(), dout.as<float>(), nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(out, dout.p, sizeof(float) * n * dim, hipMemcpyDeviceToHost));
  });
}

pyr_status pyr_merge_topk_device(const float *d_scores, const int64_t *d_labels, int64_t nq, int32_t nparts,
                                 int32_t k, float *d_out_scores, int64_t *d_out_labels, void *stream) {
  return pyr_merge_topk_parts_device(d_scores, d_labels, nq, nparts, k, 0, d_out_scores, d_out_labels, stream);
}

pyr_status pyr_merge_topk_parts_device(const float *d_scores, const int64_t *d_labels, int64_t nq, int32_t nparts,
                                       int32_t k, int32_t part_major, float *d_out_scores, int64_t *d_out_labels,
                                       void *stream) {
  if (nq < 0 || nparts <= 0 || nparts > pyr::MAX_PARTS || k <= 0 || k > pyr::KMAX)
    return fail(PYR_E_ARG, "bad merge shape");
  return guard([&] {
    pyr::launch_merge_labels(d_scores, d_labels, nq, nparts, k, d_out_scores, d_out_labels,
                             reinterpret_cast<hipStream_t>(stream), part_major != 0);
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_shard_info(const pyr_index *index, int32_t *shards, int32_t *xport, int64_t *sharded_searches,
                                int64_t *staged_searches, int64_t *last_max_failures, int64_t *last_extra_rounds) {
  if (!index) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    int32_t a = 0, b = 0;
    int64_t c = 0, d = 0, e = 0, f = 0;
    index->impl->shard_info(&a, &b, &c, &d, &e, &f);
    if (shards) *shards = a;
    if (xport) *xport = b;
    if (sharded_searches) *sharded_searches = c;
    if (staged_searches) *staged_searches = d;
    if (last_max_failures) *last_max_failures = e;
    if (last_extra_rounds) *last_extra_rounds = f;
  });
}

int64_t pyr_shard_record_bytes(int32_t k) { return k > 0 ? pyr::shard_record_bytes(k) : 0; }
int32_t pyr_shard_plan_stride(int32_t width, int64_t max_scans) {
  return width > 0 ? pyr::shard_plan_stride(width, max_scans >= 0) : 0;
}

pyr_status pyr_index_set_list_samples(pyr_index *index, const float *rows, const int64_t *counts,
                                      const int64_t *list_len, int32_t nlist) {
  if (!index || !counts || !list_len || nlist <= 0) return fail(PYR_E_ARG, "null argument");
  int64_t tot = 0;
  for (int32_t l = 0; l < nlist; ++l) tot += counts[l] > 0 ? counts[l] : 0;
  if (tot > 0 && !rows) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    HIPCHK(hipSetDevice(index->impl->device));
    std::unique_lock<std::shared_mutex> g(index->impl->mu);
    index->impl->set_list_samples(rows, counts, list_len, nlist);
  });
}

pyr_status pyr_index_shard_prepare_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                          const pyr_search_params *params, int32_t *d_plan, int32_t *width,
                                          void *stream) {
  if (!index || nq < 0 || (nq > 0 && (!d_q || !d_plan))) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    const int P = ix.shard_prepare(d_q, nq, k, defaults(params), d_plan, ws);
    if (width) *width = P;
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_shard_search_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                         const int32_t *d_plan, int32_t width, int32_t plan_budgets, void *d_records,
                                         void *stream) {
  if (!index || nq < 0 || (nq > 0 && (!d_q || !d_plan || !d_records))) return fail(PYR_E_ARG, "null argument");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    ix.shard_search(d_q, nq, k, d_plan, width, plan_budgets != 0, d_records, ws);
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_index_shard_rerun_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                        const int32_t *d_plan, int32_t width, int32_t plan_budgets,
                                        const int32_t *d_fails, int32_t nranks, int32_t fcap, int64_t nq_home,
                                        void *d_records, void *stream) {
  if (!index || nq < 0 || !d_plan || !d_fails || !d_records || nranks <= 0 || nranks > 64 || fcap <= 0)
    return fail(PYR_E_ARG, "bad argument");
  return guard([&] {
    pyr::Index &ix = *index->impl;
    HIPCHK(hipSetDevice(ix.device));
    std::shared_lock<std::shared_mutex> g(ix.mu);
    pyr::Workspace &ws = ix.ws_for_stream(reinterpret_cast<hipStream_t>(stream));
    std::lock_guard<std::mutex> wg(ws.m);
    ix.shard_rerun(d_q, nq, k, d_plan, width, plan_budgets != 0, d_fails, nranks, fcap, nq_home, d_records, ws);
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_shard_merge_device(const void *d_records, int32_t nparts, int64_t nrec, int32_t k,
                                  const int32_t *d_qsel, int32_t cap, float *d_scores, int64_t *d_labels,
                                  int32_t *d_counts, int32_t *d_fail, int32_t fcap, void *stream) {
  if (!d_records || nparts <= 0 || nparts > 64 || nrec < 0 || k <= 0 || k > 64 || !d_scores || !d_labels)
    return fail(PYR_E_ARG, "bad merge shape");
  if (d_qsel && cap <= 0) return fail(PYR_E_ARG, "bad merge shape");
  return guard([&] {
    pyr::ShardMergeArgs a{};
    a.rec = static_cast<const uint8_t *>(d_records);
    a.nparts = nparts;
    a.nrec = nrec;
    a.k = k;
    a.qsel = d_qsel;
    a.cap = cap;
    a.out_s = d_scores;
    a.out_l = d_labels;
    a.out_c = d_counts;
    a.fail = d_fail;
    a.fcap = fcap;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (d_fail) {  // the failure count restarts at 0 (a kernel, not a memset node: stream capture)
      pyr::WordFill z;
      z.add(d_fail, 1, 0);
      pyr::launch_fill_words(z, st);
    }
    pyr::launch_shard_merge(a, d_qsel ? std::min<int64_t>(cap, nrec) : nrec, st);
    HIPCHK(hipGetLastError());
  });
}

pyr_status pyr_ivf_memory_plan(int32_t dim, int64_t nrows, int32_t nlist, int64_t max_list_len, int64_t nq,
                               int32_t nprobe, int32_t k, int64_t *index_bytes, int64_t *workspace_bytes) {
  if (dim <= 0 || nrows < 0 || nlist <= 0 || max_list_len < 0 || nq < 0 || nprobe < 0 || k <= 0)
    return fail(PYR_E_ARG, "bad memory-plan shape");
  return guard([&] {
    pyr::ivf_memory_plan(dim, nrows, nlist, max_list_len, nq, nprobe, k, index_bytes, workspace_bytes);
  });
}

pyr_status pyr_generate_synthetic(int64_t count, int32_t dim, int32_t seed, float *out) {
  if (count < 0 || dim <= 0 || (count > 0 && !out)) return fail(PYR_E_ARG, "bad argument");
  pyr::NetRandom r(seed);  // Program.cs:251-263
  const int64_t n = count * (int64_t)dim;
  for (int64_t i = 0; i < n; i++) out[i] = (float)r.next_double();
  return PYR_OK;
}

pyr_status pyr_generate_synthetic_blocked(int64_t row0, int64_t count, int32_t dim, int32_t seed, int64_t block_rows,
                                          float *out) {
  if (row0 < 0 || count < 0 || dim <= 0 || block_rows <= 0 || (count > 0 && !out)) return fail(PYR_E_ARG, "bad argument");
  if (count == 0) return PYR_OK;
  // row r belongs to block b = r / block_rows, whose values are the sequence of new Random(seed + b)
  const int64_t b0 = row0 / block_rows, b1 = (row0 + count - 1) / block_rows;
  auto gen = [&](int64_t b) {
    pyr::NetRandom r((int32_t)(seed + b));
    const int64_t rb = std::max(row0, b * block_rows), re = std::min(row0 + count, (b + 1) * block_rows);
    for (int64_t i = (b * block_rows) * (int64_t)dim; i < rb * (int64_t)dim; i++) (void)r.next();  // skip to rb
    float *o = out + (rb - row0) * (int64_t)dim;
    for (int64_t i = 0; i < (re - rb) * (int64_t)dim; i++) o[i] = (float)r.next_double();
  };
  const int64_t nb = b1 - b0 + 1;
  const int nt = (int)std::min<int64_t>(nb, std::max(1u, std::min(32u, std::thread::hardware_concurrency())));
  std::atomic<int64_t> nextb{b0};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&] {
      for (int64_t b; (b = nextb.fetch_add(1)) <= b1;) gen(b);
    });
  for (auto &t : th) t.join();
  return PYR_OK;
}

const char *pyr_last_error(void) { return g_err.c_str(); }

const char *pyr_version(void) { return "pyrope_hip 0.1.0 gfx950"; }

}  // extern "C"
