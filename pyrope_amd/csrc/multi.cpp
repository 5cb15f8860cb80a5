// multi.cpp -- ONE IVF_FLAT index over several GPUs of one process (pyr_index_desc.device_mask / shards;
// SURVEY.md 8(b) "device_mask", 8(e)(i) "IVF lists shard naturally across the GPUs").
//
// The reference serves every VEC.SEARCH of an index from one process (Extensions/VectorCommandSet.cs:457-459)
// and the registry creates the index with one constructor call (Services/VectorIndexRegistry.cs:81-113), so a
// multi-GPU index has to be one pyr_index the C# shim can hold.  Design:
//
//  * the STAGE: an ordinary single-GPU IvfFlatIndex on the first device of the mask takes every write and
//    every Build, so Add / Upsert / Delete / Build / Snapshot / Load keep the reference semantics bit for bit
//    (IvfFlatVectorIndex.cs:39-145: the buffer, the k-means training over all unique rows, list order);
//  * the SHARDS: after each Build (or Load) the stage's lists are dealt WHOLE to `shards` IvfFlatIndex shards
//    (longest list first to the shard with the fewest rows -- dist.list_owners), every shard with the stage's
//    quantizer and the replicated sample of every list; a shard row's label is its stage storage position, so
//    the records' (score desc, list asc, label asc) order IS the unsharded index's storage tie order, and the
//    home maps positions back to the caller's labels at the end;
//  * a SEARCH (L2 / IP, k <= 60, empty buffer) runs the list-sharded step of dist.ListShardedIvf inside the
//    library, one stream per shard: the queries are broadcast, each shard plans its slice of the batch (coarse
//    ranking, T_q, MaxScans budgets), plans all_gather, every shard scans the pairs of the lists it owns ->
//    records, all_to_all to the homes, merge + certificate, fail lists all_gather, exact re-run, all_to_all,
//    merge; a home with more failures than one round carries gets further rounds (every rank reads the same
//    gathered counts).  Anything else (Cosine, k > 60, a non-empty buffer, an unbuilt index) is answered by
//    the stage on its GPU -- the same answers, on one device;
//  * the COLLECTIVES: RCCL (librccl.so.1, opened at the first multi-device search: ncclCommInitAll over the
//    shards' devices, grouped ncclAllGather / ncclAllToAll / ncclBroadcast on the shard streams) when every
//    shard has its own device; device copies (hipMemcpyPeerAsync, stream events on both sides) when shards
//    share a device -- the one-GPU test configuration.  PYR_SHARD_XPORT=copy|rccl forces one.
//
// Memory: the stage keeps every row on the first device (1,561 B per row at d = 128) beside
// that device's shard -- the price of bit-exact Build semantics without a host copy of the data.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <queue>

#include "engine.h"

namespace pyr {
namespace {

// ---- RCCL, opened on first use (no link-time dependency: a single-GPU host never loads it) ----
struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllToAll) all_to_all = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string why;
};

const Rccl &rccl() {
  static const Rccl r = [] {
    Rccl x;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);  // (torch's copy when torch loaded one: same soname)
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      x.why = std::string("librccl.so.1 not found: ") + dlerror();
      return x;
    }
    auto sym = [&](const char *n) { return dlsym(h, n); };
    x.init_all = reinterpret_cast<decltype(x.init_all)>(sym("ncclCommInitAll"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(sym("ncclCommDestroy"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(sym("ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(sym("ncclGroupEnd"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(sym("ncclAllGather"));
    x.all_to_all = reinterpret_cast<decltype(x.all_to_all)>(sym("ncclAllToAll"));
    x.broadcast = reinterpret_cast<decltype(x.broadcast)>(sym("ncclBroadcast"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(sym("ncclGetErrorString"));
    if (!x.init_all || !x.destroy || !x.group_start || !x.group_end || !x.all_gather || !x.all_to_all ||
        !x.broadcast || !x.error_string)
      x.why = "librccl.so.1 lacks a collective entry point";
    return x;
  }();
  return r;
}

#define NCCLCHK(x)                                                                                        \
  do {                                                                                                    \
    ncclResult_t r_ = (x);                                                                                \
    if (r_ != ncclSuccess) throw Error(PYR_E_DEVICE, std::string(#x " failed: ") + rccl().error_string(r_)); \
  } while (0)

// ---- the step's collectives between the shards (rank r: device dev[r], stream st[r]) ----
struct Xport {
  virtual ~Xport() = default;
  virtual const char *name() const = 0;
  // every rank r: out[r] + s * bytes = in[s] (bytes each)
  virtual void all_gather(const std::vector<const void *> &in, const std::vector<void *> &out, size_t bytes) = 0;
  // every rank r: out[r] + s * bytes = in[s] + r * bytes
  virtual void all_to_all(const std::vector<const void *> &in, const std::vector<void *> &out, size_t bytes) = 0;
  // every rank r: out[r] = src (on rank 0's device)
  virtual void broadcast(const void *src, const std::vector<void *> &out, size_t bytes) = 0;
};

// device copies; every destination stream first waits for every source stream, and every source stream then
// waits for the copies out of it (the next phase of a rank may overwrite what another rank still copies)
struct CopyXport : Xport {
  std::vector<int> dev;
  std::vector<hipStream_t> st;
  std::vector<hipEvent_t> ev;
  CopyXport(const std::vector<int> &d, const std::vector<hipStream_t> &s) : dev(d), st(s), ev(d.size(), nullptr) {
    for (size_t r = 0; r < dev.size(); ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      HIPCHK(hipEventCreateWithFlags(&ev[r], hipEventDisableTiming));
      for (size_t q = 0; q < dev.size(); ++q) {
        int ok = 0;
        if (dev[q] != dev[r] && hipDeviceCanAccessPeer(&ok, dev[r], dev[q]) == hipSuccess && ok) {
          const hipError_t e = hipDeviceEnablePeerAccess(dev[q], 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
          (void)hipGetLastError();
        }
      }
    }
  }
  ~CopyXport() override {
    for (size_t r = 0; r < ev.size(); ++r)
      if (ev[r]) {
        (void)hipSetDevice(dev[r]);
        (void)hipEventDestroy(ev[r]);
      }
  }
  const char *name() const override { return "device copies"; }
  void fence() {
    for (size_t r = 0; r < dev.size(); ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      HIPCHK(hipEventRecord(ev[r], st[r]));
    }
    for (size_t r = 0; r < dev.size(); ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      for (size_t s = 0; s < dev.size(); ++s)
        if (s != r) HIPCHK(hipStreamWaitEvent(st[r], ev[s], 0));
    }
  }
  void copy(size_t r, void *dst, size_t s, const void *src, size_t bytes) {
    if (!bytes) return;
    HIPCHK(hipSetDevice(dev[r]));
    if (dev[r] == dev[s]) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st[r]));
    else HIPCHK(hipMemcpyPeerAsync(dst, dev[r], src, dev[s], bytes, st[r]));
  }
  void all_gather(const std::vector<const void *> &in, const std::vector<void *> &out, size_t b) override {
    fence();
    for (size_t r = 0; r < dev.size(); ++r)
      for (size_t s = 0; s < dev.size(); ++s) copy(r, static_cast<char *>(out[r]) + s * b, s, in[s], b);
    fence();
  }
  void all_to_all(const std::vector<const void *> &in, const std::vector<void *> &out, size_t b) override {
    fence();
    for (size_t r = 0; r < dev.size(); ++r)
      for (size_t s = 0; s < dev.size(); ++s)
        copy(r, static_cast<char *>(out[r]) + s * b, s, static_cast<const char *>(in[s]) + r * b, b);
    fence();
  }
  void broadcast(const void *src, const std::vector<void *> &out, size_t b) override {
    fence();
    for (size_t r = 0; r < dev.size(); ++r) copy(r, out[r], 0, src, b);
    fence();
  }
};

// RCCL over xGMI: one communicator per shard device (ncclCommInitAll), grouped calls from this one thread
struct RcclXport : Xport {
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> st;
  RcclXport(const std::vector<int> &dev, const std::vector<hipStream_t> &s) : comm(dev.size(), nullptr), st(s) {
    const Rccl &R = rccl();
    if (!R.why.empty()) throw Error(PYR_E_DEVICE, "multi-GPU index: " + R.why);
    NCCLCHK(R.init_all(comm.data(), (int)dev.size(), dev.data()));
  }
  ~RcclXport() override {
    for (ncclComm_t c : comm)
      if (c) (void)rccl().destroy(c);
  }
  const char *name() const override { return "RCCL"; }
  void all_gather(const std::vector<const void *> &in, const std::vector<void *> &out, size_t b) override {
    const Rccl &R = rccl();
    NCCLCHK(R.group_start());
    for (size_t r = 0; r < comm.size(); ++r) NCCLCHK(R.all_gather(in[r], out[r], b, ncclUint8, comm[r], st[r]));
    NCCLCHK(R.group_end());
  }
  void all_to_all(const std::vector<const void *> &in, const std::vector<void *> &out, size_t b) override {
    const Rccl &R = rccl();
    NCCLCHK(R.group_start());
    for (size_t r = 0; r < comm.size(); ++r) NCCLCHK(R.all_to_all(in[r], out[r], b, ncclUint8, comm[r], st[r]));
    NCCLCHK(R.group_end());
  }
  void broadcast(const void *src, const std::vector<void *> &out, size_t b) override {
    const Rccl &R = rccl();
    NCCLCHK(R.group_start());
    for (size_t r = 0; r < comm.size(); ++r)
      NCCLCHK(R.broadcast(r == 0 ? src : out[r], out[r], b, ncclUint8, 0, comm[r], st[r]));
    NCCLCHK(R.group_end());
  }
};

// dist.list_owners: lists by length (desc, ties by id) to the shard with the fewest rows so far (ties: lowest)
std::vector<int32_t> list_owners(const std::vector<int32_t> &len, int W) {
  std::vector<int> order(len.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return len[a] > len[b]; });
  using E = std::pair<int64_t, int>;
  std::priority_queue<E, std::vector<E>, std::greater<E>> heap;
  for (int r = 0; r < W; ++r) heap.push({0, r});
  std::vector<int32_t> owner(len.size(), 0);
  for (int l : order) {
    E e = heap.top();
    heap.pop();
    owner[l] = e.second;
    heap.push({e.first + len[l], e.second});
  }
  return owner;
}

constexpr int SAMPLE_ROWS = 512;  // == dist.SAMPLE_ROWS: the replicated sample's rows per list

struct MultiIvfIndex : Index {
  std::unique_ptr<Index> stage;
  int W = 0;
  std::vector<int> dev;  // shard r's device
  std::vector<std::unique_ptr<Index>> shard;
  std::vector<hipStream_t> st;  // shard r's step stream
  std::vector<hipEvent_t> ev;   // shard r's last step event
  hipEvent_t ev_in = nullptr, ev_cnt = nullptr;  // the caller's stream -> the shards; the counts' copy (device 0)
  int32_t *h_counts = nullptr;                    // pinned: every home's failure count
  std::unique_ptr<Xport> xp;
  bool distinct = true;  // every shard on its own device (RCCL)
  bool dealt = false;    // the shards hold the stage's current lists
  std::vector<int32_t> owner;
  std::mutex step_mu;  // one list-sharded step at a time: its buffers and streams are shared
  int fcap = 256;
  struct Rank {  // one shard's step buffers (its device)
    DevMem q_all, plan_home, plan_all, rec, rec_home, out_s, out_l, out_c, fail_home, fail_all, fail_full,
        fail_round, rrec, rrec_home;
  };
  std::vector<std::unique_ptr<Rank>> rk;
  int64_t last_max_fail = 0, last_rounds = 0;
  std::atomic<int64_t> n_sharded{0}, n_staged{0};
  void shard_info(int32_t *shards, int32_t *xport, int64_t *sharded, int64_t *staged, int64_t *max_fail,
                  int64_t *rounds) const override {
    *shards = W;
    *xport = !xp ? 0 : std::strcmp(xp->name(), "RCCL") == 0 ? 2 : 1;
    *sharded = n_sharded.load();
    *staged = n_staged.load();
    *max_fail = last_max_fail;
    *rounds = last_rounds;
  }

  explicit MultiIvfIndex(const pyr_index_desc &d) : Index(d) {
    if (d.kind != PYR_IVF_FLAT) throw Error(PYR_E_ARG, "a multi-GPU index is IVF_FLAT (lists sharded whole)");
    std::vector<int> devs;
    for (int b = 0; b < 64; ++b)
      if (d.device_mask >> b & 1) devs.push_back(b);
    if (devs.empty()) devs.push_back(d.device);
    W = d.shards > 0 ? d.shards : (int)devs.size();
    if (W > 64) throw Error(PYR_E_ARG, "at most 64 shards");
    pyr_index_desc sd = d;
    sd.device_mask = 0;
    sd.shards = 0;
    sd.device = devs[0];
    stage.reset(create_index(sd));
    for (int r = 0; r < W; ++r) {
      dev.push_back(devs[r % devs.size()]);
      sd.device = dev.back();
      shard.emplace_back(create_index(sd));
    }
    for (int r = 0; r < W; ++r)
      for (int s = 0; s < r; ++s) distinct = distinct && dev[r] != dev[s];
    st.assign(W, nullptr);
    ev.assign(W, nullptr);
    for (int r = 0; r < W; ++r) {
      rk.push_back(std::make_unique<Rank>());
      HIPCHK(hipSetDevice(dev[r]));
      HIPCHK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&ev[r], hipEventDisableTiming));
    }
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_cnt, hipEventDisableTiming));
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&h_counts), sizeof(int32_t) * 64, hipHostMallocDefault));
    if (const char *e = knob("PYR_SHARD_FCAP")) fcap = std::max(1, atoi(e));
  }
  ~MultiIvfIndex() override {
    for (int r = 0; r < W; ++r) {
      (void)hipSetDevice(dev[r]);
      if (st[r]) (void)hipStreamSynchronize(st[r]);
    }
    xp.reset();
    for (int r = 0; r < W; ++r) {
      (void)hipSetDevice(dev[r]);
      rk[r].reset();
      if (ev[r]) (void)hipEventDestroy(ev[r]);
      if (st[r]) (void)hipStreamDestroy(st[r]);
    }
    (void)hipSetDevice(device);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_cnt) (void)hipEventDestroy(ev_cnt);
    if (h_counts) (void)hipHostFree(h_counts);
  }

  // ---- IVectorIndex on the stage; the shards follow ----
  void after_write() override {
    stage->after_write();
    stage->note_write();
  }
  void add(const float *x, int64_t n, const int64_t *labels, bool upsert) override {
    stage->add(x, n, labels, upsert);
    if (dealt) drop_from_shards(labels, n);  // a buffer row now shadows its list entry (:169-180, :210)
  }
  void remove(const int64_t *labels, int64_t n, uint8_t *removed) override {
    std::vector<int64_t> pos;
    if (dealt)
      for (int64_t i = 0; i < n; ++i) {
        const int64_t p = stage->ms_position(labels[i]);
        if (p >= 0) pos.push_back(p);
      }
    stage->remove(labels, n, removed);
    stage->note_write();
    if (dealt) drop_positions(pos);
  }
  void build() override {
    stage->build();
    deal();
  }
  void load(const std::string &path) override {
    dealt = false;
    stage->load(path);
    deal();
  }
  void snapshot(const std::string &path) override { stage->snapshot(path); }
  void set_centroids(const float *c, int nl) override { stage->set_centroids(c, nl); }
  void reserve(int64_t rows) override { stage->reserve(rows); }
  int64_t count() const override { return stage->count(); }
  void centroids(float *out, int32_t *nl) const override { stage->centroids(out, nl); }
  void ivf_layout(int64_t *off, int64_t *labels, uint8_t *live, int64_t *total) const override {
    stage->ivf_layout(off, labels, live, total);
  }
  void all_labels(std::vector<int64_t> &out) const override { stage->all_labels(out); }
  int probe_only(const float *d_q, int64_t nq, int nprobe, int32_t *d_out, Workspace &ws) override {
    Workspace &sw = stage->ws_for_stream(ws.st);
    sw.ext_probes = ws.ext_probes;
    sw.ext_nprobe = ws.ext_nprobe;
    return stage->probe_only(d_q, nq, nprobe, d_out, sw);
  }

  // the shards' entries of the given labels leave their lists (a buffer write shadows them, or a Delete)
  void drop_from_shards(const int64_t *labels, int64_t n) {
    std::vector<int64_t> pos;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t p = stage->ms_position(labels[i]);
      if (p >= 0) pos.push_back(p);
    }
    drop_positions(pos);
  }
  void drop_positions(const std::vector<int64_t> &pos) {
    if (pos.empty()) return;
    for (int r = 0; r < W; ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      shard[r]->remove(pos.data(), (int64_t)pos.size(), nullptr);  // (a shard ignores labels it does not hold)
      shard[r]->note_write();
    }
    // every shard's replicated live lengths (the MaxScans accounting of the homes)
    Index::MsLists L;
    HIPCHK(hipSetDevice(device));
    if (!stage->ms_lists(L)) return;
    std::vector<int64_t> glen(L.llive.begin(), L.llive.end());
    for (int r = 0; r < W; ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      shard[r]->ms_set_list_lengths(glen.data(), L.nlist);
    }
    HIPCHK(hipSetDevice(device));
  }

  // the stage's built lists -> the shards, whole, plus the replicated samples
  void deal() {
    dealt = false;
    Index::MsLists L;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamSynchronize(stage->wst));
    if (!stage->ms_lists(L)) return;
    int P0 = 0;
    const pyr_search_params p0{-1, 0, -1};
    if (!stage->ms_shardable(1, p0, &P0)) return;  // Cosine, dims without fp16 tiles: the stage answers alone
    const int nl = L.nlist;
    owner = list_owners(L.llive, W);
    // every shard's visible rows in list order (labels: their stage positions), and each list's first rows
    std::vector<std::vector<int64_t>> pos(W);
    std::vector<std::vector<int32_t>> asg(W);
    std::vector<int64_t> spos, counts(nl, 0), glen(nl);
    for (int l = 0; l < nl; ++l) {
      glen[l] = L.llive[l];
      for (int32_t p = L.lb[l]; p < L.lb[l] + L.llen[l]; ++p) {
        if (L.state[p] != 1) continue;
        pos[owner[l]].push_back(p);
        asg[owner[l]].push_back(l);
        if (counts[l] < SAMPLE_ROWS) {
          spos.push_back(p);
          ++counts[l];
        }
      }
    }
    const hipStream_t s0 = stage->wst;
    DevMem dpos, X;
    for (int r = 0; r < W; ++r) {
      const int64_t n = (int64_t)pos[r].size();
      HIPCHK(hipSetDevice(device));
      dpos.ensure(sizeof(int64_t) * std::max<int64_t>(n, 1));
      X.ensure(sizeof(float) * (size_t)std::max<int64_t>(n, 1) * dim);
      if (n) HIPCHK(hipMemcpyAsync(dpos.p, pos[r].data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, s0));
      stage->ms_gather_rows(dpos.as<int64_t>(), n, X.as<float>(), s0);
      HIPCHK(hipStreamSynchronize(s0));
      HIPCHK(hipSetDevice(dev[r]));
      if (dev[r] == device) {
        shard[r]->ms_commit(X.as<float>(), n, asg[r], pos[r], L.cents.data(), nl);
      } else {
        DevMem Xr;
        Xr.ensure(sizeof(float) * (size_t)std::max<int64_t>(n, 1) * dim);
        if (n) HIPCHK(hipMemcpyPeer(Xr.p, dev[r], X.p, device, sizeof(float) * (size_t)n * dim));
        shard[r]->ms_commit(Xr.as<float>(), n, asg[r], pos[r], L.cents.data(), nl);
      }
    }
    // the replicated sample of every list: its first <= 512 rows (dist.gather_samples)
    HIPCHK(hipSetDevice(device));
    const int64_t ns = (int64_t)spos.size();
    std::vector<float> srows((size_t)std::max<int64_t>(ns, 1) * dim);
    dpos.ensure(sizeof(int64_t) * std::max<int64_t>(ns, 1));
    X.ensure(sizeof(float) * (size_t)std::max<int64_t>(ns, 1) * dim);
    if (ns) {
      HIPCHK(hipMemcpyAsync(dpos.p, spos.data(), sizeof(int64_t) * ns, hipMemcpyHostToDevice, s0));
      stage->ms_gather_rows(dpos.as<int64_t>(), ns, X.as<float>(), s0);
      HIPCHK(hipMemcpyAsync(srows.data(), X.p, sizeof(float) * (size_t)ns * dim, hipMemcpyDeviceToHost, s0));
    }
    HIPCHK(hipStreamSynchronize(s0));
    for (int r = 0; r < W; ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      shard[r]->set_list_samples(srows.data(), counts.data(), glen.data(), nl);
    }
    HIPCHK(hipSetDevice(device));
    dealt = true;
  }

  // IVectorIndex.Search: the list-sharded step where it applies, else the stage alone
  void search(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, float *d_s, int64_t *d_l,
              int32_t *d_c, Workspace &ws) override {
    int P = 0;
    if (!dealt || ws.ext_probes || nq <= 0 || !stage->ms_shardable(k, prm, &P) || prm.max_scans == 0) {
      Workspace &sw = stage->ws_for_stream(ws.st);
      sw.ext_probes = ws.ext_probes;
      sw.ext_nprobe = ws.ext_nprobe;
      ++n_staged;
      try {
        stage->search(d_q, nq, k, prm, d_s, d_l, d_c, sw);
      } catch (...) {
        sw.ext_probes = nullptr;
        throw;
      }
      sw.ext_probes = nullptr;
      return;
    }
    std::lock_guard<std::mutex> g(step_mu);
    ++n_sharded;
    try {
      sharded_search(d_q, nq, k, prm, P, d_s, d_l, d_c, ws);
    } catch (...) {
      for (int r = 0; r < W; ++r) {
        (void)hipSetDevice(dev[r]);
        (void)hipStreamSynchronize(st[r]);
      }
      (void)hipSetDevice(device);
      throw;
    }
    HIPCHK(hipSetDevice(device));
  }

  void merge(int r, const void *rec, int64_t nrec, int k, const int32_t *qsel, int cap, int32_t *fail, int fc) {
    Rank &R = *rk[r];
    ShardMergeArgs a{};
    a.rec = static_cast<const uint8_t *>(rec);
    a.nparts = W;
    a.nrec = nrec;
    a.k = k;
    a.qsel = qsel;
    a.cap = cap;
    a.out_s = R.out_s.as<float>();
    a.out_l = R.out_l.as<int64_t>();
    a.out_c = R.out_c.as<int32_t>();
    a.fail = fail;
    a.fcap = fc;
    if (fail) {
      WordFill z;
      z.add(fail, 1, 0);
      launch_fill_words(z, st[r]);
    }
    launch_shard_merge(a, qsel ? std::min<int64_t>(cap, nrec) : nrec, st[r]);
  }

  template <class F>
  void each(F &&f) {
    for (int r = 0; r < W; ++r) {
      HIPCHK(hipSetDevice(dev[r]));
      f(r);
    }
  }
  template <class T>
  std::vector<const void *> cptrs(DevMem Rank::*m, size_t off = 0) {
    std::vector<const void *> v(W);
    for (int r = 0; r < W; ++r) v[r] = (rk[r].get()->*m).as<char>() + off * sizeof(T);
    return v;
  }
  std::vector<void *> ptrs(DevMem Rank::*m) {
    std::vector<void *> v(W);
    for (int r = 0; r < W; ++r) v[r] = (rk[r].get()->*m).p;
    return v;
  }

  void sharded_search(const float *d_q, int64_t nq, int k, const pyr_search_params &prm, int P, float *d_s,
                      int64_t *d_l, int32_t *d_c, Workspace &ws) {
    if (!xp) {
      const char *e = knob("PYR_SHARD_XPORT");
      const bool use_rccl = e ? std::strcmp(e, "rccl") == 0 : distinct;
      if (use_rccl && !distinct) throw Error(PYR_E_ARG, "RCCL needs one shard per device");
      if (use_rccl) xp = std::make_unique<RcclXport>(dev, st);
      else xp = std::make_unique<CopyXport>(dev, st);
    }
    const bool budget = prm.max_scans >= 0;
    const int S = shard_plan_stride(P, budget);
    const int64_t nqh = (nq + W - 1) / W, Qp = nqh * W;
    const int64_t rb = shard_record_bytes(k);
    const int fc = (int)std::min<int64_t>(fcap, nqh);
    // the caller's stream (device 0) -> every shard stream
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipEventRecord(ev_in, ws.st));
    std::vector<Workspace *> sw(W);
    each([&](int r) {
      Rank &R = *rk[r];
      R.q_all.ensure(sizeof(float) * Qp * dim);
      R.plan_home.ensure(sizeof(int32_t) * nqh * S);
      R.plan_all.ensure(sizeof(int32_t) * Qp * S);
      R.rec.ensure((size_t)(Qp * rb));
      R.rec_home.ensure((size_t)(Qp * rb));
      R.out_s.ensure(sizeof(float) * nqh * k);
      R.out_l.ensure(sizeof(int64_t) * nqh * k);
      R.out_c.ensure(sizeof(int32_t) * nqh);
      R.fail_home.ensure(sizeof(int32_t) * (1 + nqh));
      R.fail_all.ensure(sizeof(int32_t) * W * (1 + fc));
      R.fail_round.ensure(sizeof(int32_t) * W * (1 + fc));
      R.rrec.ensure((size_t)(W * fc * rb));
      R.rrec_home.ensure((size_t)(W * fc * rb));
      HIPCHK(hipStreamWaitEvent(st[r], ev_in, 0));
      if (Qp > nq)  // the last home's padding rows: zero queries, planned and scanned, their answers dropped
        HIPCHK(hipMemsetAsync(R.q_all.as<float>() + nq * dim, 0, sizeof(float) * (Qp - nq) * dim, st[r]));
      sw[r] = &shard[r]->ws_for_stream(st[r]);
    });
    xp->broadcast(d_q, ptrs(&Rank::q_all), sizeof(float) * nq * dim);
    each([&](int r) {  // 1. plan: coarse ranking, T_q (and MaxScans budgets) of the home's slice
      Rank &R = *rk[r];
      const int got = shard[r]->shard_prepare(R.q_all.as<float>() + r * nqh * dim, nqh, k, prm,
                                             R.plan_home.as<int32_t>(), *sw[r]);
      if (got != P) throw Error(PYR_E_STATE, "multi-GPU index: plan width mismatch");
    });
    xp->all_gather(cptrs<int32_t>(&Rank::plan_home), ptrs(&Rank::plan_all), sizeof(int32_t) * nqh * S);
    each([&](int r) {  // 2. every shard: the pairs of its lists -> one record per query
      Rank &R = *rk[r];
      shard[r]->shard_search(R.q_all.as<float>(), Qp, k, R.plan_all.as<int32_t>(), P, budget, R.rec.p, *sw[r]);
    });
    xp->all_to_all(cptrs<uint8_t>(&Rank::rec), ptrs(&Rank::rec_home), (size_t)(nqh * rb));
    each([&](int r) {  // 3. home: merge + certificate, every failure listed
      Rank &R = *rk[r];
      merge(r, R.rec_home.p, nqh, k, nullptr, 0, R.fail_home.as<int32_t>(), (int)nqh);
    });
    xp->all_gather(cptrs<int32_t>(&Rank::fail_home), ptrs(&Rank::fail_all), sizeof(int32_t) * (1 + fc));
    HIPCHK(hipSetDevice(dev[0]));  // every home's count, as every rank has them (rank 0's copy)
    for (int s = 0; s < W; ++s)
      HIPCHK(hipMemcpyAsync(h_counts + s, rk[0]->fail_all.as<int32_t>() + s * (1 + fc), sizeof(int32_t),
                            hipMemcpyDeviceToHost, st[0]));
    HIPCHK(hipEventRecord(ev_cnt, st[0]));
    auto rerun_round = [&](DevMem Rank::*fails) {
      each([&](int r) {
        Rank &R = *rk[r];
        shard[r]->shard_rerun(R.q_all.as<float>(), Qp, k, R.plan_all.as<int32_t>(), P, budget,
                              (R.*fails).as<int32_t>(), W, fc, nqh, R.rrec.p, *sw[r]);
      });
      xp->all_to_all(cptrs<uint8_t>(&Rank::rrec), ptrs(&Rank::rrec_home), (size_t)(fc * rb));
      each([&](int r) {
        Rank &R = *rk[r];
        merge(r, R.rrec_home.p, fc, k, (R.*fails).as<int32_t>() + r * (1 + fc), fc, nullptr, 0);
      });
    };
    HIPCHK(hipSetDevice(dev[0]));
    HIPCHK(hipEventSynchronize(ev_cnt));
    int64_t mx = 0;
    for (int s = 0; s < W; ++s) mx = std::max<int64_t>(mx, h_counts[s]);
    const int64_t rounds = mx > fc ? (mx - 1) / fc : 0;
    last_max_fail = mx;
    last_rounds = rounds;
    // 4. no failure anywhere (the usual step): no re-run; else the first fcap failures of every home
    if (mx > 0) rerun_round(&Rank::fail_all);
    if (rounds > 0) {  // 5. further rounds over the rest of every home's failures
      each([&](int r) { rk[r]->fail_full.ensure(sizeof(int32_t) * W * (1 + nqh)); });
      xp->all_gather(cptrs<int32_t>(&Rank::fail_home), ptrs(&Rank::fail_full), sizeof(int32_t) * (1 + nqh));
      for (int64_t j = 1; j <= rounds; ++j) {
        each([&](int r) {
          launch_fail_round(rk[r]->fail_full.as<int32_t>(), W, 1 + nqh, (int)(j * fc), fc,
                            rk[r]->fail_round.as<int32_t>(), st[r]);
        });
        rerun_round(&Rank::fail_round);
      }
    }
    // 6. the homes' answers -> the caller's buffers on device 0, positions -> labels
    each([&](int r) {
      Rank &R = *rk[r];
      const int64_t a = r * nqh, nr = std::max<int64_t>(0, std::min(nqh, nq - a));
      auto put = [&](void *dst, const void *src, size_t b) {
        if (!b || !dst) return;
        if (dev[r] == device) HIPCHK(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, st[r]));
        else HIPCHK(hipMemcpyPeerAsync(dst, device, src, dev[r], b, st[r]));
      };
      put(d_s ? d_s + a * k : nullptr, R.out_s.p, sizeof(float) * nr * k);
      put(d_l ? d_l + a * k : nullptr, R.out_l.p, sizeof(int64_t) * nr * k);
      put(d_c ? d_c + a : nullptr, R.out_c.p, sizeof(int32_t) * nr);
      HIPCHK(hipEventRecord(ev[r], st[r]));
    });
    HIPCHK(hipSetDevice(device));
    for (int r = 0; r < W; ++r) HIPCHK(hipStreamWaitEvent(ws.st, ev[r], 0));
    if (d_l) launch_map_positions(d_l, nq * k, stage->ms_position_labels(), ws.st);
    HIPCHK(hipGetLastError());
  }
};

}  // namespace

Index *create_multi_index(const pyr_index_desc &d) { return new MultiIvfIndex(d); }

}  // namespace pyr
