// engine.h -- host runtime of libpyrope_hip.so: device-resident index objects
// restating the reference's IVectorIndex implementations
// (src/Pyrope.GarnetServer/Vector/{BruteForce,IvfFlat,IvfPq}VectorIndex.cs).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pyrope_ann.h"
#include "kernels.h"

namespace pyr {

struct Error : std::runtime_error {
  pyr_status status;
  Error(pyr_status s, const std::string &m) : std::runtime_error(m), status(s) {}
};

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess)                                                                           \
      throw ::pyr::Error(PYR_E_DEVICE, std::string(#x " failed: ") + hipGetErrorString(e_));        \
  } while (0)

// device allocation that only grows
struct DevMem {
  void *p = nullptr;
  size_t n = 0;
  DevMem() = default;
  DevMem(const DevMem &) = delete;
  DevMem &operator=(const DevMem &) = delete;
  ~DevMem() { release(); }
  // make room for `bytes`; content discarded
  void ensure(size_t bytes);
  // make room for `bytes`; first `keep` bytes preserved (stream-ordered copy, then sync)
  void grow_keep(size_t bytes, size_t keep, hipStream_t st);
  void release();
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// Pinned (mapped) host staging for small writes: K slots the write kernel reads in place, reused in groups of
// 8 once the group's event has completed, so a write never waits for the device (RowStore::write's
// small-batch path).
struct PinnedRing {
  static constexpr int K = 64;
  char *host[K] = {};
  char *dev[K] = {};      // the slots' device addresses (hipHostGetDevicePointer)
  hipEvent_t ev[K] = {};  // (the first K / 8: one per group)
  size_t bytes = 0;
  int next = 0;
  // a slot of at least `need` bytes whose previous copy has completed; *slot = its index
  char *take(size_t need, int *slot);
  void done(int slot, hipStream_t st);  // the copy out of `slot` is enqueued on st
  ~PinnedRing();
};

// Blocked fp32 row store on device (+ host mirrors of labels and visibility).
struct RowStore {
  int dim = 0;
  bool cosine = false;
  int64_t n = 0;    // slots in use
  int64_t cap = 0;  // allocated slots (multiple of 8)
  DevMem rows, norms, live, labels;
  DevMem rsq;       // per slot |x|^2 (MFMA filter, filter.hip)
  DevMem rmax;      // score_key of the largest |x|^2 ever stored (device scalar, only grows)
  // fp16 tile copy for the fp16 filter (filter16.hip): h16 tiles of 32 slots, per-slot meta
  // (L2 -|x|^2 / IP 0 / -inf when not live), the power-of-two scale sx with the largest |x_i|
  // ever stored (amax) below 2^14.  Kept only when f16 is set (FLAT slots, IVF lists).
  bool f16 = false;
  int met16 = 0;
  // tile dimension (scan_tile_dim): dim, or the stream scan's padded dimension (96 for 65..96 ...); the
  // tiles are zero-padded, the fp32 rows and everything exact keep dim
  int dt = 0;
  int tdim() const { return dt > 0 ? dt : dim; }
  float sx = 0.0f;
  float amax = 0.0f;
  DevMem h16, meta, amaxd;
  // IVF lists: the tiles hold residuals x - c[list] (resid), with rsq16 = |x - c|^2 per row for meta.
  // FLAT L2 (center16): one center, the mean of the first rows written, fixed from then on; rmax_r =
  // score_key of the largest |x - center|^2 (the certificate's residual norm bound).
  bool resid = false;
  bool center16 = false;
  DevMem rsq16, center, rmax_r;
  // the host copy of the center and the slots in use when it was set: the center follows the rows
  // (recenter) each time the store has doubled since, and at a FLAT build (the Delta compaction)
  std::vector<float> hcenter;
  int64_t center_rows = 0;
  void recenter(hipStream_t st);
  PinnedRing ring;
  // f16 stores: a row-major fp32 copy of the rows for the exact refine (a candidate's 512 B read
  // contiguously; the blocked layout spreads one row over D 32-B sectors)
  DevMem rrm;
  // the stream scan's per-row term meta + E_row (launch_row_terms), cached for (gen, metric, kr, kx):
  // gen advances with every change of the rows, meta or norms (reserve, write, set_live, encode16, an
  // IVF commit)
  DevMem mub;
  uint64_t gen = 1, mub_gen = 0;
  int mub_met = -1;
  float mub_kr = 0.0f, mub_kx = 0.0f;
  // the refresh is enqueued on the caller's stream without a host sync; another stream using the cached
  // terms waits for mub_ev until it is seen complete.  A refresh cannot run while st is being captured
  // (the index changed since its last search: PYR_E_STATE) -- writes refresh the FLAT store's terms on the
  // write stream themselves (FlatIndex::after_write)
  hipEvent_t mub_ev = nullptr;
  hipStream_t mub_st = nullptr;
  bool mub_done = true;
  const float *row_terms(int met, float kr, float kx, hipStream_t st);
  const float *meta_norms() const { return resid ? rsq16.as<float>() : rsq.as<float>(); }
  std::vector<int64_t> hlabels;
  std::vector<uint8_t> hlive;
  void reserve(int64_t slots, hipStream_t st);
  // write rows (row-major x, n rows: host memory, or device memory when x_dev) into slots; updates
  // labels/live/norms.  A device source is read in place (no staging copy, no host hop)
  // Returns true when the small-batch path took the write (host rows, <= SMALL_WRITE rows, the fp16 scale
  // unchanged): one pinned staging copy + one fused kernel, no host synchronization and no use of stage_i;
  // otherwise the bulk path ran (stage_i then holds the device slots) and st is synchronized.
  // (need_slots: the caller reads stage_i afterwards -- the bulk path always)
  bool write(const float *x, const int64_t *slots, const int64_t *labs, int64_t cnt, hipStream_t st,
             DevMem &stage_x, DevMem &stage_i, bool x_dev = false, uint8_t *q8ok = nullptr, bool need_slots = false);
  void set_live(const std::vector<int64_t> &slots, uint8_t v, hipStream_t st, DevMem &stage);
  // fp16 copy of slots (device list, or [0, cap) when null) with the current scale; raises the
  // scale (and re-encodes every slot) when a row exceeds it.  Synchronizes st.
  void encode16(const int64_t *d_slots, int64_t cnt, hipStream_t st);
  void clear() {
    n = 0;
    hlabels.clear();
    hlive.clear();
  }
  RowStore() = default;
  RowStore(const RowStore &) = delete;
  RowStore &operator=(const RowStore &) = delete;
  ~RowStore() {
    if (mub_ev) (void)hipEventDestroy(mub_ev);
  }
};

// HBM bytes of an IVF_FLAT index of nrows rows and of one stream-path search of nq queries on it
// (engine.cpp; pyr_ivf_memory_plan)
void ivf_memory_plan(int dim, int64_t nrows, int nlist, int64_t max_len, int64_t nq, int nprobe, int k,
                     int64_t *index_bytes, int64_t *workspace_bytes);

// measurement only (PYR_WRITE_PROF=1): the write path's host time by section (engine.cpp WriteProf)
bool wprof_on();
void wprof_add(int section, double seconds);
void note_write_call();

struct Workspace {
  hipStream_t st = nullptr;
  bool own_stream = false;
  std::mutex m;
  DevMem cfail, cnfail;  // coarse ranking on the matrix cores (coarse.hip launch_coarse_mfma)
  DevMem cpr_s, cpr_l;  // coarse step through the FLAT filter (on nested()): probe scores, centroid ids
  DevMem q, qn, qt, items, nitems, items2, nitems2, items3, nitems3, qlist, part_s, part_k, probes, cpart_s, cpart_k,
      limits;
  DevMem ivf_cnt, ivf_fill, ivf_qoff, ivf_ioff, gthr;
  DevMem ivf_cnt2, ivf_fill2, ivf_qoff2, ivf_ioff2, qlist2, qpos;
  DevMem bx_s, bx_l, bx_c, lx_s, lx_l, lx_c;  // IVF_PQ with a buffer: its and the lists' answers
  DevMem rrdone;       // the device re-run's per-query unit counters (rerun_done, engine.cpp)
  WordFill pz;         // counters the next coarse ranking zeroes (defer_stream_counters, engine.cpp)
  bool pz_set = false;  // second item set (nearest-list seeding)
  DevMem out_s, out_l, out_c;
  DevMem ms, mk, fail, fail_cnt, fq, fs, fl, fc;  // MFMA filter: merged candidates, certificate failures
  DevMem fprobes;                                 // probe lists of the failing queries (IVF_PQ LUT re-run)
  DevMem q8q, q8qs;                               // 8-bit search mode: quantized queries, their sums
  // stream-and-emit list scan (stream16.hip): query operands, samples, thresholds, candidate regions
  DevMem sbq, sqsc, ssamp, sthr, scand, scn, scf, swork, fail2, fail_cnt2;
  DevMem rrpart;  // device re-run of certificate failures: per (query, probe) top-k keys
  DevMem tdbg;    // measurement only (PYR_STREAM_TIMING)
  DevMem vlb, vle, vcents;  // FLAT on the stream scan: its chunks as lists (FlatIndex::search_stream)
  DevMem cq, ccs, ccl, ccc;  // Cosine on the filter path: unit queries, inner-product candidates
  DevMem shp, shthr, rpos;  // list-sharded search: unpacked plan (probes, T_q), re-run record slots
  DevMem plim;              // IVF stream search with MaxScans: the pairs' row bounds at their qlist positions
  int64_t max_scans = -1;   // the MaxScans of the IVF stream search in progress (-1: none)
  uint64_t wgen_seen = 0;                         // the index's write generation this stream is ordered after
  const int32_t *ext_probes = nullptr;            // caller-ranked probe lists [nq][ext_nprobe] (multi-GPU)
  bool skip_buffer = false;                       // IVF_PQ LUT scan: the lists only (the buffer merged by the caller)
  int32_t ext_nprobe = 0;
  // the re-run of certificate failures searches with its own buffers on the same stream
  std::unique_ptr<Workspace> sub;
  Workspace &nested() {
    if (!sub) {
      sub = std::make_unique<Workspace>();
      sub->st = st;
    }
    return *sub;
  }
  ~Workspace() {
    if (own_stream && st) (void)hipStreamDestroy(st);
  }
};

struct Index {
  pyr_index_desc desc{};
  int dim = 0, metric = 0, device = 0;
  mutable std::shared_mutex mu;
  std::mutex wmu;             // snapshot (shared lock on mu) vs the write stream / staging buffers
  hipStream_t wst = nullptr;  // stream for writes/builds
  DevMem stage_x, stage_i, stage_b;
  std::mutex ws_mu;
  std::vector<std::unique_ptr<Workspace>> free_ws;
  std::map<hipStream_t, std::unique_ptr<Workspace>> stream_ws;
  // writes that return before the device ran them (RowStore::write's small-batch path): an event on wst
  // after every write call; a search stream waits for it once per write generation (order_after_writes)
  hipEvent_t wev = nullptr;
  uint64_t wgen = 0;
  void note_write();
  void order_after_writes(Workspace &ws);
  virtual void after_write() {}  // per-kind work at the end of a write call (on wst, no host sync)
  // measurement only: the workspace, queries and candidate capacity of the last stream-scan slice, for
  // pyr_index_debug_candidates (with PYR_STREAM_EMIT_ALL: every row's bound)
  Workspace *dbg_ws = nullptr;
  int64_t dbg_nq = 0;
  int32_t dbg_cap = 0;
  void note_stream_slice(Workspace &ws, int64_t nq, int cap);
  virtual int64_t key_label(uint32_t key) const {  // the label of a stream-scan storage key (-1: none)
    (void)key;
    return -1;
  }
  void debug_candidates(int64_t nq, int32_t cap, float *h_ub, int64_t *h_label, int32_t *h_cnt);

  explicit Index(const pyr_index_desc &d);
  virtual ~Index();
  virtual void add(const float *x, int64_t n, const int64_t *labels, bool upsert) = 0;
  virtual void remove(const int64_t *labels, int64_t n, uint8_t *removed) = 0;
  virtual void build() {}
  // enqueue a batch search of device queries on ws.st; outputs device buffers
  virtual void search(const float *d_q, int64_t nq, int k, const pyr_search_params &p, float *d_s, int64_t *d_l,
                      int32_t *d_c, Workspace &ws) = 0;
  virtual int64_t count() const = 0;
  virtual void centroids(float *out, int32_t *nlist) const {
    (void)out;
    *nlist = 0;
  }
  virtual void ivf_layout(int64_t *off, int64_t *labels, uint8_t *live, int64_t *total) const;
  virtual void pq_state(float *cb, int32_t *ksub, uint8_t *codes) const;
  // the labels of every row the index holds (buffer and lists; a label may repeat when a buffer row
  // shadows a list entry): the shim's id map of an image loaded without one (pyr_index_labels)
  virtual void all_labels(std::vector<int64_t> &out) const = 0;
  // BruteForceVectorIndex.Scan (:250-273): live rows in slot order; labels/x may be null
  virtual void scan(int64_t *labels, float *x, int64_t *n) {
    (void)labels;
    (void)x;
    (void)n;
    throw Error(PYR_E_STATE, "index kind has no Scan (BruteForceVectorIndex only)");
  }
  // IVF kinds: the coarse ranking alone (probe lists [nq][min(nprobe, nlist)]) into d_out
  virtual int probe_only(const float *d_q, int64_t nq, int nprobe, int32_t *d_out, Workspace &ws) {
    (void)d_q;
    (void)nq;
    (void)nprobe;
    (void)d_out;
    (void)ws;
    throw Error(PYR_E_STATE, "index kind has no coarse quantizer");
  }
  // BruteForceVectorIndex.EnableQuantization (BruteForceVectorIndex.cs:25-40)
  virtual void set_quantization(bool on) {
    (void)on;
    throw Error(PYR_E_STATE, "index kind has no quantized search mode (BruteForceVectorIndex only)");
  }
  // IVectorIndex.Snapshot / Load (IVectorIndex.cs:26-27): the binary image of persist.h
  virtual void snapshot(const std::string &path) {
    (void)path;
    throw Error(PYR_E_STATE, "index kind has no snapshot");
  }
  virtual void load(const std::string &path) {
    (void)path;
    throw Error(PYR_E_STATE, "index kind has no snapshot");
  }
  virtual void set_centroids(const float *c, int nlist) {
    (void)c;
    (void)nlist;
    throw Error(PYR_E_STATE, "index kind has no coarse quantizer");
  }
  virtual void set_codebooks(const float *cb, int m, int ksub) {
    (void)cb;
    (void)m;
    (void)ksub;
    throw Error(PYR_E_STATE, "index kind has no product quantizer");
  }
  // ---- list-sharded multi-GPU search (IVF_FLAT; engine.cpp IvfFlatIndex, shard.hip) ----
  // the replicated sample of every list: rows [sum counts][dim] in list order, counts[l] <= 512 rows of list
  // l (its first rows), glen[l] its full length on the rank that owns it
  virtual void set_list_samples(const float *rows, const int64_t *counts, const int64_t *glen, int nlist) {
    (void)rows;
    (void)counts;
    (void)glen;
    (void)nlist;
    throw Error(PYR_E_STATE, "index kind has no list-sharded search (IVF_FLAT only)");
  }
  // home side: coarse ranking + T_q of nq queries -> plan [nq][shard_plan_stride(P, max_scans >= 0)]; returns P
  virtual int shard_prepare(const float *d_q, int64_t nq, int k, const pyr_search_params &p, int32_t *d_plan,
                            Workspace &ws) {
    (void)d_q, (void)nq, (void)k, (void)p, (void)d_plan, (void)ws;
    throw Error(PYR_E_STATE, "index kind has no list-sharded search (IVF_FLAT only)");
  }
  // every rank: its owned lists against the plans -> one record per query
  virtual void shard_search(const float *d_q, int64_t nq, int k, const int32_t *d_plan, int P, bool budget,
                            void *d_rec, Workspace &ws) {
    (void)d_q, (void)nq, (void)k, (void)d_plan, (void)P, (void)budget, (void)d_rec, (void)ws;
    throw Error(PYR_E_STATE, "index kind has no list-sharded search (IVF_FLAT only)");
  }
  // every rank: the exact re-run of the gathered failures [nranks][1 + fcap] -> records [nranks * fcap]
  virtual void shard_rerun(const float *d_q, int64_t nq, int k, const int32_t *d_plan, int P, bool budget,
                           const int32_t *d_fails, int nranks, int fcap, int64_t nq_home, void *d_rec, Workspace &ws) {
    (void)d_q, (void)nq, (void)k, (void)d_plan, (void)P, (void)budget, (void)d_fails, (void)nranks, (void)fcap;
    (void)nq_home;
    (void)d_rec, (void)ws;
    throw Error(PYR_E_STATE, "index kind has no list-sharded search (IVF_FLAT only)");
  }
  // ---- the multi-device index (multi.cpp; pyr_index_desc.device_mask / shards): a single-device IVF_FLAT index
  // (the "stage", on the first device) holds every row and builds exactly as the unsharded index does; its lists
  // are then dealt whole to the shard indexes, whose row labels are the stage's storage positions ----
  struct MsLists {
    int nlist = 0, nprobe_default = 0;
    std::vector<int32_t> lb, llen, llive;  // per list: first storage position, rows (incl. tombstones), live rows
    std::vector<uint8_t> state;            // per storage position: 1 visible, 0 removed / padding, 2 shadowed
    std::vector<float> cents;              // nlist x dim
  };
  virtual bool ms_lists(MsLists &out) const {  // false: not a built IVF_FLAT index
    (void)out;
    return false;
  }
  // row-major fp32 rows at the given list storage positions (device, this index's device), on st
  virtual void ms_gather_rows(const int64_t *d_pos, int64_t n, float *d_out, hipStream_t st) const {
    (void)d_pos, (void)n, (void)d_out, (void)st;
    throw Error(PYR_E_STATE, "index kind has no lists");
  }
  // a shard: lists of exactly these rows (device, row-major; row i in list asg[i], label labs[i]) in this order,
  // quantizer c (host, k x dim), replacing whatever the index held
  virtual void ms_commit(const float *d_x, int64_t n, const std::vector<int32_t> &asg, const std::vector<int64_t> &labs,
                         const float *c, int k) {
    (void)d_x, (void)n, (void)asg, (void)labs, (void)c, (void)k;
    throw Error(PYR_E_STATE, "index kind has no lists");
  }
  // every list's live rows over all shards (the MaxScans accounting of the list-sharded step), after a Delete
  virtual void ms_set_list_lengths(const int64_t *glen, int nl) {
    (void)glen, (void)nl;
    throw Error(PYR_E_STATE, "index kind has no list-sharded search");
  }
  virtual int64_t ms_position(int64_t label) const {  // the list storage position of a label (-1: none)
    (void)label;
    return -1;
  }
  // the list-sharded step answers this search (built, empty buffer, L2 / IP, k within the stream scan's refine);
  // else the stage searches alone; *P = the probe width
  virtual bool ms_shardable(int k, const pyr_search_params &p, int *P) const {
    (void)k, (void)p, (void)P;
    return false;
  }
  virtual const int64_t *ms_position_labels() const { return nullptr; }  // device: storage position -> label
  // pyr_index_shard_info: shards (1: a single-GPU index), transport (0 none, 1 device copies, 2 RCCL; set by the
  // first list-sharded search), searches answered by the list-sharded step / by the stage alone, and the last
  // step's largest failure count per home and its re-run rounds past the first
  virtual void shard_info(int32_t *shards, int32_t *xport, int64_t *sharded, int64_t *staged, int64_t *max_fail,
                          int64_t *rounds) const {
    *shards = 1;
    *xport = 0;
    *sharded = *staged = *max_fail = *rounds = 0;
  }

  // capacity hint: room for `rows` more rows without re-allocation (bulk loads of 10^7-10^8 rows,
  // where a grow-by-copy would need the old and the new store at once)
  virtual void reserve(int64_t rows) { (void)rows; }

  std::unique_ptr<Workspace> take_ws();
  void give_ws(std::unique_ptr<Workspace> w);
  Workspace &ws_for_stream(hipStream_t st);
};

struct NetRandom {  // System.Random legacy (Net5CompatSeedImpl); SURVEY.md Appendix A
  int32_t sa[56];
  int32_t inext = 0, inextp = 21;
  explicit NetRandom(int32_t seed) {
    const int32_t MBIG = INT32_MAX;
    int32_t sub = seed == INT32_MIN ? INT32_MAX : (seed < 0 ? -seed : seed);
    int32_t mj = 161803398 - sub, mk = 1;
    sa[55] = mj;
    for (int i = 1; i < 55; i++) {
      int ii = (21 * i) % 55;
      sa[ii] = mk;
      mk = mj - mk;
      if (mk < 0) mk += MBIG;
      mj = sa[ii];
    }
    for (int p = 1; p < 5; p++)
      for (int i = 1; i < 56; i++) {
        sa[i] -= sa[1 + (i + 30) % 55];
        if (sa[i] < 0) sa[i] += MBIG;
      }
  }
  int32_t next() {
    if (++inext >= 56) inext = 1;
    if (++inextp >= 56) inextp = 1;
    int32_t r = sa[inext] - sa[inextp];
    if (r == INT32_MAX) r--;
    if (r < 0) r += INT32_MAX;
    sa[inext] = r;
    return r;
  }
  double next_double() { return next() * (1.0 / INT32_MAX); }
};

Index *create_index(const pyr_index_desc &d);
// a device mask left by pyr_index_create (several devices, or shards >= 1): the list-sharded index (multi.cpp)
Index *create_multi_index(const pyr_index_desc &d);
bool filter_k1_ok(int k);  // the stream scan's refine takes this k (k <= 60)

// kernel-phase profiler (pyr_profile_*): HIP events around each phase on the search stream
enum Phase { PH_COARSE = 0, PH_ITEMS = 1, PH_LIST_SCAN = 2, PH_BUF_SCAN = 3, PH_MERGE = 4, PH_FLAT_SCAN = 5,
             PH_PQ_SCAN = 6, PH_REFINE = 7, PH_FALLBACK = 8, PH_SAMPLE = 9, PH_N = 10 };
struct Profiler {
  bool on = false;
  std::mutex m;
  double ms[PH_N] = {0};
  int64_t calls[PH_N] = {0}, work[PH_N] = {0};
  struct Rec {
    int phase;
    hipEvent_t a, b;
    int64_t work;
  };
  std::vector<Rec> pending;
  void drain();
  void reset();
};
Profiler &prof();
struct PhaseTimer {
  int phase;
  hipStream_t st;
  hipEvent_t a = nullptr;
  int64_t work;
  PhaseTimer(int ph, hipStream_t s, int64_t w = 0);
  ~PhaseTimer();
};

// shared building blocks
void fill_empty_results(float *d_s, int64_t *d_l, int32_t *d_c, int64_t nq, int k, hipStream_t st);
// KMeansUtils.Train on the GPU: reference-identical init and Lloyd iterations.
int kmeans_train_gpu(const float *d_x, int64_t n, int dim, int k, int metric, int max_iter, int seed,
                     float *d_cents /* k x dim */, hipStream_t st);
// KMeansUtils.FindNearestCentroid for every row (ties -> lowest index)
void assign_gpu(const float *d_x, int64_t n, int dim, const float *d_cents, int k, int metric, int32_t *d_assign,
                hipStream_t st);

}  // namespace pyr
