// kernels.h -- host-side launchers for the gfx950 kernels in kernels.hip.
// Internal to libpyrope_hip.so (the public boundary is include/pyrope_ann.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdint.h>

#include <atomic>

namespace pyr {

// Raise a kernel's dynamic-LDS limit to the whole 160 KiB of a CU.  The attribute is per
// device, so it is set once per (kernel, device ordinal) -- `done` is the kernel's bit mask of
// devices -- and the bit is published only after the call, so a thread that sees it set (any
// thread, any index on any device) launches with the attribute in place.
inline void allow_max_lds(const void *fn, std::atomic<uint64_t> &done, int bytes = 160 * 1024) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t bit = uint64_t(1) << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done.fetch_or(bit, std::memory_order_acq_rel);
}

// Measurement and test switches (the PYR_* variables of DESIGN.md §7): honoured only when the process starts
// with PYR_DEV_KNOBS=1 (read once, at the first switch read).  A production host's environment cannot steer
// the search paths; tests/conftest.py and the A/B scripts set it.
inline const char *knob(const char *name) {
  static const bool on = [] {
    const char *e = std::getenv("PYR_DEV_KNOBS");
    return e && std::atoi(e) == 1;
  }();
  return on ? std::getenv(name) : nullptr;
}

enum Metric { L2 = 0, IP = 1, COS = 2 };

constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;
constexpr uint32_t KEY_BUF = 0x80000000u;  // buffer rows: KEY_BUF | slot (DESIGN.md "Tie rule")
// a candidate-list placeholder of the stream scans (stream16.hip, scan.hip): a score that bounds rows a
// region dropped; the merge ranks it like a row, the refine certifies against it and never re-scores it
constexpr uint32_t KEY_FLOOR = 0xFFFFFFFEu;
constexpr int QCHUNK = 128;                // queries per scan work item (fast kernel)
constexpr int QCHUNK_GENERIC = 64;         // queries per scan work item (generic kernel)
constexpr int KMAX_FAST = 64;              // largest k served by the fast kernel
constexpr int KMAX = 256;                  // largest k served at all
constexpr int MAX_PARTS = 1024;            // partial lists merged per query

// A scan work item: rows [row_begin, row_end) of a blocked row store against up to
// QCHUNK queries.  If the launch has a qlist, the queries' partial slots are
// qlist[qbeg .. qbeg+qcnt) + part (IVF: part = row chunk of the list); otherwise
// query = qbeg + i and slot = query * nparts + part.
// blocks of 256 threads for a grid-stride element loop over n items: capped at 2^22 blocks, since a
// dispatch's grid is a 32-bit work-item count (n x dim of 10^8 rows is far past it)
inline unsigned gblk(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < (int64_t(1) << 22) ? b : (int64_t(1) << 22));
}

struct ScanItem {
  int32_t row_begin;  // multiple of 8
  int32_t row_end;
  int32_t qbeg;
  int32_t qcnt;
  int32_t part;
  int32_t list;  // IVF: list id of the item
};

// IVF row chunking.  List l is split into chunk 0 = its first `warm` rows (if warm > 0)
// and then chunks of at most `chunk` rows; (query, probe p, chunk c) owns partial slot
// q * nparts + p * cmax + c.  The chunk-0 items run as a separate, earlier launch: they
// publish every query's shared bound (ScanArgs::gthr) before the main launch starts,
// so the main items skip almost every row without a top-k insertion.  Chunking also
// keeps work items uniform whatever the list-size skew.  warm, chunk: multiples of 8.
struct IvfChunking {
  int32_t chunk;  // rows per main chunk
  int32_t cmax;   // max chunks of any list (slots reserved per probe)
  int32_t warm;   // rows of chunk 0 (0 = no warm-up chunk)
  int32_t skip_empty = 0;  // an empty list gets no item (the stream scans: a list-sharded rank's lists it
                           // does not own are empty, and their (query, list) pairs must cost nothing)
  int32_t xcd = 0;         // items in 8 per-XCD queues (lists l with l % 8 == x, in list order), their
                           // bounds at n_items[1 .. 9] (pq32.hip: one list's items on one XCD)
};
__host__ __device__ inline int ivf_list_chunks(int len, IvfChunking ch) {
  if (len <= 0 && ch.skip_empty) return 0;
  if (ch.warm > 0) return len <= ch.warm ? 1 : 1 + (len - ch.warm + ch.chunk - 1) / ch.chunk;
  return len <= 0 ? 1 : (len + ch.chunk - 1) / ch.chunk;  // an empty list still gets one (empty) item
}
// rows [*b, *e) (relative to the list start) of chunk c
__host__ __device__ inline void ivf_chunk_rows(int len, int c, IvfChunking ch, int *b, int *e) {
  int s = ch.warm > 0 ? (c == 0 ? 0 : ch.warm + (c - 1) * ch.chunk) : c * ch.chunk;
  int t = ch.warm > 0 && c == 0 ? ch.warm : s + ch.chunk;
  *b = s < len ? s : len;
  *e = t < len ? t : len;
}

struct ScanArgs {
  const float *rows;      // blocked [row/8][D][8]
  const uint8_t *live;    // per row, 1 = visible
  const float *rnorm;     // per row norms (cosine) or null
  const float *queries;   // row-major nq x D (generic kernel)
  const float *queries_t; // lane-major nq x D (fast kernel; launch_transpose_queries)
  const float *qnorm;     // per query norms (cosine) or null
  const ScanItem *items;
  const int32_t *n_items; // device count (items beyond it exit)
  const int32_t *qlist;   // partial-slot ids or null
  const uint32_t *limits; // per partial slot exclusive row bound (max_scans), or null
  int32_t nparts;         // partial slots per query
  int32_t k;
  uint32_t key_base;      // OR-ed into row index to form the storage key
  int32_t dim;
  float *part_s;          // [slot][k] scores
  uint32_t *part_k;       // [slot][k] keys
  // Per-query running bound shared by every item of one search (null = off): the
  // order-preserving uint32 encoding (score_key) of a score that some k rows of that
  // query already reach.  A row strictly below it can never enter the final top-k,
  // so items skip it; owners raise it with atomicMax as their lists fill.
  uint32_t *gthr;
};

// order-preserving float <-> uint32 map (a < b  <=>  score_key(a) < score_key(b))
__host__ __device__ inline uint32_t score_key(float f) {
  union {
    float f;
    uint32_t u;
  } v{f};
  return (v.u & 0x80000000u) ? ~v.u : (v.u | 0x80000000u);
}
__host__ __device__ inline float key_score(uint32_t k) {
  union {
    uint32_t u;
    float f;
  } v{(k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k};
  return v.f;
}

// int64 labels (centroid ids, -1 = none) -> int32 probe ids
void launch_labels_to_i32(const int64_t *in, int64_t n, int32_t *out, hipStream_t st);

// V = 1: VectorMath safe functions (one Vector accumulator; IVF paths, k-means).
// V = 4: VectorMath *Unsafe functions (four accumulators; BruteForce head).
void launch_scan(const ScanArgs &a, int metric, int V, int max_items, hipStream_t st);

// FLAT-style items: rows [0, nrows) in chunks of chunk_rows x queries [0,nq) in QCHUNK blocks.
// Returns item count (also written to *d_nitems).
int make_flat_items(ScanItem *d_items, int32_t *d_nitems, int64_t nrows, int32_t chunk_rows, int64_t nq,
                    int32_t part_off, int32_t qchunk, hipStream_t st);

// fast-scan query layout: qt[q][l][t] = q[q][8t + l]
void launch_transpose_queries(const float *q, int64_t nq, int32_t dim, float *qt, hipStream_t st);

// Per-row / per-query norms (VectorMath.ComputeNorm).  blocked != 0: rows in blocked layout.
void launch_norms(const float *x, int64_t n, int32_t dim, int blocked, float *out, hipStream_t st);

// Merge nparts sorted partial lists per query into top-k.
// keys are uint32 storage keys; labels mapped through row_labels / buf_labels when given.
// With `ivf` set, parts [0, nprobe*cmax) are IVF chunk slots and slot p*cmax + c is read
// only if list probes[q][p] has more than c chunks (unwritten slots are never read).
struct MergeIvf {
  const int32_t *probes = nullptr;  // [nq][nprobe]
  const int32_t *lb = nullptr, *le = nullptr;
  int32_t nprobe = 0;
  IvfChunking ch{8, 1, 0};
};
// Exact IVF re-run of the queries whose certificate failed, on the device: the fail list and its
// count stay in HBM (no host round trip).  One block per (failing query, probed list), persistent over
// them: the exact ComputeScore (safe VectorMath form) of every live row, the list's top k (<= 64) by
// (score desc, storage slot asc); then one wave per failing query merges its lists and writes out_* at
// the query's row.
struct IvfRerunArgs {
  const float *rows;        // blocked list store
  const uint8_t *live;
  const int64_t *labels;
  const float *queries;     // row-major, the batch
  const int32_t *probes;    // [nq][nprobe]
  int32_t nprobe;
  const int32_t *lb, *le;   // device list bounds
  const int32_t *fail, *nfail;
  int32_t dim, k;
  int32_t nchunk;           // most chunks a probed list is cut into (>= 1; few failures use them all)
  int32_t v4;               // 1: the *Unsafe forms (BruteForceVectorIndex, V = 4: FLAT chunks as lists)
  const float *qnorm;       // Cosine: ComputeNorm per query and per row
  const float *rnorm;
  float *out_s;
  int64_t *out_l;
  int32_t *out_c;
  int32_t pstride;          // row stride of probes (0: nprobe; a shard plan's P + 1)
  // list-sharded search (shard.hip): failing query i's answer goes to record rec_pos[i] of rec (ShardEntry
  // x k + ShardTrailer, bound -inf: exact) instead of out_* at its row; rec_lb / rec_nlist: the list
  // bounds that name each row's list
  void *rec;
  const int32_t *rec_pos;
  const int32_t *rec_lb;
  int32_t rec_nlist;
  // or null: per failing query the units done (zero before the launch; every merge resets its own); the block
  // that finishes a query's last unit merges it, and the separate merge launch is skipped
  int32_t *done;
  // MaxScans, or null: [q][nprobe] the exclusive absolute row bound of each probed list (ivf_limits_kernel with
  // one chunk per probe)
  const uint32_t *qlim;
};
// part: ivf_rerun_part_keys() rank keys of scratch (one block per (failing query, probe, chunk), then
// a merge per query)
int64_t ivf_rerun_part_keys(int64_t max_fail, int nprobe, int k);
void launch_ivf_exact_rerun(const IvfRerunArgs &a, int metric, int64_t max_fail, uint64_t *part, hipStream_t st);

void launch_merge_keys(const float *ps, const uint32_t *pk, int64_t nq, int32_t nparts, int32_t k,
                       const int64_t *row_labels, const int64_t *buf_labels, float *out_s, int64_t *out_l,
                       int32_t *out_keys, int32_t *out_cnt, hipStream_t st, const MergeIvf *ivf = nullptr);
// Two per-query result sets (each sorted, ca / cb real entries) into the top k, a before b on equal scores
// (IVF_PQ / IVF_FLAT: the lists' certified answer and the buffer's exact one; k <= 256; the outputs distinct
// from both inputs).
void launch_merge_two(const float *as, const int64_t *al, const int32_t *ca, const float *bs, const int64_t *bl,
                      const int32_t *cb, int64_t nq, int k, float *out_s, int64_t *out_l, int32_t *out_c,
                      hipStream_t st);
// Merge partial lists that carry int64 labels (multi-GPU), ties by label asc.
void launch_merge_labels(const float *ps, const int64_t *pl, int64_t nq, int32_t nparts, int32_t k, float *out_s,
                         int64_t *out_l, hipStream_t st, bool part_major = false);

// IVF: from probes [nq][nprobe] build list-major work items.
struct IvfItemWs {
  int32_t *cnt;       // nlist
  int32_t *fill;      // nlist
  int32_t *qoff;      // nlist + 1
  int32_t *ioff;      // nlist + 1
  int32_t *qlist;     // nq * nprobe
  ScanItem *items;    // max_items
  int32_t *n_items;   // 1
  int32_t *qpos = nullptr;  // or [nq][nprobe]: the qlist position of (query, probe) (all probes only)
};
// Item list of one launch phase: phase 0 = chunk 0 of every list (all chunks when
// ch.warm == 0), phase 1 = chunks >= 1 (only with ch.warm > 0).  Phase 0 also builds
// the per-list query lists (ws.cnt/qoff/qlist) that phase 1 reuses.
int64_t ivf_max_items(int64_t nq, int32_t nprobe, int32_t nlist, int32_t qchunk, IvfChunking ch, int phase);
// [pb, pe): the probe ranks taken (pe < 0: all); partial slots keep the absolute rank.
void launch_ivf_items(const int32_t *probes, int64_t nq, int32_t nprobe, int32_t nparts, int32_t nlist,
                      const int32_t *list_begin, const int32_t *list_end, int32_t qchunk, IvfChunking ch,
                      int phase, IvfItemWs &ws, hipStream_t st, int32_t pb = 0, int32_t pe = -1,
                      bool balance = false,   // balance: a list's query groups of equal size (multiples of 16)
                      bool zeroed = false);   // zeroed: ws.cnt / ws.fill already zero (the caller's WordFill)
// IVF max_scans limits per (query, probe, chunk) slot (IvfFlatVectorIndex.cs:200-212)
void launch_ivf_limits(const int32_t *probes, int64_t nq, int32_t nprobe, int32_t nparts, int64_t remaining,
                       const int32_t *list_begin, const int32_t *list_end, const int32_t *list_live,
                       const uint8_t *live, IvfChunking ch, uint32_t *limits, hipStream_t st,
                       const int32_t *prem = nullptr, int rstride = 0);

// the per-(query, probe) bounds (cmax 1) at the pairs' qlist positions: plim[qpos[i]] = limits[i]
void launch_pos_limits(const int32_t *qpos, const uint32_t *limits, int64_t n, uint32_t *plim, hipStream_t st);

// IVF-PQ ADC scan (IvfPqVectorIndex.cs:152-198).
struct PqArgs {
  const uint8_t *codes;    // blocked codes, see kernels.hip
  const uint8_t *live;
  const float *queries;    // nq x D
  const float *cents;      // nlist x D row-major
  const float *codebooks;  // [M][ksub][sub]
  const int32_t *probes;   // [nq][nprobe]
  const int32_t *list_begin, *list_end;
  const ScanItem *items;
  const int32_t *n_items;
  const int32_t *qlist;
  int32_t nparts, nprobe, k, dim, M, ksub;
  float *part_s;
  uint32_t *part_k;
  uint32_t *gthr;          // shared per-query bounds (ScanArgs::gthr) or null; pq_adc only
  int32_t ablate;          // measurement only (PYR_PQ_ABLATE): 1 LUT once per item, 2 no top-k
};
void launch_pq_scan(const PqArgs &a, int max_items, hipStream_t st);
// four queries per LDS gather (float4 LUT entries, 8-subspace double-buffered LUT passes);
// items of at most pq_adc4_rows() rows (IvfChunking chunk), k <= 64, ksub <= 256
bool pq_adc4_supported(int dim, int M, int ksub, int k);
int pq_adc4_rows();
void launch_pq_adc4(const PqArgs &a, int max_items, hipStream_t st);
size_t pq_scan_lds_bytes(int dim, int M, int ksub, int k);
// PQ encode (ProductQuantizer.Encode on residuals x - c[assign]) -> codes n x M row-major.
void launch_pq_encode(const float *x, const int32_t *assign, const float *cents, int64_t n, int32_t dim, int32_t M,
                      int32_t ksub, const float *codebooks, uint8_t *codes, hipStream_t st);
// residuals r = x - c[assign] (IvfPqVectorIndex.cs:82-84)
void launch_residuals(const float *x, const int32_t *assign, const float *cents, int64_t n, int32_t dim, float *out,
                      hipStream_t st);
// sub-vector extraction for per-subspace k-means (ProductQuantizer.cs:39-45)
void launch_extract_sub(const float *x, int64_t n, int32_t dim, int32_t off, int32_t sub, float *out, hipStream_t st);
// codes (row-major n x M, rows in perm order) -> blocked list storage
void launch_pack_codes(const uint8_t *codes, const int64_t *src_of_dst, int64_t ndst, int32_t M, uint8_t *out,
                       hipStream_t st);

// ---- IVF coarse step as dense scores + selection (coarse.hip) ----
bool coarse_dense_supported(int nlist);
// probes [nq][nprobe] = the first nprobe centroids by (ComputeScore desc, index asc);
// scores: nq x nlist scratch.  qn / cn: query / centroid norms (cosine only).
void launch_coarse_dense(const float *q, const float *cents_rm, const float *qn, const float *cn, int64_t nq,
                         int32_t nlist, int32_t dim, int32_t metric, int32_t nprobe, float *scores, int32_t *probes,
                         hipStream_t st);

// The same ranking with the scores on the matrix cores (L2 / IP, dim % 16 == 0, nprobe <= 64): fp32 MFMA
// approximate scores, aP = the nprobe-th largest of them, the exact ComputeScore of every centroid whose
// approximate score reaches aP - 2E (E bounds the approximation) and the top nprobe of those; a query
// with more than 64 such centroids gets the dense exact ranking.  c2: |c|^2 per centroid; cnmax >=
// max |c|; c_err: the error-bound constant.  scores: nq x nlist scratch, fail: nq, nfail: 1 (device
// scratch).  Nothing synchronizes.
bool coarse_mfma_supported(int nlist, int dim, int metric, int nprobe);
// zero: words to fill by the approximate-score launch (the search's counters; no launch of their own)
struct WordFill;
// split: the centroids split into bf16 hi / lo planes in MFMA fragment order (launch_coarse_split, once per
// quantizer; coarse_split_bytes of device memory): the approximate scores then run on the bf16 matrix cores
// (three products per k-step; c_err widened by the split's bound inside); nullptr: the fp32 MFMA kernels
void launch_coarse_mfma(const float *q, const float *cents_rm, const float *c2, int64_t nq, int32_t nlist,
                        int32_t dim, int32_t metric, int32_t nprobe, double cnmax, double c_err, float *scores,
                        int32_t *fail, int32_t *nfail, int32_t *probes, hipStream_t st,
                        const WordFill *zero = nullptr, const void *split = nullptr);
size_t coarse_split_bytes(int nlist, int dim);
int coarse_bf3_max_dim();  // the split kernel's dimension limit (larger: the fp32 kernels)
void launch_coarse_split(const float *cents_rm, int nlist, int dim, void *split, hipStream_t st);

// ---- 8-bit search mode of the FLAT index (sq8.hip; BruteForceVectorIndex EnableQuantization) ----
struct Sq8Args {
  const uint8_t *codes;    // [slot][dp] ScalarQuantizer codes - 128 (int8), zero padded
  const int2 *sums;        // [slot] {sum of codes, sum of squared codes}
  const uint8_t *live;     // [slot]
  const uint8_t *ok;       // [slot] 1 = has codes (written while quantization was on)
  const uint8_t *qcodes;   // [q][dp], as codes
  const int2 *qsums;       // [q]
  const ScanItem *items;   // make_flat_items, qchunk = sq8_qgroup()
  const int32_t *n_items;
  int32_t nparts, k, dim, dp;
  uint32_t row_limit;      // rows >= row_limit are not scanned (MaxScans cutoff)
  float *part_s;           // [q * nparts + part][k]
  uint32_t *part_k;
};
int sq8_dp(int dim);       // code row stride (dim rounded up to 32)
int sq8_qgroup();          // queries per scan item
bool sq8_supported(int dim, int k);
// ScalarQuantizer.Quantize of n vectors: blocked != 0 -> rows of a blocked store at slots[i]
// (codes written at slot), else row-major src with codes at i.  shifted: store code - 128
// (the scan's int8 operands).  ok (may be null) set to 1.
void launch_sq8_quantize(const float *src, const int64_t *slots, int blocked, int64_t n, int32_t dim, int32_t dp,
                         int shifted, uint8_t *codes, int2 *sums, uint8_t *ok, hipStream_t st,
                         float2 *minmax = nullptr);  // minmax[i]: Quantize's out min / max (may be null)
// ScalarQuantizer.Dequantize (ScalarQuantizer.cs:65-84) of n code rows (n x dim) -> out (n x dim)
void launch_sq8_dequantize(const uint8_t *codes, int64_t n, int32_t dim, const float *mins, const float *maxs,
                           float *out, hipStream_t st);
void launch_sq8_scan(const Sq8Args &a, int metric, int max_items, hipStream_t st);

// ---- fp16 tiles (tiles16.hip) + the certified exact refine (filter.hip) ----
constexpr int FILTER_F16X1 = 3;   // the stream scan's arithmetic: fp16 row tiles x one-term fp16 queries
// refine_kernel constants of the fp16 tiles: relative c_bf (per u |q| max|x|) and the absolute term
// (per |q|) from fp16 subnormals of the rows, 2^-25 sqrt(D) / sx; doubled for L2.  x's fp16 rounding is
// 2^-11 = 8192 u relative; 4 u of slack (rounds 1-3's two-term query split); fp32 accumulation of 2D
// exact products <= 2D u; the one-term queries add q's own 2^-11 (+ 64).
inline double filter_f16_cerr(int dim, int metric, int prec) {
  const double c = 8192.0 + 4.0 + 2.0 * dim + 64.0 + (prec == FILTER_F16X1 ? 8192.0 + 64.0 : 0.0);
  return metric == 0 ? 2.0 * c : c;
}
inline double filter_f16_abs(int dim, int metric, float sx, int prec) {
  const double a = 2.9802322387695312e-08 * __builtin_sqrt((double)dim) / (double)sx;  // 2^-25 sqrt(D) / sx
  // one-term queries: q's own subnormal halves (|q_i| sq < 2^-14) add 2^-25 / sq per |x_i|, bounded
  // through |x| <= X in refine (q_abs there)
  (void)prec;
  return metric == 0 ? 2.0 * a : a;
}
// ---- the IVF / FLAT list scan as stream-and-emit (scan.hip; sample and merge: sample16.hip) ----
constexpr int STREAM_KO = 64;  // merged candidates per query (the deep certificate's K1)
struct StreamArgs {
  const void *h16;            // fp16 residual tiles of the lists (RowStore::h16)
  const float *meta;          // per row: L2 -|x - c|^2, IP 0, -inf dead / padding
  const float *queries;       // row-major nq x D
  const float *cents;         // row-major centroids
  const int32_t *probes;      // [q][nprobe] probe lists (pq32 prep: a position's list)
  float sx;                   // the store's power-of-two fp16 scale
  const ScanItem *items;
  const int32_t *n_items;
  const int32_t *qlist;       // per (list, query) position: q * nparts + probe * cmax
  int32_t nparts, nprobe, cmax, dim;
  int32_t dt;                 // tile dimension D (scan_tile_dim; 0: dim): tiles and bq rows; queries / cents keep dim
  _Float16 *bq;               // [pos][D] scaled query residuals (one fp16 term)
  float2 *qsc;                // [pos] {f, cq}
  float *samp;                // [q * nprobe + probe][scan_sample_values()] sampled scores
  const float *thr;           // [q] T_q (score space), or null
  // the emitted rows, query-major: query q's rows at cand[q * cap + i] = {score bits, key}, i < cand_n[q]
  // (reserved with one atomic per (item, query); past cap a row only raises the floor cand_f[q] =
  // score_key of the best row dropped, 0: none)
  uint2 *cand;
  int32_t *cand_n;
  uint32_t *cand_f;
  int32_t cap;
  int32_t *work;              // persistent-block item counter (zeroed before each launch)
  uint32_t key_base, row_limit;
  int32_t ablate;             // measurement only (PYR_FILTER_ABLATE=64: no emission)
  float thr_bias;             // measurement only (PYR_STREAM_THR_BIAS: added to T_q; results then differ)
  // Upper-bound scores (stream_ub_terms): every emitted / sampled score is approx + E_row + E_pair,
  // an upper bound of the reference's score of that row.  E_row = kr |x - c|^2 (+ kx |x|^2, IP) per
  // row, E_pair = kq A^2 + kqa A (+ kqc |q| |c|, IP) per (query, list), A = |q - c| (L2) / |q| (IP).
  const float *rsq16;         // per row |x - c|^2
  const float *rsq;           // per row |x|^2 (IP)
  float kr, kx, kq, kqa, kqc;
  const float *mub;           // per row meta + E_row (RowStore::row_terms)
  unsigned long long *tdbg;   // measurement only (PYR_STREAM_TIMING=1): per-wave cycle buckets, or null
  // [q][nprobe] the qlist position of (query, probe), every probe of every query (IvfItemWs::qpos), or null:
  // then sprep builds the operands query-major (sample16.hip); nq its query count
  const int32_t *qpos;
  int64_t nq;
  // MaxScans (IvfFlatVectorIndex.cs:202-212), or null: per qlist position the exclusive absolute row bound of
  // that (query, list) pair's scanned rows (launch_pos_limits); a row at or past it is neither sampled nor
  // emitted
  const uint32_t *plim;
  // the sample pass by list (scan.hip SMP), or null (then every item is drawn and non-chunk-0 ones skipped):
  // list l's chunk-0 items are lioff[l] .. lioff[l] + ceil(lcnt[l] / lqchunk) - 1 (ivf_list_items' order)
  const int32_t *lioff, *lcnt;
  int32_t nlist, lqchunk;
};
// per row the stream scan's additive term: meta + kr |x - c|^2 (+ kx |x|^2, IP): fmaf(kr, rsq16, meta),
// then fmaf(kx, rsq, .)
void launch_row_terms(const float *meta, const float *rsq16, const float *rsq, int64_t n, int metric, float kr,
                      float kx, float *out, hipStream_t st);
// The per-row / per-pair split of the fp16 residual tiles' error bound (refine_kernel's resid branch,
// filter.hip): products A X go to (A^2 + X^2) / 2, (A + X)^2 to 2 (A^2 + X^2), so the bound of a row
// no longer depends on its list's largest residual; the reference's own sum deviation (g) is folded in.
void stream_ub_terms(int dim, int metric, double c_bf, double c_err, double c_abs, StreamArgs &a);
// ---- IVF_PQ on the matrix cores (pq32.hip): the stream pipeline of the IVF_FLAT scan over rows decoded
// from their codes; D a multiple of 16 up to 1152, dsub 4 / 8 / 16 / 32 ----
bool pq32_supported(int dim, int M, int ksub, int k);
int pq32_qmax(int dim, int M);      // queries per item
int pq32_sample_values();           // sample values per (query, probe)
int pq32_lane_words(int dim, int M);  // 16-byte code words per lane per 32-row tile (cpack: 64 lanes of them)
// codes (row-major, source rows) -> the tile layout cpack [tile][64 lanes][lane words][16 B] of the list-major
// positions (src: position -> source row or -1; pq32.hip pq_pack_kernel) and |x^|^2 per position (fp32
// codebooks [M][ksub][dsub])
void launch_pq32_pack(const uint8_t *codes_rm, const int64_t *src, int64_t tot, int M, int dsub, const float *cb,
                      int ksub, uint8_t *cpack, float *nrm, hipStream_t st);
void launch_pq32_cb16(const float *cb, int M, int ksub, int dsub, float sc, _Float16 *cb16, hipStream_t st);
void launch_pq32_meta(const float *nrm, const uint8_t *live, int64_t tot, float *meta, hipStream_t st);
// StreamArgs as for the IVF_FLAT stream scan, with h16 = cpack, mub = the row terms, cents = coarse
// centroids, probes = the probe lists, sx = the codebook scale; items in XCD order (IvfChunking::xcd) and
// work = 8 per-XCD queue counters
void launch_pq32_prep(const StreamArgs &a, int64_t npos, hipStream_t st);
void launch_pq32_scan(const StreamArgs &a, const _Float16 *cb16, int M, int max_items, bool sample, hipStream_t st);
struct PqRefineArgs {
  const float *queries;     // nq x D
  const float *cents;       // coarse centroids, row-major
  const float *codebooks;   // fp32 [M][ksub][dsub]
  const uint8_t *cpack;     // tile code layout
  const int64_t *labels;    // per position
  const int32_t *lb;        // list starts (positions)
  const float *ms;          // merged candidate bounds [nq][ld]
  const int32_t *mk;        // their positions (-2 floor, -1 none)
  const int32_t *qsel, *nsel;  // refine only these queries (null: all nq)
  int64_t nq;
  int32_t ld, k1, k, dim, M, ksub, lw, dsub, nlist;
  float *out_s;
  int64_t *out_l;
  int32_t *out_c;
  int32_t *fail_list, *fail_cnt;
};
void launch_pq32_refine(const PqRefineArgs &a, int64_t nq, hipStream_t st);
// ---- list-sharded multi-GPU search (shard.hip; pyrope_amd/dist.py ListShardedIvf) ----
// One query's answer from one rank: k entries in (score desc, list asc, label asc) order (unused: label -1,
// score -inf), then the trailer: every row of the rank's probed lists that is not an entry scores at most
// `bound` (-inf: none was left out), n = the real entries.
struct ShardEntry {
  int64_t label;
  float score;
  int32_t list;
};
struct ShardTrailer {
  float bound;
  int32_t n;
  int64_t pad;
};
__host__ __device__ inline int64_t shard_record_bytes(int k) { return 16 * (int64_t)(k + 1); }
// the list of storage slot `key`: the last list whose start is <= key (lists laid out by id, an empty list
// shares its start with the next one)
__device__ __forceinline__ int32_t shard_list_of(const int32_t *lb, int nlist, uint32_t key) {
  int lo = 0, hi = nlist - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((uint32_t)lb[mid] <= key) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
struct ShardMergeArgs {
  const uint8_t *rec;       // [nparts][nrec] records (part-major: an all_to_all's output)
  int32_t nparts;           // 1 .. 64
  int64_t nrec;             // records per part
  int32_t k;
  const int32_t *qsel;      // null: record i answers query i; else record i answers qsel[1 + i], i < min(qsel[0], cap)
  int32_t cap;
  float *out_s;             // [nq][k]
  int64_t *out_l;
  int32_t *out_c;           // may be null
  int32_t *fail;            // null: no certificate; else fail[0] = failures (may exceed fcap), fail[1 ..] queries
  int32_t fcap;
};
void launch_shard_merge(const ShardMergeArgs &a, int64_t max_rec, hipStream_t st);
// plan [nq][P + 1] <-> probes [nq][P] + T_q [nq]
// plan rows [P probes][T_q bits][P remaining budgets, with a MaxScans budget only]: shard_plan_stride(P, budget)
inline int shard_plan_stride(int P, bool budget) { return P + 1 + (budget ? P : 0); }
void launch_pack_plan(const int32_t *probes, const float *thr, const int32_t *rem, int64_t nq, int P, int32_t *plan,
                      hipStream_t st);
void launch_unpack_plan(const int32_t *plan, int64_t nq, int P, int stride, int32_t *probes, float *thr, hipStream_t st);
// the home rank's MaxScans accounting (IvfFlatVectorIndex.cs:202-212) over every rank's lists: per (query, probe)
// the budget left when the probe's list is reached, rem[q][p] = max(0, max_scans - sum of the live lengths of
// the lists probed before it) (glive: every list's live rows, replicated), and the absolute row bound of the pair
// in the replicated sample store (slb / sle: its lists' sample rows; a sample holds no tombstones)
void launch_shard_budget(const int32_t *probes, int64_t nq, int P, int64_t max_scans, const int32_t *glive,
                         const int32_t *slb, const int32_t *sle, int32_t *rem, uint32_t *slimits, hipStream_t st);
// l[i] = table[l[i]] where l[i] >= 0 (the multi-device index: shard labels are stage storage positions)
void launch_map_positions(int64_t *l, int64_t n, const int64_t *table, hipStream_t st);
// out [W][1 + fcap] = entries [off, off + fcap) of every home's whole fail list full [W][stride] (the count first)
void launch_fail_round(const int32_t *full, int W, int64_t stride, int off, int fcap, int32_t *out, hipStream_t st);
// gathered fail lists [nranks][1 + fcap] -> global failing queries fail[], their record slots pos[], *nfail
void launch_shard_fail_compact(const int32_t *fails, int nranks, int fcap, int64_t nq_home, int32_t *fail, int32_t *pos,
                               int32_t *nfail, hipStream_t st);

struct CandMergeArgs {
  const uint2 *cand;          // StreamArgs::cand / cand_n / cand_f
  const int32_t *cand_n;
  const uint32_t *cand_f;
  const float *thr;
  int64_t nq;
  int32_t cap;
  float *out_s;               // [nq][STREAM_KO] desc; floor placeholders key -2, none -1
  int32_t *out_k;
};
// pq32.hip, k > 60: the merge + certified refine of the emitted rows at depth a.k1 (128 / 256 / 512), one
// block per query
void launch_pq32_deep_refine(const CandMergeArgs &m, const PqRefineArgs &a, hipStream_t st);
int device_cus();                   // compute units of the current device (persistent-grid launches)
// scan.hip: the one-wave-per-32-queries sample (query operands + sample values, any tile dimension) and
// the 32x32x16 list scan; sample16.hip: sprep + the 8-wave sample of tile dims 32 / 64 / 128 (same
// outputs: bq, qsc, samp with scan_sample_values() values per (query, probe))
int scan_sample_values();
// tile dimension of the stream scan for a row dimension: dims <= 128 rounded up to 32, then 256 / 512 / 768
// (tiles and query operands zero-padded; the fp32 rows and the exact refine keep dim); 0 = none
int scan_tile_dim(int dim);
int scan_qmax(int dt);               // queries per work item at tile dimension dt
bool scan_supported(int dim, int metric, int k1);
// FLAT chunks as lists: lb/le of nch chunks of crow rows over [0, cutoff), each with the centroid center
// (null: 0) -> cents [nch][dim]
void launch_chunk_lists(int32_t *lb, int32_t *le, int nch, int64_t crow, int64_t cutoff, const float *center,
                        int dim, float *cents, hipStream_t st);
// out[i][c] = c for i < rows, c < cols
void launch_iota_rows(int32_t *out, int64_t rows, int cols, hipStream_t st);
void launch_scan_sample(const StreamArgs &a, int metric, int max_items, hipStream_t st);
void launch_scan_main(const StreamArgs &a, int metric, int max_items, hipStream_t st);
// the sample pass on the main scan kernel (scan.hip, SMP): same samp layout and count as sample16 (bq / qsc
// prepared beforehand); tile dims whose blocks have SAMPLE_TILES waves
bool scan_sample_mode_supported(int dt);
void launch_scan_sample_mode(const StreamArgs &a, int metric, int max_items, hipStream_t st);
bool sample16_supported(int dim, int metric);  // dim == tile dim in {32, 64, 128}, L2 / IP
// prep_only: the query operands (bq, qsc) without the sample (a list-sharded scan takes T_q from its plan)
void launch_sample16(const StreamArgs &a, int metric, int max_items, hipStream_t st, bool prep_only = false);
// T_q per query: the R-th largest of its n sample values, R from the sampled fraction f of its probed
// rows: R = clamp(ceil(et f), rmin, rmax) (rmin == rmax: fixed)
struct StreamSelectArgs {
  const float *samp;
  int64_t nq;
  int32_t n;
  int32_t rmin, rmax;
  double et;
  const int32_t *probes;  // [nq][nprobe]
  int32_t nprobe;
  const int32_t *lb, *le;
  float *thr;
};
void launch_stream_select(const StreamSelectArgs &a, hipStream_t st);
void launch_cand_merge(const CandMergeArgs &m, hipStream_t st);

struct RefineArgs {
  const float *rows;        // blocked store the keys index
  const float *rows_rm;     // its row-major copy (RowStore::rrm: one contiguous row per key), or null
  const int64_t *row_labels;
  const float *queries;     // row-major nq x D
  const float *ms;          // merged approximate scores [nq][ld] (desc)
  const int32_t *mk;        // merged keys [nq][ld] (-1 = none, -2 = a floor placeholder)
  int32_t ld;               // row stride of ms / mk (0: k1)
  const int32_t *qsel;      // refine only queries qsel[0 .. *nsel) (null: all nq)
  const int32_t *nsel;
  const uint32_t *max_rsq;  // score_key(max |x|^2 over the store) (device scalar)
  const uint32_t *list_rmax;  // IVF: score_key(max |x|^2) per list, or null (use max_rsq)
  const int32_t *probes;      // IVF: [nq][nprobe] probed lists (with list_rmax)
  int32_t nprobe;
  int32_t tri;                // L2: also bound row norms by |q| + sqrt(-skth) (refine_kernel)
  int64_t nq;
  int32_t k1, k, dim;
  double c_err;             // error-bound constant (refine_kernel)
  double c_bf;              // extra constant of the bf16x3 / fp16 filter (0 for fp32)
  double c_abs;             // fp16 filter: absolute error per |q| (filter_f16_abs), else 0
  int32_t q16;              // fp16 filter: add the queries' own fp16 subnormal term (per X, / sq)
  // IVF residual fp16 filter (approx = estimate of the score itself): centroids, per-list max
  // |x - c|^2 (score_key), and the query's probed lists (probes / nprobe above)
  const float *cents;
  const uint32_t *list_rmax_r;
  int32_t resid;
  int32_t ub;               // resid: candidate scores are upper bounds (StreamArgs kr ..): no error term
  // Cosine over unit residual tiles (ub): the candidates' bounds are L2 scores s of the unit vectors;
  // exact scores are VectorMath.Cosine(q, x, |q|, |x|), certified against 1 + s_K1 / 2 + (2D + 256) u
  int32_t cosine;
  const float *qnorm, *rnorm;
  const float *qcert;       // the queries the filter scored, for the error terms (null: queries)
  const uint32_t *zflag;    // != 0 once a row with a norm below 1e-6 was stored (k-th score must be > 0)
  float *out_s;
  int64_t *out_l;
  int32_t *out_c;
  int32_t *fail_list;       // queries whose certificate failed
  int32_t *fail_cnt;
  // list-sharded search (shard.hip; resid + ub only): query q's exact top-k and the bound of the rows it
  // left out go to record q of rec instead of out_*, with no certificate here (the home rank's merge
  // certifies); rec_lb / rec_nlist: the list bounds that name each candidate's list
  void *rec;
  const int32_t *rec_lb;
  int32_t rec_nlist;
  const int32_t *rec_row_list;  // or null: per row slot its list (launch_list_ids), one load instead of a search
};
// per list l, out[r] = l for its rows r in [lb[l], le[l]) (the slots' lists, for shard records)
void launch_list_ids(const int32_t *lb, const int32_t *le, int nlist, int32_t *out, hipStream_t st);
// unit rows (x / n, 0 when n < 1e-6 or not finite): blocked rows at slots (norms by slot), or row-major
// x (norms[i]) when slots is null; out row-major n x dim; zflag (may be null) set to 1 by a zero row that
// is live (live: per row index, null = every row)
void launch_unit_rows(const float *x, const int64_t *slots, const float *norms, int64_t n, int32_t dim, float *out,
                      hipStream_t st, uint32_t *zflag = nullptr, const uint8_t *live = nullptr);
// fp16 tiles of blocked fp32 rows (slots[i], or rows [0, n)), scaled by sx; with cents (row-major)
// and tile_list (list of each 32-row tile) the residuals x - c[list] (IVF lists)
// rn (may be null): the rows' meta norms; a non-finite one zeroes the row's tile (encode16_kernel)
void launch_encode16(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float sx, void *h16,
                     hipStream_t st, const float *cents = nullptr, const int32_t *tile_list = nullptr,
                     const float *rn = nullptr, int32_t dpad = 0);
// (dpad > dim: tiles of dpad dims, the dims past dim zero -- scan_tile_dim)
// |x - c[list]|^2 of rows [0, n)
void launch_resid_sq(const float *rows, int64_t n, int32_t dim, const float *cents, const int32_t *tile_list,
                     float *out, hipStream_t st, const int64_t *slots = nullptr, uint32_t *out_max = nullptr);
// meta[r] = live ? (L2 ? -rsq : 0) : -inf for slots[i] (or rows [0, n))
void launch_meta16(const int64_t *slots, int64_t n, int32_t metric, const float *rsq, const uint8_t *live, float *meta,
                   hipStream_t st);
// atomicMax of the float bits of max |x_i| (finite) over the rows into *out
void launch_absmax(const float *rows, const int64_t *slots, int64_t n, int32_t dim, uint32_t *out, hipStream_t st,
                   const float *cents = nullptr, const int32_t *tile_list = nullptr);
// V: 1 = VectorMath safe form (IVF), 4 = *Unsafe form (FLAT)
void launch_refine(const RefineArgs &a, int metric, int V, hipStream_t st);
// the stream scans' candidate merge + certified refine in one wave per query (filter.hip
// merge_refine_kernel): depth a.k1 (a multiple of 8), the failures at depth STREAM_KO in the same wave,
// what fails there into a.fail_list / a.fail_cnt; a.rec: shard records instead.  Upper-bound (resid, ub)
// candidates only.
void launch_merge_refine(const CandMergeArgs &m, const RefineArgs &a, int metric, int V, hipStream_t st);
// k > 60: the same at depth K1 = 128 / 256 / 512 (k <= 0.8 K1), one block per query (IVF V = 1, FLAT V = 4); LDS per block
// deep_refine_lds_bytes (the candidate buffer must keep it within 60 KiB)
size_t deep_refine_lds_bytes(int cap, int k1);
void launch_deep_refine(const CandMergeArgs &m, const RefineArgs &a, int metric, int V, hipStream_t st);
void launch_gather_queries(const float *q, const int32_t *qidx, int64_t n, int32_t dim, float *out, hipStream_t st);
// rows idx[i] of a [*][width] array of 32-bit words (probe lists of the failing queries)
void launch_gather_words(const uint32_t *src, const int32_t *idx, int64_t n, int32_t width, uint32_t *out,
                         hipStream_t st);
void launch_scatter_results(const int32_t *qidx, int64_t n, int32_t k, const float *ss, const int64_t *sl,
                            const int32_t *sc, float *out_s, int64_t *out_l, int32_t *out_c, hipStream_t st);
// |x|^2 of blocked rows (at slots, or rows [0,n) when slots is null) + atomic running max
// per-list max |x|^2 (score_key; finite rows) of rows [lb[l], le[l]) -> out[nlist]
void launch_list_rmax(const float *rsq, const int32_t *lb, const int32_t *le, int32_t nlist, uint32_t *out,
                      hipStream_t st);
void launch_sqnorms(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float *out, uint32_t *max_key,
                    hipStream_t st);

// layout helpers
// dst blocked rows [dst_row0 ...] from row-major src rows (src_idx[i] or i when null)
void launch_to_blocked(const float *src, const int64_t *src_idx, int64_t n, int32_t dim, float *dst, int64_t dst_row0,
                       hipStream_t st);
// scattered writes: row i of src (row-major) -> blocked slot dst_slots[i]
// row-major copies (RowStore::rrm): dst row i = src row src_idx[i] (zero when < 0; src_idx null = i);
// src rows scattered to dst_slots
void launch_to_rowmajor(const float *src, const int64_t *src_idx, int64_t n, int32_t dim, float *dst, hipStream_t st);
void launch_scatter_rowmajor(const float *src, const int64_t *dst_slots, int64_t n, int32_t dim, float *dst,
                             hipStream_t st);
void launch_scatter_blocked(const float *src, const int64_t *dst_slots, int64_t n, int32_t dim, float *dst,
                            hipStream_t st);
// gather blocked rows (src_slot[i]) into row-major out
void launch_gather_blocked(const float *src, const int64_t *src_slots, int64_t n, int32_t dim, float *out,
                           hipStream_t st);
// gather rows from two blocked stores: idx >= 0 -> store A row idx, idx < 0 -> store B row (-idx-1)
void launch_gather2(const float *A, const float *B, const int64_t *idx, int64_t n, int32_t dim, float *out,
                    hipStream_t st);
void launch_gather_rows(const float *src, const int32_t *idx, int64_t n, int32_t dim, float *out, hipStream_t st);
// out[i][:] = src[idx[i]][:] for int32 rows of `width` entries (probe lists of a query subset)
void launch_gather_rows_i32(const int32_t *src, const int32_t *idx, int64_t n, int32_t width, int32_t *out,
                            hipStream_t st);

// k-means helpers (KMeansUtils.cs:40-62)
void launch_keys_to_assign(const uint32_t *keys, int64_t n, int32_t *assign, hipStream_t st);
void launch_kmeans_update(const float *data, const int32_t *members, const int32_t *coff, int32_t k, int32_t dim,
                          float *cents, float *tmp, int32_t *flags, int32_t *changed, hipStream_t st);
// stable counting sort of [0,n) by key in [0,k): members and offsets (hipCUB radix sort)
size_t sort_temp_bytes(int64_t n, int32_t k);
void sort_by_key(const int32_t *keys, int64_t n, int32_t k, int32_t *keys_tmp, int32_t *idx_in, int32_t *members,
                 int32_t *counts, int32_t *coff, void *temp, size_t temp_bytes, hipStream_t st);

void fill_u8(uint8_t *p, uint8_t v, int64_t n, hipStream_t st);
// Up to 8 ranges of 32-bit words set to a value each, in ONE kernel.  Every per-search counter reset goes
// through it: hipMemsetAsync / hipMemsetD32Async captured into a hipGraph write stale values from the
// graph's second replay on in the HIP runtime PyTorch ships (scripts/diag/graph_memset.py), and
// one kernel node also replaces up to 8 fill nodes of ~5 us each.
struct WordFill {
  static constexpr int MAXR = 8;
  uint32_t *p[MAXR] = {};
  int64_t n[MAXR] = {};
  uint32_t v[MAXR] = {};
  int cnt = 0;
  void add(void *ptr, int64_t words, uint32_t value);  // ignored when ptr is null or words <= 0
};
void launch_fill_words(const WordFill &f, hipStream_t st);
// device-to-device copy of 32-bit words on a search path (a kernel, not a hipMemcpyAsync node: the same
// graph-replay rule as WordFill)
void launch_copy_words(void *dst, const void *src, int64_t words, hipStream_t st);
void launch_scatter_i64(int64_t *dst, const int64_t *idx, const int64_t *vals, int64_t n, hipStream_t st);
void launch_scatter_u8(uint8_t *dst, const int64_t *idx, uint8_t v, int64_t n, hipStream_t st);
// norms of blocked rows at the given slots (VectorMath.ComputeNorm)
void launch_norms_slots(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float *out, hipStream_t st);
// A few rows written in ONE launch (RowStore::write's small-batch path): everything the separate write
// kernels do for them -- blocked rows, the row-major copy, label, live, |x|^2 (+ the store's max key or its
// non-finite flag), the Cosine norm (ComputeNorm), and for fp16 stores the residual |x - center|^2, the
// fp16 tile entries at the current scale and meta -- with the same arithmetic, in the same order.
struct SmallWriteArgs {
  const float *x;        // staged rows, row-major [cnt][dim]
  const int64_t *slots;  // [cnt]
  const int64_t *labs;   // [cnt]
  int32_t cnt, dim, dp;  // dp: the tile dimension
  float *rows, *rrm;     // blocked rows; the row-major copy (null: none)
  int64_t *labels;
  uint8_t *live;
  float *norms;          // Cosine stores: ComputeNorm per slot (null: none)
  float *rsq;
  uint32_t *rmax;        // [0] max score key of the finite |x|^2, [1] non-finite flag
  _Float16 *h16;         // fp16 tiles (null: none)
  float sx;
  const float *center;   // FLAT L2: the tiles hold x - center (null: x)
  float *rsq16;
  uint32_t *rmax_r;
  float *meta;
  int32_t met16;
  uint8_t *q8ok;         // FLAT: the slot's 8-bit codes are invalid now (null: untouched)
  float *mub;            // the stream scan's cached per-row terms (RowStore::row_terms), kept current for these
  float mkr, mkx;        // rows with its constants (null: the cache is stale anyway)
  int32_t mmet;
};
// the rows themselves as kernel arguments (a.x == null): a host write never stages through pinned memory
// (CPU stores into it measured ~22 us per 528 B row)
constexpr int SMALL_INLINE_FLOATS = 832, SMALL_INLINE_ROWS = 8, SMALL_WRITE_MAX_DIM = 4096;
struct SmallWriteRows {
  float x[SMALL_INLINE_FLOATS];
  int64_t slot[SMALL_INLINE_ROWS], lab[SMALL_INLINE_ROWS];
};
void launch_write_small(const SmallWriteArgs &a, hipStream_t st, const SmallWriteRows *rows = nullptr);
// per-dimension sums (fp64) of the live rows among [0, n) of a blocked store and their count -> sums[dim],
// *count (both zeroed by the caller): the FLAT L2 tiles' re-centring (RowStore::recenter)
void launch_live_sums(const float *rows, const uint8_t *live, int64_t n, int32_t dim, double *sums,
                      unsigned long long *count, hipStream_t st);
// empty result rows: score -inf, label -1, count 0
void launch_fill_results(float *s, int64_t *l, int32_t *c, int64_t nq, int32_t k, hipStream_t st);
bool fast_path(int dim, int k);

}  // namespace pyr
