/*
 * pyrope_ann.h -- C ABI of libpyrope_hip.so, the MI355X (gfx950) engine for
 * Pyrope's batched ANN distance-scan hot path.
 *
 * This is the drop-in boundary.  Each entry point replaces one member of the
 * reference plugin contract `IVectorIndex` (reference:
 * src/Pyrope.GarnetServer/Vector/IVectorIndex.cs:14-29) or its factory branch
 * (Services/VectorIndexRegistry.cs:81-113), and is what a C# P/Invoke shim
 * (`HipVectorIndex : IVectorIndex, ICentroidsProvider`)
 * binds.  Plain C: no exceptions cross the ABI, caller-owned buffers, the
 * library copies every input and keeps no caller pointer after return.
 *
 * Ids: the reference keys rows by `string id`; the shim maps each id to a
 * unique int64 label and back.  Labels < 0 are rejected.
 *
 * Threading (reference: one ReaderWriterLockSlim per index, e.g.
 * BruteForceVectorIndex.cs:23): any number of concurrent pyr_index_search*
 * calls; add/upsert/remove/build take the index exclusively.
 *
 * Scores: "higher is better", with the reference's signs
 * (L2 -> -sum((q-x)^2), IP -> q.x, Cosine -> q.x/(|q||x|), IVF-PQ -> -ADC for
 * every metric).  Results per query are sorted by score descending, ties by
 * storage order (DESIGN.md "Tie rule").  Empty result slots hold
 * score = -INFINITY and label = -1.
 */
#ifndef PYROPE_ANN_H
#define PYROPE_ANN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pyr_index pyr_index; /* opaque */

typedef enum {
  PYR_OK = 0,
  PYR_E_DIM = 1,       /* -> ArgumentException("Vector dimension mismatch.") => VEC_ERR_DIM (VectorCommandSet.cs:837-847) */
  PYR_E_ARG = 2,       /* -> ArgumentException / ArgumentOutOfRangeException (e.g. topK <= 0, BruteForceVectorIndex.cs:278) */
  PYR_E_STATE = 3,     /* -> InvalidOperationException (wrong index kind / not built) */
  PYR_E_OOM = 4,       /* device or host allocation failed */
  PYR_E_DEVICE = 5,    /* HIP runtime error, or no gfx950 device */
  PYR_E_DUPLICATE = 6, /* -> InvalidOperationException("Vector with id ... already exists.") (BruteForceVectorIndex.cs:141-144) */
  PYR_E_NOT_FOUND = 7, /* -> FileNotFoundException("Snapshot file not found.") (BruteForceVectorIndex.cs:87, IvfFlatVectorIndex.cs:259) */
  PYR_E_FORMAT = 8,    /* -> JsonException: the file is not an index image of this kind / dimension / metric */
  PYR_E_IO = 9         /* -> IOException: the image could not be written */
} pyr_status;

/* == VectorMetric ordinals (IVectorIndex.cs:5-10) */
typedef enum { PYR_L2 = 0, PYR_IP = 1, PYR_COS = 2 } pyr_metric;

/* FLAT   = BruteForceVectorIndex (the Delta head; BruteForceVectorIndex.cs)
 * IVF_FLAT = IvfFlatVectorIndex (IvfFlatVectorIndex.cs)
 * IVF_PQ = IvfPqVectorIndex + ProductQuantizer (IvfPqVectorIndex.cs, ProductQuantizer.cs) */
typedef enum { PYR_FLAT = 0, PYR_IVF_FLAT = 1, PYR_IVF_PQ = 2 } pyr_kind;

typedef struct {
  int32_t kind;           /* pyr_kind */
  int32_t dim;            /* > 0 (BruteForceVectorIndex.cs:43-46) */
  int32_t metric;         /* pyr_metric */
  int32_t nlist;          /* IVF: NList (registry default 100, VectorIndexRegistry.cs:100,106) */
  int32_t pq_m;           /* IVF_PQ: M, dim % M == 0 (ProductQuantizer.cs:18) */
  int32_t pq_k;           /* IVF_PQ: K <= 256 (ProductQuantizer.cs:19) */
  int32_t device;         /* HIP device ordinal when device_mask is 0 */
  int32_t default_nprobe; /* <= 0 -> reference default: 3 IVF_FLAT (IvfFlatVectorIndex.cs:14), 1 IVF_PQ (IvfPqVectorIndex.cs:125) */
  /* Multi-GPU (SURVEY.md 8(b) device_mask; 8(e)(i) lists sharded whole; DESIGN.md §5 "One process, several
   * GPUs").  device_mask: bit d = HIP device d (0 -> `device` alone).  One bit and shards = 0: an ordinary
   * single-GPU index on that device.  More bits, or shards >= 1 (IVF_FLAT only): ONE index whose lists are
   * dealt whole to `shards` shard indexes (0 -> one per device of the mask; shard r on the (r mod n)-th device
   * of the mask), searched by the list-sharded step inside the library with RCCL collectives between the
   * devices (device copies when two shards share a device).  Every IVectorIndex call works on it: writes and
   * Build go to a single-GPU index on the first device that holds every row (the reference Build, bit for
   * bit), which then deals its lists to the shards; pyr_index_search* answers by the list-sharded step
   * (L2 / IP, k <= 60, empty buffer) or else on that first-device index.  Results equal the single-GPU
   * index's, ids and score bits. */
  uint64_t device_mask;
  int32_t shards;
  int32_t reserved;
} pyr_index_desc;

/* SearchOptions (SearchOptions.cs:3) */
typedef struct {
  int32_t nprobe;    /* < 0 -> index default; 0 -> no list is probed (Math.Min(nProbe, n) <= 0) */
  int32_t reserved;
  int64_t max_scans; /* < 0 -> unlimited; 0 -> empty result (BruteForceVectorIndex.cs:288-289). IVF_PQ ignores it. */
} pyr_search_params;

/* new XxxVectorIndex(...) inside VectorIndexRegistry.IndexState (VectorIndexRegistry.cs:81-113). */
pyr_status pyr_index_create(const pyr_index_desc *desc, pyr_index **out);
void pyr_index_destroy(pyr_index *index);

/* IVectorIndex.Add (IVectorIndex.cs:19).  x: n x dim row-major fp32.
 * FLAT: a label that already exists -> PYR_E_DUPLICATE and nothing is added.
 * IVF_*: Add == Upsert into the pre-build buffer (IvfFlatVectorIndex.cs:39-59, IvfPqVectorIndex.cs:37-47). */
pyr_status pyr_index_add(pyr_index *index, const float *x, int64_t n, const int64_t *labels);
/* IVectorIndex.Upsert (IVectorIndex.cs:20; BruteForceVectorIndex.cs:181-222). */
pyr_status pyr_index_upsert(pyr_index *index, const float *x, int64_t n, const int64_t *labels);
/* IVectorIndex.Delete (IVectorIndex.cs:21).  removed[i] = 1 if labels[i] was present (may be NULL). */
pyr_status pyr_index_remove(pyr_index *index, const int64_t *labels, int64_t n, uint8_t *removed);
/* IVectorIndex.Build (IVectorIndex.cs:25): reference-identical k-means training
 * (KMeansUtils.Train semantics, run on the GPU), assignment and PQ encoding.  FLAT: no-op. */
pyr_status pyr_index_build(pyr_index *index);

/* Supply a trained coarse quantizer (nlist x dim, row-major) for the next Build of an IVF index,
 * which then only assigns (and, for IVF_PQ, trains codebooks).  The C# shim uses it to hand over
 * KMeansUtils.Train output; the multi-GPU path uses it so every shard shares one quantizer. */
pyr_status pyr_index_set_centroids(pyr_index *index, const float *centroids, int32_t nlist);

/* IVF_PQ: supply trained ProductQuantizer codebooks (m x ksub x dim/m, ProductQuantizer._centroids,
 * ProductQuantizer.cs:7-8) together with pyr_index_set_centroids; the next Build then only assigns
 * and encodes (Encode, :60-80), streaming the buffer in chunks -- what a 50M x 768 build needs
 * (training on every row is the reference's behaviour when no quantizer is supplied). */
pyr_status pyr_index_set_codebooks(pyr_index *index, const float *codebooks, int32_t m, int32_t ksub);

/* Capacity hint: room for `rows` more rows (FLAT slots / IVF buffer) without re-allocation.  The
 * .NET collections the reference fills grow by copying; a device store of 10^8 rows cannot hold the
 * old and the new copy at once, so bulk loaders reserve first.  No effect on results. */
pyr_status pyr_index_reserve(pyr_index *index, int64_t rows);

/* KMeansUtils.Train (KMeansUtils.cs:10-68) on the GPU, reference-identical: OrderBy(rnd.Next())
 * initialisation, <= max_iter Lloyd iterations, member sums in data order, ArraysEqual(1e-6) stop.
 * data: n x dim host row-major.  out: k x dim (k clamped to [1, n]); *k_out = k used. */
pyr_status pyr_kmeans_train(int32_t device, const float *data, int64_t n, int32_t dim, int32_t k, int32_t metric,
                            int32_t max_iter, int32_t seed, float *out, int32_t *k_out);

/* IVectorIndex.Search (IVectorIndex.cs:22) for a batch of queries.  Host buffers.
 * q: nq x dim; out_scores/out_labels: nq x k; out_counts: nq (may be NULL).
 * params may be NULL (= SearchOptions null). */
pyr_status pyr_index_search(pyr_index *index, const float *q, int64_t nq, int32_t k,
                            const pyr_search_params *params, float *out_scores, int64_t *out_labels,
                            int32_t *out_counts);
/* Request coalescing for pyr_index_search (the reference serves one query per VEC.SEARCH call,
 * Extensions/VectorCommandSet.cs:457-459, from many session threads): with max_wait_us > 0,
 * concurrent pyr_index_search calls of fewer than max_batch queries and equal (k, params) are merged
 * into one device search of up to max_batch queries.  A batch starts at once when no coalesced
 * search of the index is running (an idle device adds no wait), else when the running one finishes,
 * when it is full, or at the latest max_wait_us after its first query arrived; each caller gets
 * exactly its own rows (results are per-query identical to uncoalesced calls).  max_wait_us <= 0
 * turns it off (the default). */
pyr_status pyr_index_set_coalescing(pyr_index *index, int32_t max_batch, int32_t max_wait_us);
/* Same on device-resident buffers (HBM), enqueued on `stream` (hipStream_t, NULL = default).
 * On a built IVF_FLAT index with an empty buffer (the stream scan: L2 / IP / Cosine, d = 32 / 64 / 128)
 * it only enqueues work: no host synchronisation, capturable into a hipGraph.  The FLAT filter and
 * the exact / PQ paths may synchronize `stream` once to size the re-run of certificate failures. */
pyr_status pyr_index_search_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                   const pyr_search_params *params, float *d_scores, int64_t *d_labels,
                                   int32_t *d_counts, void *stream);

/* Multi-GPU split of the coarse step (DESIGN.md "Multi-GPU"): every rank ranks the coarse quantizer
 * (IvfFlatVectorIndex.cs:186-198) for its slice of the batch, the probe lists are all-gathered, and
 * every rank searches its shard with the gathered lists.  IVF_FLAT only.
 * pyr_index_probe_device: d_probes = nq x P device int32 list ids in rank order, P = min(nprobe, nlist)
 *   (nprobe < 0 -> index default), written to *probes_out (may be NULL).
 * pyr_index_search_probed_device: pyr_index_search_device with those lists instead of the coarse
 *   step; nprobe = their width, which must equal what params select. */
pyr_status pyr_index_probe_device(pyr_index *index, const float *d_q, int64_t nq, int32_t nprobe, int32_t *d_probes,
                                  int32_t *probes_out, void *stream);
pyr_status pyr_index_search_probed_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                          const pyr_search_params *params, const int32_t *d_probes, int32_t nprobe,
                                          float *d_scores, int64_t *d_labels, int32_t *d_counts, void *stream);

/* IVectorIndex.Snapshot (IVectorIndex.cs:26): write a binary image of the index to `path` (UTF-8,
 * NUL-terminated) through path + ".tmp" and a rename (the temp + move of DeltaVectorIndex.cs:160-191).
 * The image holds what the reference's snapshot DTOs hold (BruteForceVectorIndex.cs:58-82: live rows
 * with their labels in slot order; IvfFlatVectorIndex.cs:233-257: IsBuilt, centroids, buffer, inverted
 * lists in order) as raw arrays that load into HBM with one copy each; IVF_PQ images also hold the
 * codebooks and codes (the reference's IvfPq Snapshot/Load are no-ops, IvfPqVectorIndex.cs:228-229).
 * Layout: pyrope_amd/csrc/persist.h.  Takes the index shared (concurrent searches may run). */
pyr_status pyr_index_snapshot(pyr_index *index, const char *path);
/* IVectorIndex.Load (IVectorIndex.cs:27): replace the index's state with the image at `path`.
 * PYR_E_NOT_FOUND if there is no file; PYR_E_FORMAT if it is not an image of an index of this kind
 * and dimension (the recorded metric is not enforced, as the reference ignores IvfStateDto.Metric).  Sections missing from an image load as empty (IvfFlatVectorIndexTests.cs:
 * 144-165).  FLAT rows are re-added in slot order (BruteForceVectorIndex.cs:84-106: Clear, then
 * InternalAdd, so the 8-bit codes follow the loading index's EnableQuantization).  Exclusive. */
pyr_status pyr_index_load(pyr_index *index, const char *path);
/* The 16 random bytes every pyr_index_snapshot draws for its image (all zero for an image written
 * before they were recorded).  No reference counterpart: the Python shim stores them in its
 * path + ".ids" id map and ignores a map whose bytes differ from the image's, so a crash between the
 * two renames cannot pair an image with another snapshot's ids (the reference keeps ids inside its
 * DTOs, BruteForceVectorIndex.cs:58-82).  Host only; PYR_E_NOT_FOUND / PYR_E_FORMAT as pyr_index_load. */
pyr_status pyr_image_nonce(const char *path, uint8_t *nonce);

/* IVectorIndex.GetStats (IVectorIndex.cs:28): Count with the reference's semantics
 * (IvfFlat counts buffer + list rows, IvfFlatVectorIndex.cs:305; IvfPq reports 0, IvfPqVectorIndex.cs:230). */
pyr_status pyr_index_stats(const pyr_index *index, int64_t *count, int32_t *dim, int32_t *metric);

/* ICentroidsProvider.GetCentroids (ICentroidsProvider.cs:14; IvfFlatVectorIndex.cs:314-325).
 * out may be NULL to query *nlist; *nlist = 0 when not built. */
pyr_status pyr_index_get_centroids(const pyr_index *index, float *out, int32_t *nlist);

/* BruteForceVectorIndex.Scan (BruteForceVectorIndex.cs:250-273; the source of DeltaVectorIndex.Build's
 * head -> tail compaction, DeltaVectorIndex.cs:124-158): the live rows in slot order.
 * labels: *n entries, x: *n x dim row-major; either may be NULL (call with both NULL to size).
 * FLAT only (PYR_E_STATE otherwise).  Takes the index exclusively (it uses the write stream). */
pyr_status pyr_index_scan(pyr_index *index, int64_t *labels, float *x, int64_t *n);

/* The labels of every row the index holds (FLAT slots; IVF buffer and list entries; a label may
 * repeat when a buffer row shadows a list entry).  labels may be NULL to size (*n = count); else *n
 * is its capacity on entry (PYR_E_ARG if too small) and the count on return.  The shim rebuilds its
 * id <-> label map from it after pyr_index_load of an image written without one (the reference's
 * snapshot DTOs carry the ids themselves, BruteForceVectorIndex.cs:58-82, IvfFlatVectorIndex.cs:233-257). */
pyr_status pyr_index_labels(const pyr_index *index, int64_t *labels, int64_t *n);

/* BruteForceVectorIndex.EnableQuantization (BruteForceVectorIndex.cs:25-40), FLAT only:
 * rows added / upserted while it is on carry ScalarQuantizer codes, and searches run in the
 * 8-bit mode (:296-336): the query is quantized, scores are -L2Squared8Bit / DotProduct8Bit
 * (cosine too) as float, rows written while it was off count as scanned but are skipped.
 * Scores come from exact int8 MFMA sums; supported for dim <= 512 and topK <= 64 (PYR_E_ARG
 * otherwise). */
pyr_status pyr_index_set_quantization(pyr_index *index, int32_t enable);

/* ScalarQuantizer.Quantize (ScalarQuantizer.cs:23-62) of n vectors (n x dim, row-major) on the
 * GPU: per-vector min/max, codes = clamp(round_half_even((x - min) * (255 / (max - min)))). */
pyr_status pyr_scalar_quantize(int32_t device, const float *x, int64_t n, int32_t dim, uint8_t *codes);
/* The same with Quantize's `out float min, out float max` per vector (mins / maxs: n entries, may be NULL). */
pyr_status pyr_scalar_quantize_minmax(int32_t device, const float *x, int64_t n, int32_t dim, uint8_t *codes,
                                      float *mins, float *maxs);
/* ScalarQuantizer.Dequantize (ScalarQuantizer.cs:65-84) of n code rows: out = min + q * ((max - min) / 255)
 * in fp32, or min everywhere when max == min. */
pyr_status pyr_scalar_dequantize(int32_t device, const uint8_t *codes, int64_t n, int32_t dim, const float *mins,
                                 const float *maxs, float *out);

/* Introspection of the built IVF layout (list-major storage order, used by the
 * parity tests and the CPU baseline).  list_off: nlist+1 (row offsets without padding),
 * labels: total rows (state of removed rows: label -1), live: 1 visible, 0 removed/shadowed.
 * Any output may be NULL; *total receives the row count. */
pyr_status pyr_index_ivf_layout(const pyr_index *index, int64_t *list_off, int64_t *labels, uint8_t *live,
                                int64_t *total);
/* IVF_PQ trained state: codebooks [M][ksub][dim/M]; codes list-major (total x M).  Any output may be NULL. */
pyr_status pyr_index_pq_state(const pyr_index *index, float *codebooks, int32_t *ksub, uint8_t *codes);

/* Multi-GPU merge (RCCL allgather of per-GPU partial top-k; DESIGN.md "Multi-GPU"):
 * d_scores/d_labels: nq x nparts x k partial lists, each sorted (score desc, label asc);
 * writes the global top-k per query, ties by label asc.  Device buffers, async on stream. */
pyr_status pyr_merge_topk_device(const float *d_scores, const int64_t *d_labels, int64_t nq, int32_t nparts,
                                 int32_t k, float *d_out_scores, int64_t *d_out_labels, void *stream);
/* The same over either layout: part_major = 0 reads nq x nparts x k (as above); part_major = 1 reads
 * nparts x nq x k, the buffer an all_gather of per-GPU nq x k partials leaves (no transpose). */
pyr_status pyr_merge_topk_parts_device(const float *d_scores, const int64_t *d_labels, int64_t nq, int32_t nparts,
                                       int32_t k, int32_t part_major, float *d_out_scores, int64_t *d_out_labels,
                                       void *stream);

/* ---- List-sharded multi-GPU IVF_FLAT search ("IVF lists shard naturally across the
 * GPUs"; orchestration: pyrope_amd/dist.py ListShardedIvf).  The reference path split is
 * the probed-list loop of IvfFlatVectorIndex.Search (IvfFlatVectorIndex.cs:198-218): every rank holds
 * WHOLE lists (the rows FindNearestCentroid sends to a list it owns, in label order) plus the shared
 * quantizer, so a (query, list) pair is scanned by exactly one rank.  A step:
 *   home rank (its slice of the batch)  pyr_index_shard_prepare_device -> plan [nq][P + 1 (+ P)]
 *   all ranks, all_gather(plans)        pyr_index_shard_search_device  -> one record per query
 *   all_to_all(records) to the homes    pyr_shard_merge_device         -> results + failed certificates
 *   all_gather(fail lists)              pyr_index_shard_rerun_device   -> exact records of the failures
 *   all_to_all(records) to the homes    pyr_shard_merge_device(qsel)   -> their exact results
 * Results equal the unsharded index's, ties included ((score desc, list asc, label asc) is the unsharded
 * storage order).  Device buffers, enqueued on `stream`; no host synchronisation.
 * A home may have more failing certificates than one re-run round carries (fcap per home): its fail list
 * (d_fail, sized to its batch) keeps every one, and the caller runs further rounds over the later entries
 * (pyrope_amd/dist.py ListShardedIvf: a round takes entries [off, off + fcap) of every home's list).
 * MaxScans (SearchOptions.MaxScans, IvfFlatVectorIndex.cs:202-212): the home runs the budget down its
 * queries' probe order over every rank's lists (their lengths from pyr_index_set_list_samples) and the plan
 * carries, per probe, what is left of it when that list is reached; the owning rank scans the list up to
 * that many live rows.  A rank refuses a budgeted search (PYR_E_STATE) once one of its lists lost rows since
 * its samples were set. */

/* The multi-GPU index (pyr_index_desc.device_mask / shards): its shard count (1 for a single-GPU index), the
 * transport of its list-sharded step (0 none yet, 1 device copies, 2 RCCL), the searches the step answered and
 * those the first-device index answered alone (Cosine, k > 60, a non-empty buffer), and the last step's largest
 * certificate-failure count at one home with its re-run rounds past the first.  Any output may be NULL. */
pyr_status pyr_index_shard_info(const pyr_index *index, int32_t *shards, int32_t *xport, int64_t *sharded_searches,
                                int64_t *staged_searches, int64_t *last_max_failures, int64_t *last_extra_rounds);

/* KMeansUtils.FindNearestCentroid (KMeansUtils.cs:70-93; the assignment of IvfFlatVectorIndex.Build,
 * :128-132) of n host rows against nlist host centroids: assign[i] = the list row i belongs to (ties ->
 * lowest index).  The row exchange that gives every rank its whole lists uses it. */
pyr_status pyr_assign(int32_t device, const float *centroids, int32_t nlist, const float *x, int64_t n, int32_t dim,
                      int32_t metric, int32_t *assign);
/* Bytes of one record: k entries {int64 label, float score, int32 list} in (score desc, list asc, label
 * asc) order (empty: label -1, score -inf), then {float bound, int32 n, 8 pad}: every row of the rank's
 * probed lists that is not an entry scores at most `bound` (-inf: none was left out).  16 (k + 1). */
int64_t pyr_shard_record_bytes(int32_t k);
/* The replicated sample of every list, on a built shard index (L2 / IP): rows = the first counts[l] <= 512
 * rows of each list l in list order, concatenated (sum counts x dim, host); list_len[l] = list l's full
 * length on the rank that owns it.  It is what the unsharded index's sample pass scores, so the home
 * rank's T_q equals the unsharded one. */
pyr_status pyr_index_set_list_samples(pyr_index *index, const float *rows, const int64_t *counts,
                                      const int64_t *list_len, int32_t nlist);
/* Home rank: the coarse ranking (IvfFlatVectorIndex.cs:186-198) and the threshold T_q of nq queries:
 * d_plan [nq][P + 1] int32 = P probe ids in rank order, then T_q's float bits; *width = P = min(nprobe, nlist).
 * With params->max_scans >= 0 the rows are [nq][2P + 1]: then, per probe, the MaxScans budget left when its
 * list is reached (plan_budgets = 1 in the calls below).  Row stride: pyr_shard_plan_stride. */
pyr_status pyr_index_shard_prepare_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                          const pyr_search_params *params, int32_t *d_plan, int32_t *width,
                                          void *stream);
/* The int32 row stride of a plan: P + 1, or 2P + 1 with a MaxScans budget (max_scans >= 0). */
int32_t pyr_shard_plan_stride(int32_t width, int64_t max_scans);
/* Every rank: the stream scan of the (query, list) pairs of the gathered plans whose list this rank owns
 * (the others are empty here) against T_q, the exact refine of each query's best candidates, and one
 * record per query (d_records: nq x pyr_shard_record_bytes(k)).  k <= 60.  plan_budgets: the plans carry
 * MaxScans budgets (prepared with max_scans >= 0); each owned list is then scanned up to its pair's budget. */
pyr_status pyr_index_shard_search_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                         const int32_t *d_plan, int32_t width, int32_t plan_budgets, void *d_records,
                                         void *stream);
/* Merge nparts (<= 64) records per query and certify.  d_records: [nparts][nrec] (an all_to_all's
 * output).  d_qsel = NULL: record i answers query i (i < nrec), results to row i, and with d_fail the
 * certificate (the k-th merged score beats every bound) lists failing queries: d_fail[0] = their count
 * (may exceed fcap: the caller must then re-run the excess), d_fail[1 .. fcap].  d_qsel = a fail list
 * [1 + cap]: record i answers query d_qsel[1 + i], i < min(d_qsel[0], cap) (the re-run's answers). */
pyr_status pyr_shard_merge_device(const void *d_records, int32_t nparts, int64_t nrec, int32_t k,
                                  const int32_t *d_qsel, int32_t cap, float *d_scores, int64_t *d_labels,
                                  int32_t *d_counts, int32_t *d_fail, int32_t fcap, void *stream);
/* Every rank: the exact search (the *safe* VectorMath forms, IvfFlatVectorIndex.cs:200-218) of the
 * gathered failures d_fails [nranks][1 + fcap] (home-local query ids; home s's queries are rows
 * s * nq_home .. of d_q / d_plan; nq = all of them) over this rank's lists: the answer to home s's j-th
 * failure is record s * fcap + j of d_records ([nranks * fcap] records, bound -inf).  plan_budgets: as
 * pyr_index_shard_search_device (the re-run stops where the scan did). */
pyr_status pyr_index_shard_rerun_device(pyr_index *index, const float *d_q, int64_t nq, int32_t k,
                                        const int32_t *d_plan, int32_t width, int32_t plan_budgets,
                                        const int32_t *d_fails, int32_t nranks, int32_t fcap, int64_t nq_home,
                                        void *d_records, void *stream);

/* HBM plan (host arithmetic, no device needed): the bytes an IVF_FLAT index of nrows rows in nlist
 * lists (longest max_list_len rows) holds on one GPU, and the workspace one batched search of nq queries
 * (nprobe, k) on the default list scan allocates.  A multi-GPU launcher sizes each rank with it before
 * loading its shard (no reference counterpart: the reference is one process on the host heap). */
pyr_status pyr_ivf_memory_plan(int32_t dim, int64_t nrows, int32_t nlist, int64_t max_list_len, int64_t nq,
                               int32_t nprobe, int32_t k, int64_t *index_bytes, int64_t *workspace_bytes);

/* Pyrope.Benchmarks synthetic generator (Program.cs:251-263): v[d] = (float)new Random(seed).NextDouble(),
 * row by row.  Host buffer count x dim.  Measurement-harness utility. */
pyr_status pyr_generate_synthetic(int64_t count, int32_t dim, int32_t seed, float *out);
/* Row-blocked form for large N (block b of `block_rows` rows is the sequence of
 * new Random(seed + b)), so a shard of whole blocks is generated without the rows before it.
 * Writes rows [row0, row0 + count) to out (count x dim); blocks are generated in parallel.
 * With row0 + count <= block_rows it equals pyr_generate_synthetic. */
pyr_status pyr_generate_synthetic_blocked(int64_t row0, int64_t count, int32_t dim, int32_t seed, int64_t block_rows,
                                          float *out);

/* Kernel-phase profiler (HIP events on the search stream; adds a host sync per search while on).
 * phase: 0 coarse scan+select, 1 IVF work lists, 2 IVF list scan, 3 buffer scan, 4 final merge,
 * 5 FLAT scan, 6 IVF-PQ LUT+ADC scan, 7 MFMA-filter refine (exact re-score + certificate),
 * 8 exact re-run of queries whose certificate failed.  *work = (query, row) pairs the phase
 * scored (phase 8: queries re-run). */
void pyr_profile_enable(int32_t on);
void pyr_profile_reset(void);
pyr_status pyr_profile_get(int32_t phase, double *total_ms, int64_t *calls, int64_t *work);

/* Measurement only (tests/test_gpu_bounds.py, scripts/bound_slack.py, scripts/write_path.py): the rows
 * the last stream-scan query slice emitted (with the environment PYR_STREAM_EMIT_ALL=1 the stream scans
 * emit every visible row of the scanned lists, without the sampled threshold, and with PYR_STREAM_CAP >=
 * the rows a query scans all of them are kept): per query q, h_cnt[q] rows (h_cnt > cap: some were dropped) at [q * cap, ...) with
 * h_ub = the row's upper-bound score (stream_ub_terms) and h_label = its label (-1: a row no longer
 * visible).  nq / cap must be that slice's.  No reference counterpart. */
pyr_status pyr_index_debug_candidates(pyr_index *index, int64_t nq, int32_t cap, float *h_ub, int64_t *h_label,
                                      int32_t *h_cnt);

/* thread-local message of the last failing call on this thread */
const char *pyr_last_error(void);
/* library / device information string, e.g. "pyrope_hip 0.1 gfx950" */
const char *pyr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PYROPE_ANN_H */
