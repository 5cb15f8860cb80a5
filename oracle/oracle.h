/*
 * oracle.h -- CPU restatement of Pyrope's C# ANN scan engine.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (pyrope_amd/,
 * libpyrope_hip.so) may include, link or call this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 * as the checker / the timed CPU baseline.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * src/Pyrope.GarnetServer/ unless stated).  The reference is C#/.NET 8 and
 * cannot run in this image (no dotnet); see DESIGN.md "Oracle" for what pins it.
 *
 * Arithmetic boundary (third-party, not in the reference tree):
 *   - System.Numerics.Vector<float> is restated as 8 fp32 lanes (x64 AVX2
 *     lowering of .NET 8 RyuJIT).  No FMA contraction (RyuJIT never contracts
 *     `acc += a*b`).
 *   - Vector.Dot(v, Vector<float>.One) is restated as the AVX lowering
 *     vdpps(0xFF)+vperm2f128+vaddps:  ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7)).
 *   - System.Random(int) is the .NET legacy subtractive generator
 *     (Net5CompatSeedImpl), see SURVEY.md Appendix A.
 *   - PriorityQueue / List.Sort tie order is unspecified by the BCL; the oracle
 *     (and the GPU engine) use the canonical rule: score descending, then
 *     storage key ascending.
 */
#ifndef PYROPE_ORACLE_H
#define PYROPE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_L2 = 0, ORC_IP = 1, ORC_COS = 2 };

/* storage keys of IVF buffer rows are ORC_BUFKEY | slot; list rows use their
 * list-major position (see DESIGN.md "Tie rule"). */
#define ORC_BUFKEY ((int64_t)1 << 31)

/* ---- System.Random (legacy) ---- */
typedef struct { int32_t sa[56]; int32_t inext, inextp; } orc_random;
void orc_random_init(orc_random *r, int32_t seed);
int32_t orc_random_next(orc_random *r);
double orc_random_next_double(orc_random *r);
/* Pyrope.Benchmarks/Program.cs:251-263 GenerateRandomVectors */
void orc_generate_vectors(int64_t count, int32_t dim, int32_t seed, float *out);

/* ---- VectorMath.cs ---- */
float orc_dot(const float *a, const float *b, int32_t n);          /* :8-37 */
float orc_l2sq(const float *a, const float *b, int32_t n);         /* :39-70 */
float orc_norm(const float *v, int32_t n);                         /* :72-100 */
float orc_cosine(const float *q, const float *v, int32_t n, float qn, float vn); /* :102-109 */
float orc_dot_unsafe(const float *a, const float *b, int32_t n);   /* :128-186 */
float orc_l2sq_unsafe(const float *a, const float *b, int32_t n);  /* :188-253 */
int64_t orc_l2sq_8bit(const uint8_t *a, const uint8_t *b, int32_t n); /* :441-564 */
int64_t orc_dot_8bit(const uint8_t *a, const uint8_t *b, int32_t n);  /* :572-681 */

/* ---- BruteForceVectorIndex.Search (:275-379), fp32 path ----
 * rows: nslots x dim (slot order), live[slot] != 0 for non-deleted slots.
 * max_scans < 0 = unlimited.  Keys = slot.  Returns #results (<= k). */
int32_t orc_bf_search(const float *rows, const uint8_t *live, int64_t nslots, int32_t dim,
                      int32_t metric, const float *q, int32_t k, int64_t max_scans,
                      float *out_scores, int64_t *out_keys);

/* ---- KMeansUtils.cs ---- */
int32_t orc_find_nearest_centroid(const float *v, const float *cents, const float *cnorms,
                                  int32_t k, int32_t dim, int32_t metric);           /* :70-93 */
int32_t orc_kmeans_train(const float *data, int64_t n, int32_t dim, int32_t k, int32_t metric,
                         int32_t max_iter, int32_t seed, float *out_centroids);     /* :10-68 */

/* ---- IvfFlatVectorIndex ----
 * Build (:85-145) on rows already in uniqueData order: trains (seed 42), assigns.
 * Returns k actually used; out_assign[i] = list of row i. */
int32_t orc_ivf_build(const float *data, int64_t n, int32_t dim, int32_t nlist, int32_t metric,
                      float *out_centroids, int32_t *out_assign);
/* Search (:147-231).  buffer: nbuf_slots x dim in Dictionary slot order with
 * buf_live; lists: list-major rows (ntot x dim) with list_off[nlist+1] and
 * row_live (0 = deleted or shadowed by a buffer id).  nprobe < 0 -> 3. */
int32_t orc_ivf_search(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                       const float *lrows, const uint8_t *row_live, const int64_t *list_off,
                       const float *cents, int32_t nlist, int32_t built, int32_t dim, int32_t metric,
                       const float *q, int32_t k, int32_t nprobe, int64_t max_scans,
                       float *out_scores, int64_t *out_keys);

/* ---- ProductQuantizer.cs / IvfPqVectorIndex.cs ---- */
/* Train (:28-58): codebooks[m][j][sub] for j < ksub_actual; returns ksub_actual. */
int32_t orc_pq_train(const float *data, int64_t n, int32_t dim, int32_t M, int32_t K, float *out_codebooks);
void orc_pq_encode(const float *v, int32_t dim, int32_t M, int32_t ksub, const float *codebooks, uint8_t *out_code); /* :60-80 */
void orc_pq_distance_table(const float *q, int32_t dim, int32_t M, int32_t ksub, const float *codebooks, float *out_table); /* :98-120 */
/* IvfPq.Build (:55-116): coarse k-means seed 123, residual PQ, encode. Returns nlist used. */
int32_t orc_ivfpq_build(const float *data, int64_t n, int32_t dim, int32_t nlist, int32_t M, int32_t K,
                        int32_t metric, float *out_centroids, int32_t *out_assign, float *out_codebooks,
                        int32_t *out_ksub, uint8_t *out_codes /* n x M, row order */);
/* IvfPq.Search (:118-212).  codes list-major (ntot x M).  nprobe < 0 -> 1. */
int32_t orc_ivfpq_search(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                         const uint8_t *codes, const uint8_t *row_live, const int64_t *list_off,
                         const float *cents, int32_t nlist, int32_t built, const float *codebooks,
                         int32_t M, int32_t ksub, int32_t dim, int32_t metric,
                         const float *q, int32_t k, int32_t nprobe,
                         float *out_scores, int64_t *out_keys);

/* ---- scalar quantization and the 8-bit search mode of BruteForceVectorIndex ---- */
void orc_scalar_quantize(const float *v, int32_t n, uint8_t *out, float *out_min, float *out_max);
int64_t orc_l2sq_8bit_net(const uint8_t *a, const uint8_t *b, int32_t n);
int64_t orc_dot_8bit_net(const uint8_t *a, const uint8_t *b, int32_t n);
int32_t orc_bf_search_sq8(const float *rows, const uint8_t *live, const uint8_t *has_q, int64_t nslots,
                          int32_t dim, int32_t metric, const float *q, int32_t k, int64_t max_scans,
                          float *out_scores, int64_t *out_keys);

/* ---- batched drivers for the CPU baseline (one query per worker thread,
 * mirroring the reference's concurrent VEC.SEARCH workers, Program.cs:363-388) ---- */
void orc_ivf_search_batch(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                          const float *lrows, const uint8_t *row_live, const int64_t *list_off,
                          const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                          const float *qs, int64_t nq, int32_t k, int32_t nprobe, int32_t nthreads,
                          float *out_scores, int64_t *out_keys, int32_t *out_counts);
int32_t orc_ivf_probe(const float *q, const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                      int32_t nprobe, int32_t *out);
int32_t orc_ivf_search_probed(const float *lrows, const int64_t *row_idx, const uint8_t *row_live,
                              const int64_t *list_off, const int32_t *probes, int32_t nprobe, int32_t dim,
                              int32_t metric, const float *q, int32_t k, float *out_scores, int64_t *out_keys);
void orc_ivf_search_batch_idx(const float *rows, const int64_t *row_idx, const uint8_t *row_live,
                              const int64_t *list_off, const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                              const float *qs, int64_t nq, int32_t k, int32_t nprobe, int32_t nthreads,
                              float *out_scores, int64_t *out_keys, int32_t *out_counts);
void orc_bf_search_batch(const float *rows, const uint8_t *live, int64_t nslots, int32_t dim,
                         int32_t metric, const float *qs, int64_t nq, int32_t k, int32_t nthreads,
                         float *out_scores, int64_t *out_keys, int32_t *out_counts);

#ifdef __cplusplus
}
#endif
#endif
