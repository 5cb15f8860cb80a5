/*
 * oracle.c -- CPU restatement of Pyrope's C# ANN scan engine.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled with
 *   gcc -O3 -mavx2 -ffp-contract=off -fno-fast-math
 * so that every fp32 operation rounds exactly once, as RyuJIT's
 * System.Numerics.Vector<float> code does (no FMA contraction).
 * Citations: paths relative to /root/reference/src/Pyrope.GarnetServer/.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#ifndef ORC_LANES
#define W 8 /* Vector<float>.Count on x64 AVX2 */
#else
#define W ORC_LANES /* liboracle_w4.so: Vector<float>.Count on Arm64 NEON (lane-width study only) */
#endif

/* ------------------------------------------------------------------ */
/* System.Random legacy generator (BCL Net5CompatSeedImpl) */
/* ------------------------------------------------------------------ */
void orc_random_init(orc_random *r, int32_t seed) {
  const int32_t MBIG = INT32_MAX, MSEED = 161803398;
  int32_t sub = (seed == INT32_MIN) ? INT32_MAX : (seed < 0 ? -seed : seed);
  int32_t mj = MSEED - sub, mk = 1;
  r->sa[55] = mj;
  for (int i = 1; i < 55; i++) {
    int ii = (21 * i) % 55;
    r->sa[ii] = mk;
    mk = mj - mk;
    if (mk < 0) mk += MBIG;
    mj = r->sa[ii];
  }
  for (int pass = 1; pass < 5; pass++)
    for (int i = 1; i < 56; i++) {
      r->sa[i] -= r->sa[1 + (i + 30) % 55];
      if (r->sa[i] < 0) r->sa[i] += MBIG;
    }
  r->inext = 0;
  r->inextp = 21;
}

static inline int32_t internal_sample(orc_random *r) {
  int32_t a = r->inext, b = r->inextp;
  if (++a >= 56) a = 1;
  if (++b >= 56) b = 1;
  int32_t ret = r->sa[a] - r->sa[b];
  if (ret == INT32_MAX) ret--;
  if (ret < 0) ret += INT32_MAX;
  r->sa[a] = ret;
  r->inext = a;
  r->inextp = b;
  return ret;
}

int32_t orc_random_next(orc_random *r) { return internal_sample(r); }
double orc_random_next_double(orc_random *r) { return internal_sample(r) * (1.0 / INT32_MAX); }

/* Program.cs:251-263: v[d] = (float)rng.NextDouble(), rows in order. */
void orc_generate_vectors(int64_t count, int32_t dim, int32_t seed, float *out) {
  orc_random r;
  orc_random_init(&r, seed);
  for (int64_t i = 0; i < count * (int64_t)dim; i++) out[i] = (float)orc_random_next_double(&r);
}

/* ------------------------------------------------------------------ */
/* VectorMath.cs                                                        */
/* ------------------------------------------------------------------ */
/* Vector.Dot(v, One): AVX vdpps per 128-bit half, then add halves (W = 8); the 4-lane NEON
 * form (faddp pairwise adds) for the lane-width study. */
static inline float hsum8(const float v[W]) {
#if W == 8
  float lo = (v[0] + v[1]) + (v[2] + v[3]);
  float hi = (v[4] + v[5]) + (v[6] + v[7]);
  return lo + hi;
#else
  return (v[0] + v[1]) + (v[2] + v[3]);
#endif
}

/* VectorMath.cs:8-37  DotProduct: one Vector accumulator. */
float orc_dot(const float *a, const float *b, int32_t n) {
  int32_t i = 0;
  float sum = 0.0f;
  if (n >= W) {
    float acc[W] = {0};
    for (; i <= n - W; i += W)
      for (int l = 0; l < W; l++) acc[l] = acc[l] + a[i + l] * b[i + l];
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + a[i] * b[i];
  return sum;
}

/* VectorMath.cs:39-70  L2Squared: diff = a - b; vSum += diff*diff. */
float orc_l2sq(const float *a, const float *b, int32_t n) {
  int32_t i = 0;
  float sum = 0.0f;
  if (n >= W) {
    float acc[W] = {0};
    for (; i <= n - W; i += W)
      for (int l = 0; l < W; l++) {
        float d = a[i + l] - b[i + l];
        acc[l] = acc[l] + d * d;
      }
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) {
    float d = a[i] - b[i];
    sum = sum + d * d;
  }
  return sum;
}

/* VectorMath.cs:72-100  ComputeNorm = MathF.Sqrt(sum of squares). */
float orc_norm(const float *v, int32_t n) {
  int32_t i = 0;
  float sum = 0.0f;
  if (n >= W) {
    float acc[W] = {0};
    for (; i <= n - W; i += W)
      for (int l = 0; l < W; l++) acc[l] = acc[l] + v[i + l] * v[i + l];
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + v[i] * v[i];
  return sqrtf(sum);
}

/* VectorMath.cs:102-109  Cosine(q, v, qn, vn). */
float orc_cosine(const float *q, const float *v, int32_t n, float qn, float vn) {
  if (qn < 1e-6f || vn < 1e-6f) return 0.0f;
  float dot = orc_dot(q, v, n);
  return dot / (qn * vn);
}

/* VectorMath.cs:128-186  DotProductUnsafe: 4 accumulators, remainder, tail. */
float orc_dot_unsafe(const float *a, const float *b, int32_t n) {
  int32_t i = 0;
  float sum = 0.0f;
  if (n >= 4 * W) {
    float a1[W] = {0}, a2[W] = {0}, a3[W] = {0}, a4[W] = {0}, fin[W];
    for (; i <= n - 4 * W; i += 4 * W)
      for (int l = 0; l < W; l++) {
        a1[l] = a1[l] + a[i + l] * b[i + l];
        a2[l] = a2[l] + a[i + W + l] * b[i + W + l];
        a3[l] = a3[l] + a[i + 2 * W + l] * b[i + 2 * W + l];
        a4[l] = a4[l] + a[i + 3 * W + l] * b[i + 3 * W + l];
      }
    for (int l = 0; l < W; l++) fin[l] = ((a1[l] + a2[l]) + a3[l]) + a4[l];
    sum = sum + hsum8(fin);
  }
  if (i <= n - W) {
    float acc[W] = {0};
    for (; i <= n - W; i += W)
      for (int l = 0; l < W; l++) acc[l] = acc[l] + a[i + l] * b[i + l];
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + a[i] * b[i];
  return sum;
}

/* VectorMath.cs:188-253  L2SquaredUnsafe. */
float orc_l2sq_unsafe(const float *a, const float *b, int32_t n) {
  int32_t i = 0;
  float sum = 0.0f;
  if (n >= 4 * W) {
    float a1[W] = {0}, a2[W] = {0}, a3[W] = {0}, a4[W] = {0}, fin[W];
    for (; i <= n - 4 * W; i += 4 * W)
      for (int l = 0; l < W; l++) {
        float d1 = a[i + l] - b[i + l];
        float d2 = a[i + W + l] - b[i + W + l];
        float d3 = a[i + 2 * W + l] - b[i + 2 * W + l];
        float d4 = a[i + 3 * W + l] - b[i + 3 * W + l];
        a1[l] = a1[l] + d1 * d1;
        a2[l] = a2[l] + d2 * d2;
        a3[l] = a3[l] + d3 * d3;
        a4[l] = a4[l] + d4 * d4;
      }
    for (int l = 0; l < W; l++) fin[l] = ((a1[l] + a2[l]) + a3[l]) + a4[l];
    sum = sum + hsum8(fin);
  }
  if (i <= n - W) {
    float acc[W] = {0};
    for (; i <= n - W; i += W)
      for (int l = 0; l < W; l++) {
        float d = a[i + l] - b[i + l];
        acc[l] = acc[l] + d * d;
      }
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) {
    float d = a[i] - b[i];
    sum = sum + d * d;
  }
  return sum;
}

/* VectorMath.cs:441-564 / 572-681: exact integer sums (order irrelevant). */
int64_t orc_l2sq_8bit(const uint8_t *a, const uint8_t *b, int32_t n) {
  int64_t s = 0;
  for (int32_t i = 0; i < n; i++) {
    int64_t d = (int64_t)a[i] - (int64_t)b[i];
    s += d * d;
  }
  return s;
}
int64_t orc_dot_8bit(const uint8_t *a, const uint8_t *b, int32_t n) {
  int64_t s = 0;
  for (int32_t i = 0; i < n; i++) s += (int64_t)a[i] * (int64_t)b[i];
  return s;
}

/* ------------------------------------------------------------------ */
/* top-k (PriorityQueue min-heap + final Sort desc; canonical ties)     */
/* ------------------------------------------------------------------ */
typedef struct {
  float s;
  int64_t key;
} cand;

static inline int better(float s1, int64_t k1, float s2, int64_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

static inline void topk_push(cand *h, int32_t *cnt, int32_t k, float s, int64_t key) {
  int32_t n = *cnt;
  if (n == k) {
    if (!better(s, key, h[k - 1].s, h[k - 1].key)) return;
    n = k - 1;
  }
  int32_t j = n;
  while (j > 0 && better(s, key, h[j - 1].s, h[j - 1].key)) {
    h[j] = h[j - 1];
    j--;
  }
  h[j].s = s;
  h[j].key = key;
  *cnt = n + 1;
}

static int32_t topk_emit(const cand *h, int32_t cnt, float *os, int64_t *ok) {
  for (int32_t i = 0; i < cnt; i++) {
    os[i] = h[i].s;
    ok[i] = h[i].key;
  }
  return cnt;
}

/* ------------------------------------------------------------------ */
/* BruteForceVectorIndex.Search (BruteForceVectorIndex.cs:275-379)      */
/* ------------------------------------------------------------------ */
int32_t orc_bf_search(const float *rows, const uint8_t *live, int64_t nslots, int32_t dim,
                      int32_t metric, const float *q, int32_t k, int64_t max_scans,
                      float *out_scores, int64_t *out_keys) {
  if (k <= 0 || nslots == 0) return 0;                                   /* :278, :285 */
  int64_t scan_limit = (max_scans >= 0 && max_scans < nslots) ? max_scans : nslots; /* :288 */
  if (scan_limit <= 0) return 0;                                         /* :289 */
  cand *h = (cand *)malloc(sizeof(cand) * (size_t)k);
  int32_t cnt = 0;
  int64_t scanned = 0;
  float qn = metric == ORC_COS ? orc_norm(q, dim) : 0.0f;                /* :339 */
  for (int64_t i = 0; i < nslots; i++) {
    if (!live[i]) continue;                                              /* :343 */
    if (scanned >= scan_limit) break;                                    /* :344 */
    scanned++;
    const float *x = rows + i * (int64_t)dim;
    float s;
    if (metric == ORC_L2) s = -orc_l2sq_unsafe(q, x, dim);              /* :352 */
    else if (metric == ORC_IP) s = orc_dot_unsafe(q, x, dim);           /* :353 */
    else {                                                               /* :354, norm cached at Add :146 */
      float n = orc_norm(x, dim);
      s = (qn < 1e-6f || n < 1e-6f) ? 0.0f : orc_dot_unsafe(q, x, dim) / (qn * n);
    }
    topk_push(h, &cnt, k, s, i);
  }
  int32_t r = topk_emit(h, cnt, out_scores, out_keys);
  free(h);
  return r;
}

/* ------------------------------------------------------------------ */
/* Scalar quantization (ScalarQuantizer.cs) and the 8-bit search mode   */
/* of BruteForceVectorIndex (EnableQuantization, :25-40, :166-178,      */
/* :200-211, :296-336).                                                  */
/* ------------------------------------------------------------------ */
/* (int)Math.Round(double) as .NET 8 on x64 evaluates it: banker's rounding, and the
 * cvttsd2si "integer indefinite" (int.MinValue) for NaN and out-of-range values. */
static int32_t net_round_to_int(float v) {
  double r = nearbyint((double)v); /* default rounding mode: to nearest, ties to even */
  if (!(r >= -2147483648.0 && r < 2147483648.0)) return INT32_MIN;
  return (int32_t)r;
}

/* ScalarQuantizer.Quantize(ReadOnlySpan<float>, Span<byte>, out min, out max) :23-62 */
void orc_scalar_quantize(const float *v, int32_t n, uint8_t *out, float *out_min, float *out_max) {
  if (n == 0) {
    *out_min = 0.0f;
    *out_max = 0.0f;
    return;
  }
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (int32_t i = 0; i < n; i++) {
    if (v[i] < mn) mn = v[i];
    if (v[i] > mx) mx = v[i];
  }
  *out_min = mn;
  *out_max = mx;
  float range = mx - mn;
  if (range == 0.0f) {
    memset(out, 0, (size_t)n);
    return;
  }
  float scale = 255.0f / range;
  for (int32_t i = 0; i < n; i++) {
    float normalized = (v[i] - mn) * scale;
    int32_t r = net_round_to_int(normalized);
    out[i] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r)); /* Math.Clamp(.., 0, 255) */
  }
}

/* VectorMath.L2Squared8Bit / DotProduct8Bit exactly as the x64 SIMD path computes them:
 * for n >= 32 (Vector<byte>.Count) the first n - n % 32 terms are summed in int32 lanes and
 * reduced with Vector.Dot in int32 (wrapping modulo 2^32), the scalar tail in long. */
static int64_t sq8_combine(uint32_t simd, int64_t tail) { return (int64_t)(int32_t)simd + tail; }
int64_t orc_l2sq_8bit_net(const uint8_t *a, const uint8_t *b, int32_t n) {
  int32_t sl = n >= 32 ? n - n % 32 : 0;
  uint32_t s = 0;
  int64_t t = 0;
  for (int32_t i = 0; i < n; i++) {
    int32_t d = (int32_t)a[i] - (int32_t)b[i];
    if (i < sl) s += (uint32_t)(d * d);
    else t += d * d;
  }
  return sq8_combine(s, t);
}
int64_t orc_dot_8bit_net(const uint8_t *a, const uint8_t *b, int32_t n) {
  int32_t sl = n >= 32 ? n - n % 32 : 0;
  uint32_t s = 0;
  int64_t t = 0;
  for (int32_t i = 0; i < n; i++) {
    if (i < sl) s += (uint32_t)a[i] * (uint32_t)b[i];
    else t += (int64_t)a[i] * (int64_t)b[i];
  }
  return sq8_combine(s, t);
}

/* BruteForceVectorIndex.Search with EnableQuantization (:296-336).  has_q[i] = 0 for rows
 * written while quantization was off (empty quantized data: counted as scanned, skipped). */
int32_t orc_bf_search_sq8(const float *rows, const uint8_t *live, const uint8_t *has_q, int64_t nslots,
                          int32_t dim, int32_t metric, const float *q, int32_t k, int64_t max_scans,
                          float *out_scores, int64_t *out_keys) {
  if (k <= 0 || nslots == 0) return 0;
  int64_t scan_limit = (max_scans >= 0 && max_scans < nslots) ? max_scans : nslots;
  if (scan_limit <= 0) return 0;
  uint8_t *qq = (uint8_t *)malloc((size_t)dim + 1), *xq = (uint8_t *)malloc((size_t)dim + 1);
  float mn, mx;
  orc_scalar_quantize(q, dim, qq, &mn, &mx); /* :304 */
  cand *h = (cand *)malloc(sizeof(cand) * (size_t)k);
  int32_t cnt = 0;
  int64_t scanned = 0;
  for (int64_t i = 0; i < nslots; i++) {
    if (!live[i]) continue;           /* :308 */
    if (scanned >= scan_limit) break; /* :309 */
    scanned++;
    if (!has_q[i]) continue;          /* :314 */
    orc_scalar_quantize(rows + i * (int64_t)dim, dim, xq, &mn, &mx);
    int64_t v = metric == ORC_L2 ? -orc_l2sq_8bit_net(qq, xq, dim) : orc_dot_8bit_net(qq, xq, dim); /* :325-331 */
    topk_push(h, &cnt, k, (float)v, i);
  }
  int32_t r = topk_emit(h, cnt, out_scores, out_keys);
  free(h);
  free(qq);
  free(xq);
  return r;
}

/* ------------------------------------------------------------------ */
/* KMeansUtils.cs                                                       */
/* ------------------------------------------------------------------ */
/* :70-93 FindNearestCentroid: strict '>' from float.MinValue -> lowest index on ties. */
int32_t orc_find_nearest_centroid(const float *v, const float *cents, const float *cnorms,
                                  int32_t k, int32_t dim, int32_t metric) {
  int32_t best = 0;
  float best_s = -FLT_MAX;
  float vn = metric == ORC_COS ? orc_norm(v, dim) : 0.0f;
  for (int32_t i = 0; i < k; i++) {
    const float *c = cents + (int64_t)i * dim;
    float s;
    if (metric == ORC_L2) s = -orc_l2sq(v, c, dim);
    else if (metric == ORC_IP) s = orc_dot(v, c, dim);
    else s = orc_cosine(v, c, dim, vn, cnorms[i]);
    if (s > best_s) {
      best_s = s;
      best = i;
    }
  }
  return best;
}

typedef struct {
  int32_t key;
  int64_t idx;
} keyidx;
static int cmp_keyidx(const void *a, const void *b) {
  const keyidx *x = (const keyidx *)a, *y = (const keyidx *)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx ? 1 : 0); /* LINQ OrderBy is stable */
}

/* :10-68 Train. */
int32_t orc_kmeans_train(const float *data, int64_t n, int32_t dim, int32_t k, int32_t metric,
                         int32_t max_iter, int32_t seed, float *out) {
  if (n == 0) return 0;                                   /* :12 */
  if (k <= 0) k = 1;                                      /* :13 */
  if (k > n) k = (int32_t)n;                              /* :14 */
  orc_random r;
  orc_random_init(&r, seed);
  keyidx *ki = (keyidx *)malloc(sizeof(keyidx) * (size_t)n);
  for (int64_t i = 0; i < n; i++) {                       /* :20 OrderBy(_ => rnd.Next()) */
    ki[i].key = orc_random_next(&r);
    ki[i].idx = i;
  }
  qsort(ki, (size_t)n, sizeof(keyidx), cmp_keyidx);
  for (int32_t c = 0; c < k; c++) memcpy(out + (int64_t)c * dim, data + ki[c].idx * dim, sizeof(float) * (size_t)dim);
  free(ki);

  int32_t *assign = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
  int64_t *count = (int64_t *)malloc(sizeof(int64_t) * (size_t)k);
  float *sums = (float *)malloc(sizeof(float) * (size_t)k * dim);
  float *cn = (float *)malloc(sizeof(float) * (size_t)k);
  for (int32_t it = 0; it < max_iter; it++) {             /* :22 */
    for (int32_t c = 0; c < k; c++) cn[c] = metric == ORC_COS ? orc_norm(out + (int64_t)c * dim, dim) : 0.0f; /* :30 */
    for (int64_t i = 0; i < n; i++)                       /* :34-38 */
      assign[i] = orc_find_nearest_centroid(data + i * dim, out, cn, k, dim, metric);
    memset(count, 0, sizeof(int64_t) * (size_t)k);
    memset(sums, 0, sizeof(float) * (size_t)k * dim);
    for (int64_t i = 0; i < n; i++) {                     /* :40-43 members in data order */
      float *s = sums + (int64_t)assign[i] * dim;
      const float *x = data + i * dim;
      for (int32_t d = 0; d < dim; d++) s[d] = s[d] + x[d]; /* :51-54 */
      count[assign[i]]++;
    }
    int changed = 0;
    for (int32_t c = 0; c < k; c++) {                     /* :46-62 */
      if (count[c] == 0) continue;
      float *s = sums + (int64_t)c * dim;
      float cntf = (float)count[c];
      for (int32_t d = 0; d < dim; d++) s[d] = s[d] / cntf; /* :55 */
      float *old = out + (int64_t)c * dim;
      int eq = 1;                                         /* ArraysEqual :95-101 */
      for (int32_t d = 0; d < dim; d++)
        if ((double)fabsf(old[d] - s[d]) > 1e-6) { eq = 0; break; }
      if (!eq) {
        memcpy(old, s, sizeof(float) * (size_t)dim);
        changed = 1;
      }
    }
    if (!changed) break;                                  /* :64 */
  }
  free(assign);
  free(count);
  free(sums);
  free(cn);
  return k;
}

/* ------------------------------------------------------------------ */
/* IvfFlatVectorIndex                                                   */
/* ------------------------------------------------------------------ */
/* Build :111-132 on rows in uniqueData order. */
int32_t orc_ivf_build(const float *data, int64_t n, int32_t dim, int32_t nlist, int32_t metric,
                      float *out_centroids, int32_t *out_assign) {
  if (n == 0) return 0;
  int32_t k = nlist < n ? nlist : (int32_t)n;
  if (k <= 0) k = 1;
  k = orc_kmeans_train(data, n, dim, k, metric, 10, 42, out_centroids);
  float *cn = (float *)malloc(sizeof(float) * (size_t)k);
  for (int32_t c = 0; c < k; c++) cn[c] = metric == ORC_COS ? orc_norm(out_centroids + (int64_t)c * dim, dim) : 0.0f;
  for (int64_t i = 0; i < n; i++)
    out_assign[i] = orc_find_nearest_centroid(data + i * dim, out_centroids, cn, k, dim, metric);
  free(cn);
  return k;
}

/* IvfFlatVectorIndex.cs:351-360 ComputeScore (safe VectorMath). */
static inline float ivf_score(const float *q, const float *x, int32_t dim, int32_t metric, float qn, float xn) {
  if (metric == ORC_L2) return -orc_l2sq(q, x, dim);
  if (metric == ORC_IP) return orc_dot(q, x, dim);
  return orc_cosine(q, x, dim, qn, xn);
}

typedef struct {
  float s;
  int32_t idx;
} cscore;
static int cmp_cscore(const void *a, const void *b) {
  const cscore *x = (const cscore *)a, *y = (const cscore *)b;
  if (x->s != y->s) return x->s > y->s ? -1 : 1; /* descending (:196) */
  return x->idx < y->idx ? -1 : (x->idx > y->idx ? 1 : 0);
}

/* coarse scoring + sort (IvfFlatVectorIndex.cs:186-196, IvfPqVectorIndex.cs:141-148) */
static cscore *coarse_rank(const float *q, const float *cents, int32_t nlist, int32_t dim, int32_t metric, float qn) {
  cscore *cs = (cscore *)malloc(sizeof(cscore) * (size_t)nlist);
  for (int32_t i = 0; i < nlist; i++) {
    const float *c = cents + (int64_t)i * dim;
    float cnorm = metric == ORC_COS ? orc_norm(c, dim) : 0.0f;
    cs[i].s = ivf_score(q, c, dim, metric, qn, cnorm);
    cs[i].idx = i;
  }
  qsort(cs, (size_t)nlist, sizeof(cscore), cmp_cscore);
  return cs;
}

/* Search :147-231 */
int32_t orc_ivf_search(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                       const float *lrows, const uint8_t *row_live, const int64_t *list_off,
                       const float *cents, int32_t nlist, int32_t built, int32_t dim, int32_t metric,
                       const float *q, int32_t k, int32_t nprobe, int64_t max_scans,
                       float *out_scores, int64_t *out_keys) {
  if (k <= 0) return 0;
  if (nprobe < 0) nprobe = 3;                                   /* :14, :151 */
  int64_t maxs = max_scans < 0 ? (int64_t)INT32_MAX : max_scans; /* :152 */
  cand *h = (cand *)malloc(sizeof(cand) * (size_t)k);
  int32_t cnt = 0;
  int64_t scanned = 0;
  float qn = metric == ORC_COS ? orc_norm(q, dim) : 0.0f;       /* :167 */
  for (int64_t s = 0; s < nbuf_slots; s++) {                    /* :170-180 */
    if (!buf_live[s]) continue;
    if (scanned >= maxs) break;
    scanned++;
    const float *x = buf + s * dim;
    float xn = metric == ORC_COS ? orc_norm(x, dim) : 0.0f;
    topk_push(h, &cnt, k, ivf_score(q, x, dim, metric, qn, xn), ORC_BUFKEY | s);
  }
  if (built && nlist > 0 && scanned < maxs) {                   /* :183 */
    cscore *cs = coarse_rank(q, cents, nlist, dim, metric, qn);
    int32_t probes = nprobe < nlist ? nprobe : nlist;           /* :198 */
    for (int32_t p = 0; p < probes; p++) {
      if (scanned >= maxs) break;                               /* :202 */
      int32_t l = cs[p].idx;
      for (int64_t pos = list_off[l]; pos < list_off[l + 1]; pos++) {
        if (scanned >= maxs) break;                             /* :209 */
        if (!row_live[pos]) continue;                           /* :210 (seen) / removed rows */
        scanned++;
        const float *x = lrows + pos * dim;
        float xn = metric == ORC_COS ? orc_norm(x, dim) : 0.0f;
        topk_push(h, &cnt, k, ivf_score(q, x, dim, metric, qn, xn), pos);
      }
    }
    free(cs);
  }
  int32_t r = topk_emit(h, cnt, out_scores, out_keys);
  free(h);
  return r;
}

/* The coarse ranking alone (:186-198): the first min(nprobe, nlist) list ids in rank order.
 * The multi-GPU step ranks each query once and hands the lists to every shard. */
int32_t orc_ivf_probe(const float *q, const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                      int32_t nprobe, int32_t *out) {
  if (nprobe < 0) nprobe = 3; /* :14, :151 */
  int32_t probes = nprobe < nlist ? nprobe : nlist;
  if (probes <= 0) return 0;
  float qn = metric == ORC_COS ? orc_norm(q, dim) : 0.0f;
  cscore *cs = coarse_rank(q, cents, nlist, dim, metric, qn);
  for (int32_t p = 0; p < probes; p++) out[p] = cs[p].idx;
  free(cs);
  return probes;
}

/* The list scan of Search (:200-218) over caller-ranked lists (built index, empty buffer, no
 * MaxScans).  Row pos of the list-major store is lrows[row_idx ? row_idx[pos] : pos], so a
 * caller can pass base rows plus the layout's labels instead of a list-major copy. */
int32_t orc_ivf_search_probed(const float *lrows, const int64_t *row_idx, const uint8_t *row_live,
                              const int64_t *list_off, const int32_t *probes, int32_t nprobe, int32_t dim,
                              int32_t metric, const float *q, int32_t k, float *out_scores, int64_t *out_keys) {
  if (k <= 0) return 0;
  cand *h = (cand *)malloc(sizeof(cand) * (size_t)k);
  int32_t cnt = 0;
  float qn = metric == ORC_COS ? orc_norm(q, dim) : 0.0f;
  for (int32_t p = 0; p < nprobe; p++) {
    int32_t l = probes[p];
    if (l < 0) continue;
    for (int64_t pos = list_off[l]; pos < list_off[l + 1]; pos++) {
      if (row_live && !row_live[pos]) continue;
      const float *x = lrows + (row_idx ? row_idx[pos] : pos) * dim;
      float xn = metric == ORC_COS ? orc_norm(x, dim) : 0.0f;
      topk_push(h, &cnt, k, ivf_score(q, x, dim, metric, qn, xn), pos);
    }
  }
  int32_t r = topk_emit(h, cnt, out_scores, out_keys);
  free(h);
  return r;
}

/* ------------------------------------------------------------------ */
/* ProductQuantizer.cs                                                  */
/* ------------------------------------------------------------------ */
/* :28-58 Train: per-subspace k-means, L2, 10 iterations, seed 42+m. */
int32_t orc_pq_train(const float *data, int64_t n, int32_t dim, int32_t M, int32_t K, float *out_codebooks) {
  int32_t sub = dim / M;
  if (n == 0) return 0;
  float *sd = (float *)malloc(sizeof(float) * (size_t)n * sub);
  int32_t ksub = 0;
  for (int32_t m = 0; m < M; m++) {
    for (int64_t i = 0; i < n; i++) memcpy(sd + i * sub, data + i * dim + (int64_t)m * sub, sizeof(float) * (size_t)sub);
    int32_t kk = (int32_t)(K < n ? K : n);
    if (kk <= 0) kk = 1;
    ksub = orc_kmeans_train(sd, n, sub, K, ORC_L2, 10, 42 + m, out_codebooks + (int64_t)m * kk * sub);
  }
  free(sd);
  return ksub;
}

/* :60-80 Encode + :122-136 FindNearest (strict '<' from float.MaxValue). */
void orc_pq_encode(const float *v, int32_t dim, int32_t M, int32_t ksub, const float *cb, uint8_t *code) {
  int32_t sub = dim / M;
  for (int32_t m = 0; m < M; m++) {
    float mind = FLT_MAX;
    int32_t best = 0;
    for (int32_t j = 0; j < ksub; j++) {
      float d = orc_l2sq_unsafe(v + (int64_t)m * sub, cb + ((int64_t)m * ksub + j) * sub, sub);
      if (d < mind) {
        mind = d;
        best = j;
      }
    }
    code[m] = (uint8_t)best;
  }
}

/* :98-120 ComputeDistanceTable: table[m][j] = L2SquaredUnsafe(q_m, C_mj). */
void orc_pq_distance_table(const float *q, int32_t dim, int32_t M, int32_t ksub, const float *cb, float *t) {
  int32_t sub = dim / M;
  for (int32_t m = 0; m < M; m++)
    for (int32_t j = 0; j < ksub; j++)
      t[(int64_t)m * ksub + j] = orc_l2sq_unsafe(q + (int64_t)m * sub, cb + ((int64_t)m * ksub + j) * sub, sub);
}

/* IvfPqVectorIndex.cs:55-116 Build. */
int32_t orc_ivfpq_build(const float *data, int64_t n, int32_t dim, int32_t nlist, int32_t M, int32_t K,
                        int32_t metric, float *cents, int32_t *assign, float *cb, int32_t *out_ksub,
                        uint8_t *codes) {
  if (n == 0) return 0;
  int32_t nc = nlist < n ? nlist : (int32_t)n;                    /* :68 */
  nc = orc_kmeans_train(data, n, dim, nc, metric, 10, 123, cents); /* :69 */
  float *cn = (float *)malloc(sizeof(float) * (size_t)nc);
  for (int32_t c = 0; c < nc; c++) cn[c] = metric == ORC_COS ? orc_norm(cents + (int64_t)c * dim, dim) : 0.0f;
  float *res = (float *)malloc(sizeof(float) * (size_t)n * dim);
  for (int64_t i = 0; i < n; i++) {                               /* :76-86 */
    const float *v = data + i * dim;
    int32_t c = orc_find_nearest_centroid(v, cents, cn, nc, dim, metric);
    assign[i] = c;
    for (int32_t d = 0; d < dim; d++) res[i * dim + d] = v[d] - cents[(int64_t)c * dim + d];
  }
  int32_t ksub = orc_pq_train(res, n, dim, M, K, cb);             /* :89 */
  *out_ksub = ksub;
  for (int64_t i = 0; i < n; i++) orc_pq_encode(res + i * dim, dim, M, ksub, cb, codes + i * M); /* :99-107 */
  free(res);
  free(cn);
  return nc;
}

/* IvfPqVectorIndex.cs:118-224 Search. */
int32_t orc_ivfpq_search(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                         const uint8_t *codes, const uint8_t *row_live, const int64_t *list_off,
                         const float *cents, int32_t nlist, int32_t built, const float *cb,
                         int32_t M, int32_t ksub, int32_t dim, int32_t metric,
                         const float *q, int32_t k, int32_t nprobe, float *out_scores, int64_t *out_keys) {
  if (k <= 0) return 0;
  if (nprobe < 0) nprobe = 1;                                     /* :125 */
  cand *h = (cand *)malloc(sizeof(cand) * (size_t)k);
  int32_t cnt = 0;
  float qn = metric == ORC_COS ? orc_norm(q, dim) : 0.0f;         /* :127 */
  for (int64_t s = 0; s < nbuf_slots; s++) {                      /* :130-136 */
    if (!buf_live[s]) continue;
    const float *x = buf + s * dim;
    float xn = metric == ORC_COS ? orc_norm(x, dim) : 0.0f;       /* :216 */
    topk_push(h, &cnt, k, ivf_score(q, x, dim, metric, qn, xn), ORC_BUFKEY | s);
  }
  if (built && nlist > 0) {
    cscore *cs = coarse_rank(q, cents, nlist, dim, metric, qn);   /* :141-148 */
    int32_t probes = nprobe < nlist ? nprobe : nlist;             /* :150 */
    float *res = (float *)malloc(sizeof(float) * (size_t)dim);
    float *tab = (float *)malloc(sizeof(float) * (size_t)M * ksub);
    for (int32_t p = 0; p < probes; p++) {
      int32_t l = cs[p].idx;
      if (list_off[l + 1] == list_off[l]) continue;               /* :157 */
      const float *c = cents + (int64_t)l * dim;
      for (int32_t d = 0; d < dim; d++) res[d] = q[d] - c[d];      /* :161-163 */
      orc_pq_distance_table(res, dim, M, ksub, cb, tab);          /* :166 */
      for (int64_t pos = list_off[l]; pos < list_off[l + 1]; pos++) {
        if (!row_live[pos]) continue;                             /* :170 */
        const uint8_t *code = codes + pos * M;
        float dist = 0.0f;
        for (int32_t m = 0; m < M; m++) dist = dist + tab[(int64_t)m * ksub + code[m]]; /* :182-186 */
        topk_push(h, &cnt, k, -dist, pos);                        /* :194 */
      }
    }
    free(res);
    free(tab);
    free(cs);
  }
  int32_t r = topk_emit(h, cnt, out_scores, out_keys);
  free(h);
  return r;
}

/* ------------------------------------------------------------------ */
/* batched CPU-baseline drivers                                         */
/* ------------------------------------------------------------------ */
typedef struct {
  int kind; /* 0 = ivf, 1 = bf */
  const float *buf;
  const uint8_t *buf_live;
  int64_t nbuf;
  const float *lrows;
  const uint8_t *row_live;
  const int64_t *list_off;
  const float *cents;
  int32_t nlist, dim, metric, k, nprobe;
  const float *qs;
  int64_t nq;
  float *os;
  int64_t *ok;
  int32_t *oc;
  int32_t tid, nthreads;
  const int64_t *row_idx; /* kind 2 */
} batch_arg;

static void *batch_worker(void *p) {
  batch_arg *a = (batch_arg *)p;
  int32_t *pr = a->kind == 2 ? (int32_t *)malloc(sizeof(int32_t) * (size_t)(a->nprobe > 0 ? a->nprobe : 1)) : NULL;
  for (int64_t i = a->tid; i < a->nq; i += a->nthreads) {
    const float *q = a->qs + i * a->dim;
    if (a->kind == 2) { /* Search with rows through row_idx: probe, then the list scan */
      int32_t np = orc_ivf_probe(q, a->cents, a->nlist, a->dim, a->metric, a->nprobe, pr);
      a->oc[i] = orc_ivf_search_probed(a->lrows, a->row_idx, a->row_live, a->list_off, pr, np, a->dim, a->metric, q,
                                       a->k, a->os + i * a->k, a->ok + i * a->k);
    } else if (a->kind == 0)
      a->oc[i] = orc_ivf_search(a->buf, a->buf_live, a->nbuf, a->lrows, a->row_live, a->list_off, a->cents,
                                a->nlist, 1, a->dim, a->metric, q, a->k, a->nprobe, -1,
                                a->os + i * a->k, a->ok + i * a->k);
    else
      a->oc[i] = orc_bf_search(a->lrows, a->row_live, a->nbuf, a->dim, a->metric, q, a->k, -1,
                               a->os + i * a->k, a->ok + i * a->k);
  }
  free(pr);
  return NULL;
}

static void run_batch(batch_arg *tmpl, int32_t nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  batch_arg *args = (batch_arg *)malloc(sizeof(batch_arg) * (size_t)nthreads);
  for (int32_t t = 0; t < nthreads; t++) {
    args[t] = *tmpl;
    args[t].tid = t;
    args[t].nthreads = nthreads;
    pthread_create(&th[t], NULL, batch_worker, &args[t]);
  }
  for (int32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(args);
}

void orc_ivf_search_batch(const float *buf, const uint8_t *buf_live, int64_t nbuf_slots,
                          const float *lrows, const uint8_t *row_live, const int64_t *list_off,
                          const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                          const float *qs, int64_t nq, int32_t k, int32_t nprobe, int32_t nthreads,
                          float *out_scores, int64_t *out_keys, int32_t *out_counts) {
  batch_arg a = {0, buf, buf_live, nbuf_slots, lrows, row_live, list_off, cents, nlist, dim, metric, k, nprobe,
                 qs, nq, out_scores, out_keys, out_counts, 0, 1, NULL};
  run_batch(&a, nthreads);
}

/* orc_ivf_search_batch over base rows + the layout's row index (rows[row_idx[pos]] is list-major
 * position pos), built index, empty buffer: one query per worker thread. */
void orc_ivf_search_batch_idx(const float *rows, const int64_t *row_idx, const uint8_t *row_live,
                              const int64_t *list_off, const float *cents, int32_t nlist, int32_t dim, int32_t metric,
                              const float *qs, int64_t nq, int32_t k, int32_t nprobe, int32_t nthreads,
                              float *out_scores, int64_t *out_keys, int32_t *out_counts) {
  batch_arg a = {2, NULL, NULL, 0, rows, row_live, list_off, cents, nlist, dim, metric, k, nprobe,
                 qs, nq, out_scores, out_keys, out_counts, 0, 1, row_idx};
  run_batch(&a, nthreads);
}

void orc_bf_search_batch(const float *rows, const uint8_t *live, int64_t nslots, int32_t dim,
                         int32_t metric, const float *qs, int64_t nq, int32_t k, int32_t nthreads,
                         float *out_scores, int64_t *out_keys, int32_t *out_counts) {
  batch_arg a = {1, NULL, NULL, nslots, rows, live, NULL, NULL, 0, dim, metric, k, 0,
                 qs, nq, out_scores, out_keys, out_counts, 0, 1, NULL};
  run_batch(&a, nthreads);
}
