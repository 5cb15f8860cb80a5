// filter.hip -- the certified exact refine of the stream scan's candidates (gfx950), plus the small
// kernels around it (unit rows, query gathers, row norms, per-list norm maxima).
//
// The reference's scores are fixed fp32 operation sequences (VectorMath.cs): sub, mul, add per element,
// 8-lane Vector accumulators and a horizontal tree.  The stream scan (scan.hip) ranks rows by fp16
// matrix-core scores with a per-row error bound; refine_kernel takes each query's best 64 of those,
// re-scores them with the reference's exact arithmetic (the same restatement as the exact scan and the
// oracle), ranks them by (score desc, key asc), and certifies the top-k: every row it did not see scored
// at most s~_K1 + E, so if the k-th exact score beats that no excluded row can enter the top-k and the
// result equals the exact scan's.  Queries whose certificate fails are listed and re-run exactly on
// the device (kernels.hip ivf_rerun_*).
//
// (Rounds 1-3 also kept an fp32 / bf16x3 MFMA filter here and an fp16 tile filter in filter16.hip;
// the stream scan superseded both and round 4 removed them.)
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace pyr {
namespace {

#include "candmerge.h"
#include "deeprank.h"

__device__ __forceinline__ bool better(float s1, uint32_t k1, float s2, uint32_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

__device__ __forceinline__ size_t blk_off(int64_t r, int d, int D) {
  return ((size_t)(r >> 3) * (size_t)D + (size_t)d) * 8 + (size_t)(r & 7);
}

// ---------------------------------------------------------------------------
// Exact restatements (VectorMath.cs) for the refine step -- the operation order of
// kernels.hip em_* and oracle/oracle.c, on one blocked-store row.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float hsum8(const float *v) {
  float lo = (v[0] + v[1]) + (v[2] + v[3]);
  float hi = (v[4] + v[5]) + (v[6] + v[7]);
  return lo + hi;
}

// V = 1: L2Squared (VectorMath.cs:39-70) / DotProduct (:8-37);
// V = 4: L2SquaredUnsafe (:188-253) / DotProductUnsafe (:128-186).  Any D (the tail runs in order).
// (kernels.hip em_* hold the one-lane form; the refine spreads it over 8 lanes, below.)

// hsum8 over the 8 lanes of an aligned lane group, lane l holding v[l]: the same three levels of
// pairwise adds (fp32 adds commute, so every lane of the group ends with the identical value)
__device__ __forceinline__ float hsum8_lanes(float v) {
  v = v + __shfl_xor(v, 1);  // (v0 + v1), (v2 + v3), ...
  v = v + __shfl_xor(v, 2);  // lo = (v0 + v1) + (v2 + v3), hi
  return v + __shfl_xor(v, 4);  // lo + hi
}

// exact_score with its 8 accumulator lanes spread over an 8-lane group: lane l (0..7) runs the
// chains of accumulator l (a1..a4[l] for V = 4, acc[l] for the 8-wide loop), in the same order, and
// the group reduces them as hsum8 does.  Every lane of the group returns the score.
// DT > 0: the dimension as a compile-time constant (every loop unrolls, so all of a row's loads are in
// flight at once; the additions keep their order)
template <int V, int MET, int DT = 0, bool RM = false>
__device__ float exact_score_l8(const float *q, const float *rows, int64_t r, int Dr, int l) {
  const int D = DT > 0 ? DT : Dr;
  constexpr int UNR32 = DT > 0 ? DT / 32 : 1, UNR8 = DT > 0 ? DT / 8 : 4;
  // RM: rows is row-major (a row's dims contiguous: the 8 lanes of a group read 32 B together instead
  // of 8 scattered sectors of the blocked store)
  auto X = [&](int d) { return RM ? rows[(size_t)r * D + d] : rows[blk_off(r, d, D)]; };
  float sum = 0.0f;
  int i = 0;
  if (V == 4 && D >= 32) {
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll UNR32
    for (; i <= D - 32; i += 32)
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const float x = X(i + 8 * v + l);
        float t;
        if (MET == L2) {
          const float d = q[i + 8 * v + l] - x;
          t = d * d;
        } else {
          t = q[i + 8 * v + l] * x;
        }
        a[v] = a[v] + t;
      }
    const float fin = ((a[0] + a[1]) + a[2]) + a[3];
    sum = sum + hsum8_lanes(fin);
  }
  if (i <= D - 8) {
    float acc = 0.0f;
#pragma unroll UNR8
    for (; i <= D - 8; i += 8) {
      const float x = X(i + l);
      if (MET == L2) {
        const float d = q[i + l] - x;
        acc = acc + d * d;
      } else {
        acc = acc + q[i + l] * x;
      }
    }
    sum = sum + hsum8_lanes(acc);
  }
  // the scalar tail (VectorMath.cs:243-250 / :182-185 and the safe forms' remainder loops), in order;
  // every lane of the group adds the same terms
  for (; i < D; ++i) {
    const float x = X(i);
    if (MET == L2) {
      const float d = q[i] - x;
      sum = sum + d * d;
    } else {
      sum = sum + q[i] * x;
    }
  }
  return MET == L2 ? -sum : sum;
}

// One wave per query: lane c < K1 re-scores candidate c exactly, ranks it among the
// candidates by (exact score desc, key asc); lanes with rank < k write the result.
// Certificate (file header), with s~_K1 the merged K1-th approximate score:
//   L2: approx = 2 q.x - |x|^2 - |q|^2,  IP: approx = q.x, and for every row
//   |approx - reference| <= E = c_err * u * (|q| + X)^2   (L2)
//                              c_err * u * |q| * X       (IP)
// with X >= every row norm of the index and u = 2^-24: the fp32 MFMA dot is an fmaf
// chain of D terms (error <= D u sum|q_i x_i| <= D u |q||x|), |x|^2 and |q|^2 are fp32
// sums (<= D u |.|^2 each), one more rounding combines them, and the reference's own
// sum is within (D/8 + 5) u (|q| + |x|)^2 of the real value: < (3.2 D + 6) u (|q|+|x|)^2
// in all, against c_err = 4 D + 64 (engine).  The bf16x3 filter adds c_bf u |q| X
// (kernels.h filter_bf16x3_cerr) and an absolute term for flushed subnormal halves.  If fewer than K1 candidates exist no row
// was excluded and the result is exact as it stands.
template <int V, int MET, int DT>
__global__ __launch_bounds__(256) void refine_kernel(RefineArgs a) {
  const int lane = threadIdx.x & 63;
  int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  if (a.qsel) {  // a device-sized subset (the failures of an earlier certificate): no host round trip
    if (q >= *a.nsel) return;
    q = a.qsel[q];
  }
  const int D = DT > 0 ? DT : a.dim, k1 = a.k1, k = a.k;
  constexpr int UNR8 = DT > 0 ? DT / 8 : 4;
  const int ld = a.ld > 0 ? a.ld : k1;
  const float *qp = a.queries + (size_t)q * D;
  float part = 0.0f;  // |q|^2, any order (covered by E); a shard record certifies nowhere here: not needed
  if (!a.rec)
    for (int d = lane; d < D; d += 64) part += qp[d] * qp[d];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
  const float qsq = part;
  float qa = 0.0f;  // max |q_i|: the fp16 filter's query scale (filter16.hip pow2_scale)
  if (a.q16 && !a.rec) {
    for (int d = lane; d < D; d += 64) qa = fmaxf(qa, fabsf(qp[d]));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) qa = fmaxf(qa, __shfl_xor(qa, off));
  }

  const float *ms = a.ms + (size_t)q * ld;
  const int32_t *mk = a.mk + (size_t)q * ld;
  uint32_t key = KEY_NONE;
  float s = -INFINITY;
  if (lane < k1 && mk[lane] >= 0) key = (uint32_t)mk[lane];
  // exact scores, 8 candidates per pass (an 8-lane group per candidate), then candidate c's score
  // moves to lane c
  const uint64_t real = __builtin_amdgcn_ballot_w64(key != KEY_NONE);
  for (int p = 0; 8 * p < k1; ++p) {
    // a pass whose 8 candidates are all empty or floor placeholders scores nothing (a list-sharded rank
    // often holds only a few of a query's candidates)
    if (((real >> (8 * p)) & 0xFFull) == 0ull) continue;
    const int c = 8 * p + (lane >> 3);
    const int32_t kc = __shfl((int)key, c);  // (k1 <= 64: every candidate's key sits on lane c)
    const int64_t rk = kc >= 0 ? (int64_t)kc : 0;
    float sc;
    if (MET == L2 && a.cosine) {  // VectorMath.Cosine (:102-109) with the cached norms
      const float dot = a.rows_rm ? exact_score_l8<V, IP, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                                  : exact_score_l8<V, IP, DT, false>(qp, a.rows, rk, D, lane & 7);
      const float qn = a.qnorm[q], xn = a.rnorm[rk];
      sc = (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
    } else {
      sc = a.rows_rm ? exact_score_l8<V, MET, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                     : exact_score_l8<V, MET, DT, false>(qp, a.rows, rk, D, lane & 7);
    }
    const float t = __shfl(sc, 8 * (lane & 7));
    if ((lane >> 3) == p && key != KEY_NONE) s = t;
  }
  int rank = 0, valid = 0;
  for (int c = 0; c < k1; ++c) {
    const float sc = __shfl(s, c);
    const uint32_t kc = __shfl(key, c);
    if (kc == KEY_NONE) continue;
    ++valid;
    if (key != KEY_NONE && better(sc, kc, s, key)) ++rank;
  }
  const int nout = min(valid, k);
  if (a.rec) {
    // list-sharded search (shard.hip): this rank's exact top-k and the bound of every row it left out (the
    // K1-th merged bound: candidates past it, the rows below T_q and a full buffer's floor all score at
    // most that), no certificate here -- the home rank's merge certifies against every rank's bound
    uint8_t *rp = static_cast<uint8_t *>(a.rec) + (size_t)q * shard_record_bytes(k);
    ShardEntry *ent = reinterpret_cast<ShardEntry *>(rp);
    if (key != KEY_NONE && rank < k) {
      ShardEntry e;
      e.label = a.row_labels ? a.row_labels[key] : (int64_t)key;
      e.score = s;
      e.list = a.rec_row_list ? a.rec_row_list[key] : shard_list_of(a.rec_lb, a.rec_nlist, key);
      ent[rank] = e;
    }
    if (lane >= nout && lane < k) {
      ShardEntry e;
      e.label = -1;
      e.score = -INFINITY;
      e.list = 0x7FFFFFFF;
      ent[lane] = e;
    }
    if (lane == 0) {
      ShardTrailer t;
      t.bound = mk[k1 - 1] != -1 ? ms[k1 - 1] : -INFINITY;
      t.n = nout;
      t.pad = 0;
      *reinterpret_cast<ShardTrailer *>(rp + 16 * (size_t)k) = t;
    }
    return;
  }
  if (key != KEY_NONE && rank < k) {
    a.out_s[(size_t)q * k + rank] = s;
    a.out_l[(size_t)q * k + rank] = a.row_labels ? a.row_labels[key] : (int64_t)key;
  }
  if (lane >= nout && lane < k) {
    a.out_s[(size_t)q * k + lane] = -INFINITY;
    a.out_l[(size_t)q * k + lane] = -1;
  }
  bool ok = true;
  // K1 candidates (rows, or a part's floor placeholder KEY_FLOOR = -2 that stands for rows the scan
  // dropped at or below its score): rows were excluded, check the margin against the K1-th score
  if (mk[k1 - 1] != -1) {
    float skth = -INFINITY;
    for (int c = 0; c < k1; ++c) {
      const int rc = __shfl(rank, c);
      const uint32_t kc = __shfl(key, c);
      const float sc = __shfl(s, c);
      if (kc != KEY_NONE && rc == k - 1) skth = sc;
    }
    const double u = 5.9604644775390625e-8;  // 2^-24
    const double qn = sqrt((double)qsq) * (1.0 + 1e-5);
    if (a.resid && a.ub) {
      // upper-bound candidates (stream16.hip, stream_ub_terms): every row left out -- below T_q, a
      // region's floor, or merged below the K1-th -- has a reference score at most the K1-th entry
      if (MET == L2 && a.cosine) {
        // the bounds are L2 scores s of the unit vectors: 1 + s / 2 bounds q^.x^, within (D/2 + 66) u of
        // the real cosine, the reference Cosine within (D/4 + 28) u of it (cos_rerank_kernel)
        const double pk = 1.0 + 0.5 * (double)ms[k1 - 1];
        const float qn = a.qnorm[q];
        ok = nout == k && (double)skth > pk + (2.0 * D + 256.0) * u && qn >= 1e-6f && isfinite(qn) &&
             !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
      } else {
        ok = nout == k && skth > ms[k1 - 1];
      }
      if (lane == 0) {
        if (a.out_c) a.out_c[q] = nout;
        if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
      }
      return;
    }
    if (a.resid) {
      // IVF fp16 filter over residual tiles (filter16.hip, stream16.hip): approx estimates the score
      // itself,  L2: -|q - x|^2 = 2 (q-c).(x-c) - |x-c|^2 - |q-c|^2,  IP: q.x = q.(x-c) + q.c,
      // so for a row of list l its error is relative to the residuals: fp16 rows and queries
      // c_bf u A_l X_l (A_l = |q - c_l| for L2, |q| for IP; X_l = max |x - c_l| over the list), fp32
      // sums / adds (D + 8) u (A_l + X_l)^2, subnormal halves (c_abs A_l, and the query's, below
      // 2^-36 sqrt(D) A_l X_l), IP's q.c constant (D + 8) u |q||c_l|.  The reference's own sum: L2
      // adds non-negative terms, so R = T (1 +- g), g = (D/8 + 8) u; IP |R - T| <= g |q| max|x|.
      // Per list: a probed list none of whose rows can reach skth whatever the filter
      // saw -- L2: |q - c_l| - X_l >= r with r^2 = -skth (1 + 2 c_err u); IP: q.c_l + |q| X_l plus its
      // roundings below skth -- adds no error term; E is the largest term of the other lists.
      const double g = (D / 8.0 + 8.0) * u;
      const double r = sqrt(fmax(0.0, -(double)skth) * (1.0 + 2.0 * a.c_err * u) + 1e-30) * (1.0 + 1e-6);
      double emax = 0.0;
      // FLAT (no probes): one center, list 0
      // 8 probes per pass, an 8-lane group per probe, lane j of it summing dims j, j + 8, ...
      const int np = a.probes ? a.nprobe : 1;
      // probe ids of 64 probes at a time, one per lane, handed to the 8-lane groups by shuffle (no
      // dependent id load inside the passes)
      int pid = 0;
      for (int p0 = 0; p0 < np; p0 += 8) {
        if ((p0 & 63) == 0)
          pid = a.probes && p0 + lane < np ? a.probes[(size_t)q * a.nprobe + p0 + lane] : 0;
        const int p = p0 + (lane >> 3), j = lane & 7;
        const int lp = __shfl(pid, (p0 & 63) + (lane >> 3));
        float d2 = 0.0f, c2 = 0.0f, qc = 0.0f;
        if (p < np) {
          const float *c = a.cents + (size_t)lp * D;
          // the error terms follow the query the filter scored: the unit query for Cosine (qcert)
          const float *qe = a.qcert ? a.qcert + (size_t)q * D : qp;
#pragma unroll UNR8
          for (int d = j; d < D; d += 8) {
            const float t = qe[d] - c[d];
            d2 += t * t;
            c2 += c[d] * c[d];
            qc += qe[d] * c[d];
          }
        }
#pragma unroll
        for (int off = 1; off <= 4; off <<= 1) {
          d2 += __shfl_xor(d2, off);
          c2 += __shfl_xor(c2, off);
          qc += __shfl_xor(qc, off);
        }
        if (p < np) {
          const double Xr = sqrt((double)key_score(a.list_rmax_r[lp])) * (1.0 + 1e-5);
          const double cn = sqrt((double)c2) * (1.0 + 1e-5);
          double el = 0.0;
          if (MET == L2) {
            const double Al = sqrt((double)d2) * (1.0 + 1e-5) + 1e-30;
            const double Alo = sqrt((double)d2) * (1.0 - 1e-5);
            // (fp32 |q - c|^2: relative error <= (D + 8) u, far inside the 1e-5 margins)
            if (!a.tri || Alo - Xr < r) {
              const double X = a.tri ? fmin(Xr, Al + r) : Xr;
              el = a.c_bf * u * Al * X + a.c_err * u * (Al + X) * (Al + X) + a.c_abs * Al +
                   2.0 * 1.4551915228366852e-11 * sqrt((double)D) * Al * X;
            }
          } else {
            const double Xf = sqrt((double)key_score(a.list_rmax ? a.list_rmax[lp] : *a.max_rsq)) * (1.0 + 1e-5);
            // every row x of l: q.x <= q.c + |q| X_l; fp32 q.c is within (D + 8) u |q||c| of the real
            // value, the reference's sum within g |q||x|
            const double hi = (double)qc + qn * Xr + (g + a.c_err * u) * qn * (cn + Xr + Xf);
            if (!a.tri || hi >= (double)skth)
              el = a.c_bf * u * qn * Xr + a.c_err * u * qn * Xr + a.c_abs * qn +
                   1.4551915228366852e-11 * sqrt((double)D) * qn * Xr + a.c_err * u * qn * cn + g * qn * Xf;
          }
          emax = fmax(emax, el);
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) emax = fmax(emax, __shfl_xor(emax, off));
      const double ak = (double)ms[k1 - 1];
      if (MET == L2 && a.cosine) {
        // unit-row L2 approximations (FlatIndex::search_cosine): a row left out has -|q^ - x^|^2 <= ak + emax
        // (real arithmetic), so q^.x^ <= 1 + (ak + emax) / 2, within (D/4 + 28) u of its cosine; the
        // reference Cosine within (D/4 + 28) u of that (cos_rerank_kernel)
        const float qn = a.qnorm[q];
        ok = nout == k && (double)skth > 1.0 + 0.5 * (ak + emax) + (2.0 * D + 256.0) * u && qn >= 1e-6f &&
             isfinite(qn) && !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
      } else if (MET == L2) {
        ok = nout == k && (double)skth > (ak + emax) + g * fabs(ak + emax);
      } else {
        ok = nout == k && (double)skth > ak + emax;
      }
      if (lane == 0) {
        if (a.out_c) a.out_c[q] = nout;
        if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
      }
      return;
    }
    // X bounds the norm of every row this query's scan could have excluded: the largest |x|^2
    // of its probed lists (IVF), else of the whole store
    uint32_t xk = 0;
    if (a.list_rmax) {
      for (int p = lane; p < a.nprobe; p += 64) xk = max(xk, a.list_rmax[a.probes[(size_t)q * a.nprobe + p]]);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) xk = max(xk, (uint32_t)__shfl_xor((int)xk, off));
    } else {
      xk = *a.max_rsq;
    }
    double X = sqrt((double)key_score(xk)) * (1.0 + 1e-5);
    if (MET == L2 && a.tri) {
      // Rows far from the query cannot reach skth whatever the filter saw: the reference's L2 sum
      // adds non-negative terms, so its value is |q - x|^2 (1 +- 22u) (D <= 128; c_err u is far
      // above that), and |q - x| >= |x| - |q|.  A row with |x| >= |q| + r, r^2 = -skth (1 + 2 c_err u),
      // therefore scores below skth; only rows with |x| < |q| + r need the error bound, so X may
      // be lowered to |q| + r (one large-norm outlier in a probed list then costs nothing).
      const double r = sqrt(fmax(0.0, -(double)skth) * (1.0 + 2.0 * a.c_err * u) + 1e-30) * (1.0 + 1e-6);
      X = fmin(X, qn + r);
    }
    double e = (MET == L2 ? a.c_err * u * (qn + X) * (qn + X) : a.c_err * u * qn * X) +
                     a.c_bf * u * qn * X + (a.c_bf > 0.0 ? 1e-30 * (1.0 + qn + X) * D : 0.0);  // bf16 subnormals
    if (a.q16) {
      // fp16 filter: the rows' subnormal halves (c_abs |q|) and the query's, 2^-25 sqrt(D) X / sq
      double sqs = 1.0;
      if (qa > 0.0f && isfinite(qa)) {
        int ex;
        frexp((double)qa, &ex);
        sqs = ldexp(1.0, 14 - ex);
      }
      e += a.c_abs * qn + (MET == L2 ? 2.0 : 1.0) * 2.9802322387695312e-08 * sqrt((double)D) * X / sqs;
    }
    const double approx_k1 = MET == L2 ? (double)ms[k1 - 1] - (double)qsq : (double)ms[k1 - 1];
    ok = nout == k && (double)skth > approx_k1 + e;
    if (!a.q16 && a.max_rsq && a.max_rsq[1] != 0u) ok = false;  // a non-finite row the filter cannot score
  }
  if (lane == 0) {
    if (a.out_c) a.out_c[q] = nout;
    if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
  }
}

// The stream scans' merge and certified refine in ONE wave per query (replaces cand_merge_kernel + the
// depth-K1 refine + the depth-64 refine of the failures: no merged-candidate round trip through HBM, no
// second launch).  The merge leaves lane j with the query's j-th best candidate bound (a row, or a floor
// placeholder max(T_q, floor)); the candidates of depth K1 are re-scored exactly and certified as in
// refine_kernel's upper-bound branch; a query that fails goes on to depth 64 in the same wave (its other 48
// candidates scored then), and what fails there is listed for the exact re-run.  Shard records (a.rec): the
// depth-K1 answer and bound, no certificate.
template <int V, int MET, int DT>
__global__ __launch_bounds__(256) void merge_refine_kernel(CandMergeArgs m, RefineArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  // fewer emitted rows than K1 and none dropped (a list-sharded rank holds a few of most queries' rows):
  // they all sit within depth K1 whatever their order, the rest of the list is the floor -- no sort
  uint64_t cur;
  const int tot0 = m.cand_n[q];
  if (tot0 < a.k1 && m.cand_f[q] == 0u) {
    const float F = m.thr ? m.thr[q] : -INFINITY;
    cur = F > -INFINITY ? pack_cand(F, KEY_FLOOR) : 0ull;
    if (lane < tot0) {
      const uint2 e = m.cand[(size_t)q * m.cap + lane];
      cur = pack_cand(__uint_as_float(e.x), e.y);
    }
  } else {
    cur = cand_merge_wave<STREAM_KO>(m, q, lane);
  }
  const uint32_t kk = ~(uint32_t)cur;
  const float msl = cur != 0ull ? key_score((uint32_t)(cur >> 32)) : -INFINITY;   // lane j: ms[j]
  const int32_t mkl = cur == 0ull ? -1 : (kk == KEY_FLOOR ? -2 : (int32_t)kk);    // lane j: mk[j]
  const int D = DT > 0 ? DT : a.dim, k = a.k, k1 = a.k1;
  const float *qp = a.queries + (size_t)q * D;
  const uint32_t key = mkl >= 0 ? (uint32_t)mkl : KEY_NONE;
  const uint64_t real = __builtin_amdgcn_ballot_w64(key != KEY_NONE);
  float s = -INFINITY;  // lane j: the exact score of candidate j (a row)
  auto score_one = [&](int32_t kc) -> float {
    const int64_t rk = kc >= 0 ? (int64_t)kc : 0;
    if (MET == L2 && a.cosine) {  // VectorMath.Cosine (:102-109) with the cached norms
      const float dot = a.rows_rm ? exact_score_l8<V, IP, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                                  : exact_score_l8<V, IP, DT, false>(qp, a.rows, rk, D, lane & 7);
      const float qn = a.qnorm[q], xn = a.rnorm[rk];
      return (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
    }
    return a.rows_rm ? exact_score_l8<V, MET, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                     : exact_score_l8<V, MET, DT, false>(qp, a.rows, rk, D, lane & 7);
  };
  auto score_passes = [&](int p0, int p1) {
    if (p1 - p0 == 2 && ((real >> (8 * p0)) & 0xFFFFull) != 0ull) {
      // the depth-16 passes together: both rows' loads in flight before either sum (one round trip, not two)
      const int c = 8 * p0 + (lane >> 3);
      const int32_t k0 = __shfl((int)key, c), k1 = __shfl((int)key, c + 8);
      const float s0 = score_one(k0), s1 = score_one(k1);
      const float t0 = __shfl(s0, 8 * (lane & 7)), t1 = __shfl(s1, 8 * (lane & 7));
      if ((lane >> 3) == p0 && key != KEY_NONE) s = t0;
      if ((lane >> 3) == p0 + 1 && key != KEY_NONE) s = t1;
      return;
    }
    for (int p = p0; p < p1; ++p) {
      if (((real >> (8 * p)) & 0xFFull) == 0ull) continue;  // 8 placeholders / empties: nothing to score
      const int c = 8 * p + (lane >> 3);
      const int32_t kc = __shfl((int)key, c);
      const int64_t rk = kc >= 0 ? (int64_t)kc : 0;
      float sc;
      if (MET == L2 && a.cosine) {  // VectorMath.Cosine (:102-109) with the cached norms
        const float dot = a.rows_rm ? exact_score_l8<V, IP, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                                    : exact_score_l8<V, IP, DT, false>(qp, a.rows, rk, D, lane & 7);
        const float qn = a.qnorm[q], xn = a.rnorm[rk];
        sc = (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
      } else {
        sc = a.rows_rm ? exact_score_l8<V, MET, DT, true>(qp, a.rows_rm, rk, D, lane & 7)
                       : exact_score_l8<V, MET, DT, false>(qp, a.rows, rk, D, lane & 7);
      }
      const float t = __shfl(sc, 8 * (lane & 7));
      if ((lane >> 3) == p && key != KEY_NONE) s = t;
    }
  };
  int d = k1, rank = 0, nout = 0;
  float skth = -INFINITY, bound = -INFINITY;
  bool excluded = false;
  // the ranking of depth d's candidates by (exact score desc, key asc), its k-th score and the bound of
  // everything past depth d
  // (only the real candidates' lanes are visited: a list-sharded rank often holds few or none of a query's)
  auto rank_at = [&](int dd) {
    const uint32_t kd = lane < dd ? key : KEY_NONE;
    const uint64_t rd = real & (dd >= 64 ? ~0ull : ((1ull << dd) - 1ull));
    rank = 0;
    for (uint64_t rm = rd; rm; rm &= rm - 1ull) {
      const int c = (int)__builtin_ctzll(rm);
      const float sc = __shfl(s, c);
      const uint32_t kc = __shfl(kd, c);
      if (kd != KEY_NONE && better(sc, kc, s, kd)) ++rank;
    }
    nout = min((int)__builtin_popcountll(rd), k);
    skth = -INFINITY;
    for (uint64_t rm = rd; rm; rm &= rm - 1ull) {
      const int c = (int)__builtin_ctzll(rm);
      const int rc = __shfl(rank, c);
      const float sc = __shfl(s, c);
      if (rc == k - 1) skth = sc;
    }
    excluded = __shfl(mkl, dd - 1) != -1;
    bound = __shfl(msl, dd - 1);
    if (lane >= dd) rank = 64;  // not a candidate at this depth
  };
  score_passes(0, k1 / 8);
  rank_at(k1);
  if (a.rec) {  // list-sharded record (see refine_kernel)
    uint8_t *rp = static_cast<uint8_t *>(a.rec) + (size_t)q * shard_record_bytes(k);
    ShardEntry *ent = reinterpret_cast<ShardEntry *>(rp);
    if (key != KEY_NONE && rank < k) {
      ShardEntry e;
      e.label = a.row_labels ? a.row_labels[key] : (int64_t)key;
      e.score = s;
      e.list = shard_list_of(a.rec_lb, a.rec_nlist, key);
      ent[rank] = e;
    }
    if (lane >= nout && lane < k) {
      ShardEntry e;
      e.label = -1;
      e.score = -INFINITY;
      e.list = 0x7FFFFFFF;
      ent[lane] = e;
    }
    if (lane == 0) {
      ShardTrailer t;
      t.bound = excluded ? bound : -INFINITY;
      t.n = nout;
      t.pad = 0;
      *reinterpret_cast<ShardTrailer *>(rp + 16 * (size_t)k) = t;
    }
    return;
  }
  const double u = 5.9604644775390625e-8;  // 2^-24
  auto certified = [&]() -> bool {
    if (!excluded) return true;  // no row was left out
    if (MET == L2 && a.cosine) {
      const float qn = a.qnorm[q];
      return nout == k && (double)skth > 1.0 + 0.5 * (double)bound + (2.0 * D + 256.0) * u && qn >= 1e-6f &&
             isfinite(qn) && !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
    }
    return nout == k && skth > bound;
  };
  bool ok = certified();
  if (!ok && d < STREAM_KO && k + 4 <= STREAM_KO) {  // (wave-uniform) the same candidates at depth 64
    score_passes(k1 / 8, STREAM_KO / 8);
    d = STREAM_KO;
    rank_at(d);
    ok = certified();
  }
  if (key != KEY_NONE && rank < k) {
    a.out_s[(size_t)q * k + rank] = s;
    a.out_l[(size_t)q * k + rank] = a.row_labels ? a.row_labels[key] : (int64_t)key;
  }
  if (lane >= nout && lane < k) {
    a.out_s[(size_t)q * k + lane] = -INFINITY;
    a.out_l[(size_t)q * k + lane] = -1;
  }
  if (lane == 0) {
    if (a.out_c) a.out_c[q] = nout;
    if (!ok) a.fail_list[atomicAdd(a.fail_cnt, 1)] = (int32_t)q;
  }
}

// k > 60: the stream scans' merge and certified refine at depth K1 = 128 / 256 / 512 (deeprank.h: the select of
// the K1 best emitted rows, their exact scores in the reference's order, as merge_refine_kernel's, and their
// ranks); the top k written, and the certificate of refine_kernel's upper-bound branch.
template <int V, int MET, int DT>
__global__ __launch_bounds__(256) void deep_refine_kernel(CandMergeArgs m, RefineArgs a) {
  extern __shared__ uint64_t dk[];  // the emitted rows' rank keys (pack_cand), in buffer order
  const int64_t q = blockIdx.x;
  const int k = a.k, D = DT > 0 ? DT : a.dim;
  const float *qp = a.queries + (size_t)q * D;
  const DeepRank R = deep_select_rank(m, q, a.k1, dk, [&](uint32_t kc, int l) {
    if (MET == L2 && a.cosine) {  // VectorMath.Cosine (:102-109) with the cached norms
      const float dot = a.rows_rm ? exact_score_l8<V, IP, DT, true>(qp, a.rows_rm, kc, D, l)
                                  : exact_score_l8<V, IP, DT, false>(qp, a.rows, kc, D, l);
      const float qn = a.qnorm[q], xn = a.rnorm[kc];
      return (qn < 1e-6f || xn < 1e-6f) ? 0.0f : dot / (qn * xn);
    }
    return a.rows_rm ? exact_score_l8<V, MET, DT, true>(qp, a.rows_rm, kc, D, l)
                     : exact_score_l8<V, MET, DT, false>(qp, a.rows, kc, D, l);
  });
  const int nout = min(R.j, k);
  const float skth = deep_kth(R, k);
  bool ok;
  if (!R.excluded) {
    ok = true;
  } else if (MET == L2 && a.cosine) {
    const double u = 5.9604644775390625e-8;  // 2^-24
    const float qn = a.qnorm[q];
    ok = nout == k && (double)skth > 1.0 + 0.5 * (double)R.bound + (2.0 * D + 256.0) * u && qn >= 1e-6f &&
         isfinite(qn) && !(a.max_rsq && a.max_rsq[1] != 0u) && !(a.zflag && *a.zflag != 0u && !(skth > 0.0f));
  } else {
    ok = nout == k && skth > R.bound;
  }
  ok = ok && !R.nan;
  deep_write(R, q, k, ok, a.row_labels, a.out_s, a.out_l, a.out_c, a.fail_list, a.fail_cnt);
}

__global__ void unit_rows_kernel(const float *x, const int64_t *slots, const float *norms, int64_t n, int D,
                                 float *out, uint32_t *zflag, const uint8_t *live) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / D;
    const int d = (int)(e % D);
    const int64_t r = slots ? slots[i] : i;
    const float nr = norms[r];
    const float v = slots ? x[blk_off(r, d, D)] : x[e];
    const bool unit = nr >= 1e-6f && isfinite(nr);
    out[e] = unit ? v * (1.0f / nr) : 0.0f;
    if (zflag && d == 0 && !unit && (!live || live[r])) *zflag = 1u;
  }
}

// result rows of the exact re-run (sub-batch order) back to their queries
__global__ void scatter_results_kernel(const int32_t *qidx, int64_t n, int k, const float *ss, const int64_t *sl,
                                       const int32_t *sc, float *out_s, int64_t *out_l, int32_t *out_c) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * k) return;
  const int64_t i = e / k;
  const int j = (int)(e % k);
  const int64_t q = qidx[i];
  out_s[q * k + j] = ss[e];
  out_l[q * k + j] = sl[e];
  if (j == 0 && out_c) out_c[q] = sc[i];
}

// rows qidx[i] of a [*][D] array of 32-bit words (queries, probe lists), copied bit for bit
__global__ void gather_words_kernel(const uint32_t *q, const int32_t *qidx, int64_t n, int D, uint32_t *out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid-stride: grids stay below 2^32 work-items
    const int64_t i = e / D;
    out[e] = q[(size_t)qidx[i] * D + e % D];
  }
}

// |x|^2 of blocked rows (slots[i], or i when slots is null) and the running maximum
// (score_key-encoded, only grows) that the refine certificate bounds row norms with
__global__ void sqnorms_kernel(const float *rows, const int64_t *slots, int64_t n, int D, float *out,
                               uint32_t *max_key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = slots ? slots[i] : i;
  float s = 0.0f;
  for (int d = 0; d < D; ++d) {
    const float x = rows[blk_off(r, d, D)];
    s = s + x * x;
  }
  out[r] = s;
  // a NaN / inf row is left out of the norm bound (one bad row would fail every later certificate);
  // the fp16 tile filters carry it in meta (+inf: always a candidate), the bf16x3 / fp32 filters
  // cannot score it (hi = inf, lo = inf - inf = NaN), so max_key[1] marks the store and their
  // certificate fails
  if (isfinite(s)) atomicMax(max_key, score_key(s));
  else max_key[1] = 1u;
}

// per-list max of |x|^2 (score_key, finite rows only) over rows [lb[l], le[l]): the refine
// certificate of an IVF query bounds row norms over its probed lists only
__global__ __launch_bounds__(256) void list_rmax_kernel(const float *rsq, const int32_t *lb, const int32_t *le,
                                                        int nlist, uint32_t *out) {
  const int l = blockIdx.x;
  if (l >= nlist) return;
  uint32_t m = 0;
  for (int r = lb[l] + (int)threadIdx.x; r < le[l]; r += 256) {
    const float v = rsq[r];
    if (isfinite(v)) m = max(m, score_key(v));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
  __shared__ uint32_t wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[l] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

void launch_unit_rows(const float *x, const int64_t *slots, const float *norms, int64_t n, int32_t dim, float *out,
                      hipStream_t st, uint32_t *zflag, const uint8_t *live) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n * dim + 255) / 256, int64_t(1) << 22);
  hipLaunchKernelGGL(unit_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, slots, norms, n, dim, out,
                     zflag, live);
}

void launch_refine(const RefineArgs &a, int metric, int V, hipStream_t st) {
  if (a.nq <= 0) return;
  const dim3 g(nblk(a.nq, 4)), b(256);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, g, b, 0, st, a); };
  // the common dimensions as compile-time constants (fully unrolled row loads), others at run time
  auto by_dim = [&](auto k0, auto k32, auto k64, auto k128) {
    switch (a.dim) {
      case 32: go(k32); return;
      case 64: go(k64); return;
      case 128: go(k128); return;
      default: go(k0); return;
    }
  };
  if (V == 4) {
    if (metric == L2) by_dim(refine_kernel<4, L2, 0>, refine_kernel<4, L2, 32>, refine_kernel<4, L2, 64>, refine_kernel<4, L2, 128>);
    else by_dim(refine_kernel<4, IP, 0>, refine_kernel<4, IP, 32>, refine_kernel<4, IP, 64>, refine_kernel<4, IP, 128>);
  } else {
    if (metric == L2) by_dim(refine_kernel<1, L2, 0>, refine_kernel<1, L2, 32>, refine_kernel<1, L2, 64>, refine_kernel<1, L2, 128>);
    else by_dim(refine_kernel<1, IP, 0>, refine_kernel<1, IP, 32>, refine_kernel<1, IP, 64>, refine_kernel<1, IP, 128>);
  }
}

void launch_merge_refine(const CandMergeArgs &m, const RefineArgs &a, int metric, int V, hipStream_t st) {
  if (a.nq <= 0) return;
  if (a.k1 % 8 != 0 || a.k1 > STREAM_KO || a.k1 < a.k) throw std::invalid_argument("merge_refine: depth");
  const dim3 g(nblk(a.nq, 4)), b(256);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, g, b, 0, st, m, a); };
  auto by_dim = [&](auto k0, auto k32, auto k64, auto k128) {
    switch (a.dim) {
      case 32: go(k32); return;
      case 64: go(k64); return;
      case 128: go(k128); return;
      default: go(k0); return;
    }
  };
  if (V == 4) {
    if (metric == L2)
      by_dim(merge_refine_kernel<4, L2, 0>, merge_refine_kernel<4, L2, 32>, merge_refine_kernel<4, L2, 64>,
             merge_refine_kernel<4, L2, 128>);
    else
      by_dim(merge_refine_kernel<4, IP, 0>, merge_refine_kernel<4, IP, 32>, merge_refine_kernel<4, IP, 64>,
             merge_refine_kernel<4, IP, 128>);
  } else {
    if (metric == L2)
      by_dim(merge_refine_kernel<1, L2, 0>, merge_refine_kernel<1, L2, 32>, merge_refine_kernel<1, L2, 64>,
             merge_refine_kernel<1, L2, 128>);
    else
      by_dim(merge_refine_kernel<1, IP, 0>, merge_refine_kernel<1, IP, 32>, merge_refine_kernel<1, IP, 64>,
             merge_refine_kernel<1, IP, 128>);
  }
}

size_t deep_refine_lds_bytes(int cap, int k1) {  // the staged rank keys of a full candidate buffer
  return (size_t)std::max(cap, 256) * sizeof(uint64_t);
}

// the dynamic-LDS limit of each instantiation is raised once per device to the largest launch deep_k1 allows
// (144 KiB: the static LDS, ~4 KiB, sits beside it; asking for the whole 160 KiB fails), never lowered -- so
// concurrent searches of different k on other streams cannot shrink it under one another
constexpr int DEEP_LDS_MAX = 144 * 1024;
template <int V, int MET, int D>
static void go_deep(const CandMergeArgs &m, const RefineArgs &a, size_t lds, hipStream_t st) {
  static std::atomic<uint64_t> done{0};
  allow_max_lds(reinterpret_cast<const void *>(&deep_refine_kernel<V, MET, D>), done, DEEP_LDS_MAX);
  hipLaunchKernelGGL((deep_refine_kernel<V, MET, D>), dim3((unsigned)a.nq), dim3(256), lds, st, m, a);
}

void launch_deep_refine(const CandMergeArgs &m, const RefineArgs &a, int metric, int V, hipStream_t st) {
  if (a.nq <= 0) return;
  if (a.k1 > DEEP_MAX || a.k1 < a.k || a.k > 256) throw std::invalid_argument("deep_refine: depth");
  const size_t lds = deep_refine_lds_bytes(m.cap, a.k1);
  if (lds > (size_t)DEEP_LDS_MAX) throw std::invalid_argument("deep_refine: candidate buffer too large");
  // V = 1: the safe VectorMath forms (IVF); V = 4: the *Unsafe forms (FLAT, BruteForceVectorIndex.cs:350-356)
  if (V == 4) {
    if (metric == L2) {
      if (a.dim == 128) go_deep<4, L2, 128>(m, a, lds, st);
      else go_deep<4, L2, 0>(m, a, lds, st);
    } else {
      if (a.dim == 128) go_deep<4, IP, 128>(m, a, lds, st);
      else go_deep<4, IP, 0>(m, a, lds, st);
    }
  } else if (metric == L2) {
    if (a.dim == 128) go_deep<1, L2, 128>(m, a, lds, st);
    else go_deep<1, L2, 0>(m, a, lds, st);
  } else {
    if (a.dim == 128) go_deep<1, IP, 128>(m, a, lds, st);
    else go_deep<1, IP, 0>(m, a, lds, st);
  }
}

void launch_gather_queries(const float *q, const int32_t *qidx, int64_t n, int32_t dim, float *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_words_kernel, dim3(gblk(n * dim)), dim3(256), 0, st, reinterpret_cast<const uint32_t *>(q),
                     qidx, n, dim, reinterpret_cast<uint32_t *>(out));
}
void launch_gather_words(const uint32_t *src, const int32_t *idx, int64_t n, int32_t width, uint32_t *out,
                         hipStream_t st) {
  if (n <= 0 || width <= 0) return;
  hipLaunchKernelGGL(gather_words_kernel, dim3(gblk(n * width)), dim3(256), 0, st, src, idx, n, width, out);
}

void launch_scatter_results(const int32_t *qidx, int64_t n, int32_t k, const float *ss, const int64_t *sl,
                            const int32_t *sc, float *out_s, int64_t *out_l, int32_t *out_c, hipStream_t st) {
  if (n <= 0 || k <= 0) return;
  hipLaunchKernelGGL(scatter_results_kernel, dim3(nblk(n * k, 256)), dim3(256), 0, st, qidx, n, k, ss, sl, sc, out_s,
                     out_l, out_c);
}

void launch_list_rmax(const float *rsq, const int32_t *lb, const int32_t *le, int32_t nlist, uint32_t *out,
                      hipStream_t st) {
  if (nlist <= 0) return;
  hipLaunchKernelGGL(list_rmax_kernel, dim3(nlist), dim3(256), 0, st, rsq, lb, le, nlist, out);
}

void launch_sqnorms(const float *rows, const int64_t *slots, int64_t n, int32_t dim, float *out, uint32_t *max_key,
                    hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sqnorms_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, rows, slots, n, dim, out, max_key);
}

}  // namespace pyr
