// vmath.h -- exact restatements of VectorMath.cs (src/Pyrope.GarnetServer/Vector/VectorMath.cs) on
// accessors, in the reference's fp32 operation order (x64 AVX2: 8 lanes, no contraction, the horizontal
// sum ((v0+v1)+(v2+v3))+((v4+v5)+(v6+v7))).  Internal to libpyrope_hip.so; include inside an anonymous
// namespace of a .hip file's pyr namespace compiled with -ffp-contract=off (kernels.hip, pq32.hip).
#pragma once

// ---------------------------------------------------------------------------
// Exact restatements of VectorMath.cs on accessors (generic dims).
// ---------------------------------------------------------------------------
struct Lin {
  const float *p;
  __device__ float operator()(int i) const { return p[i]; }
};
struct Blk {
  const float *base;
  int D;
  int64_t r;
  __device__ float operator()(int i) const { return base[blk_off(r, i, D)]; }
};
struct Off {  // sub-range accessor
  const float *p;
  __device__ float operator()(int i) const { return p[i]; }
};

__device__ __forceinline__ float hsum8(const float *v) {
  float lo = (v[0] + v[1]) + (v[2] + v[3]);
  float hi = (v[4] + v[5]) + (v[6] + v[7]);
  return lo + hi;
}

// VectorMath.cs:8-37 DotProduct
template <class A, class B>
__device__ float em_dot(A a, B b, int n) {
  int i = 0;
  float sum = 0.0f;
  if (n >= 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; i <= n - 8; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) acc[l] = acc[l] + a(i + l) * b(i + l);
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + a(i) * b(i);
  return sum;
}
// VectorMath.cs:39-70 L2Squared
template <class A, class B>
__device__ float em_l2sq(A a, B b, int n) {
  int i = 0;
  float sum = 0.0f;
  if (n >= 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; i <= n - 8; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        float d = a(i + l) - b(i + l);
        acc[l] = acc[l] + d * d;
      }
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) {
    float d = a(i) - b(i);
    sum = sum + d * d;
  }
  return sum;
}
// VectorMath.cs:72-100 ComputeNorm
template <class A>
__device__ float em_norm(A a, int n) {
  int i = 0;
  float sum = 0.0f;
  if (n >= 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; i <= n - 8; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) acc[l] = acc[l] + a(i + l) * a(i + l);
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + a(i) * a(i);
  return sqrtf(sum);
}
// VectorMath.cs:128-186 DotProductUnsafe
template <class A, class B>
__device__ float em_dot_unsafe(A a, B b, int n) {
  int i = 0;
  float sum = 0.0f;
  if (n >= 32) {
    float a1[8] = {0}, a2[8] = {0}, a3[8] = {0}, a4[8] = {0}, fin[8];
    for (; i <= n - 32; i += 32)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        a1[l] = a1[l] + a(i + l) * b(i + l);
        a2[l] = a2[l] + a(i + 8 + l) * b(i + 8 + l);
        a3[l] = a3[l] + a(i + 16 + l) * b(i + 16 + l);
        a4[l] = a4[l] + a(i + 24 + l) * b(i + 24 + l);
      }
#pragma unroll
    for (int l = 0; l < 8; l++) fin[l] = ((a1[l] + a2[l]) + a3[l]) + a4[l];
    sum = sum + hsum8(fin);
  }
  if (i <= n - 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; i <= n - 8; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) acc[l] = acc[l] + a(i + l) * b(i + l);
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) sum = sum + a(i) * b(i);
  return sum;
}
// VectorMath.cs:188-253 L2SquaredUnsafe
template <class A, class B>
__device__ float em_l2sq_unsafe(A a, B b, int n) {
  int i = 0;
  float sum = 0.0f;
  if (n >= 32) {
    float a1[8] = {0}, a2[8] = {0}, a3[8] = {0}, a4[8] = {0}, fin[8];
    for (; i <= n - 32; i += 32)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        float d1 = a(i + l) - b(i + l);
        float d2 = a(i + 8 + l) - b(i + 8 + l);
        float d3 = a(i + 16 + l) - b(i + 16 + l);
        float d4 = a(i + 24 + l) - b(i + 24 + l);
        a1[l] = a1[l] + d1 * d1;
        a2[l] = a2[l] + d2 * d2;
        a3[l] = a3[l] + d3 * d3;
        a4[l] = a4[l] + d4 * d4;
      }
#pragma unroll
    for (int l = 0; l < 8; l++) fin[l] = ((a1[l] + a2[l]) + a3[l]) + a4[l];
    sum = sum + hsum8(fin);
  }
  if (i <= n - 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; i <= n - 8; i += 8)
#pragma unroll
      for (int l = 0; l < 8; l++) {
        float d = a(i + l) - b(i + l);
        acc[l] = acc[l] + d * d;
      }
    sum = sum + hsum8(acc);
  }
  for (; i < n; i++) {
    float d = a(i) - b(i);
    sum = sum + d * d;
  }
  return sum;
}

// score of one (query, row) pair with the reference's formula for the path:
// V=4 -> BruteForceVectorIndex.cs:350-356 (Unsafe), V=1 -> IvfFlatVectorIndex.cs:351-360 (safe)
template <int V, int MET, class A, class B>
__device__ float em_score(A q, B x, int n, float qn, float xn) {
  if (MET == L2) return V == 4 ? -em_l2sq_unsafe(q, x, n) : -em_l2sq(q, x, n);
  if (MET == IP) return V == 4 ? em_dot_unsafe(q, x, n) : em_dot(q, x, n);
  if (qn < 1e-6f || xn < 1e-6f) return 0.0f;
  float d = V == 4 ? em_dot_unsafe(q, x, n) : em_dot(q, x, n);
  return d / (qn * xn);
}

