// f16util.h -- device helpers shared by the fp16 tile kernels (tiles16.hip, sample16.hip, scan.hip, pq32.hip).
// Internal to libpyrope_hip.so; include inside an anonymous namespace of a .hip file's pyr namespace.
// (include after <hip/hip_runtime.h> and <cmath>)
#pragma once

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

// the candidate order of every list: score desc, storage key asc
__device__ __forceinline__ bool better(float s1, uint32_t k1, float s2, uint32_t k2) {
  return s1 > s2 || (s1 == s2 && k1 < k2);
}

// LDS-DMA of SIZE (16 or 4) bytes per lane: global g (per lane) -> LDS lds + lane * SIZE (lds
// wave-uniform, in M0).  Written in inline asm on purpose: the compiler does not track these
// writes, so it does not drain every in-flight tile (vmcnt(0)) before each LDS access it cannot
// prove disjoint; the kernels' own counted vmcnt waits + barriers order the ring instead.
// SIZE 16: row pieces; 4: meta; 5: a 4-byte agent-coherent read (sc1, the shared bounds, as
// __hip_atomic_load with agent scope compiles to).
template <int SIZE>
__device__ __forceinline__ void glds(const void *g, uint32_t lds_addr) {
  int keep;
  const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform: an SGPR for M0
  if (SIZE == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
  else if (SIZE == 4)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, N] (immediate operand; larger n waits for N)
template <int N>
__device__ __forceinline__ void wait_vm_le(int n) {
  if constexpr (N > 0) {
    if (n >= N) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
      return;
    }
    wait_vm_le<N - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// query scale: a power of two putting max |q_i| below 2^14 (1 for a zero query)
__device__ __forceinline__ float pow2_scale(float amax) {
  if (!(amax > 0.0f) || !isfinite(amax)) return 1.0f;
  int e;
  frexpf(amax, &e);  // amax < 2^e
  return ldexpf(1.0f, 14 - e);
}

// a threshold t in score space moved to the pre-constant score y (score = y + c): lowered by a
// margin that covers both roundings (y + c rounded >= t implies y >= the result), -inf -> -FLT_MAX,
// +inf stays +inf
__device__ __forceinline__ float lower_thr(float t, float c) {
  const float lowered = (t - c) - 0x1p-20f * (fabsf(t) + fabsf(c));
  return isinf(t) ? (t > 0.0f ? t : -3.402823466e+38f) : fmaxf(lowered, -3.402823466e+38f);
}

#ifdef PYR_STREAM_EMIT
// ---- the stream scans' candidate emission (scan.hip, pq32.hip): query-major buffers (StreamArgs::cand)
// one row straight to query q's buffer (a row that finds it full raises the query's floor)
__device__ __forceinline__ void cand_put(const StreamArgs &a, int q, float sc, uint32_t key) {
  const int slot = atomicAdd(a.cand_n + q, 1);
  if (slot < a.cap) a.cand[(size_t)q * a.cap + slot] = make_uint2(__float_as_uint(sc), key);
  else atomicMax(a.cand_f + q, score_key(sc));
}
// An item's staged rows eb[0, n) ({score bits, query slot << 23 | row offset}) to their queries'
// buffers: the rows per query slot are counted (LDS), each query reserves its run with ONE global
// atomic, then every row takes its place in the run.  cnt / base: per query slot LDS arrays (cnt zero
// on entry; the next item's prologue zeroes it again); qid(i): the query of slot i.  Block-wide (NT
// threads, barriers).
template <int NT, class QID>
__device__ __forceinline__ void cand_flush(const StreamArgs &a, const uint2 *eb, int n, int qcnt, int r0, int *cnt,
                                           int *base, QID qid) {
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += NT) atomicAdd(&cnt[eb[i].y >> 23], 1);
  __syncthreads();
  for (int i = tid; i < qcnt; i += NT) {
    const int c = cnt[i];
    base[i] = c > 0 ? atomicAdd(a.cand_n + qid(i), c) : 0;
    cnt[i] = 0;
  }
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    const uint2 e = eb[i];
    const int qi = (int)(e.y >> 23);
    const int slot = base[qi] + atomicAdd(&cnt[qi], 1);
    const int q = qid(qi);
    if (slot < a.cap) a.cand[(size_t)q * a.cap + slot] = make_uint2(e.x, a.key_base | (uint32_t)(r0 + (int)(e.y & 0x7FFFFFu)));
    else atomicMax(a.cand_f + q, score_key(__uint_as_float(e.x)));
  }
}
#endif
