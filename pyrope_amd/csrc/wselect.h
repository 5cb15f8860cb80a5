// wselect.h -- one wave's radix select over a row of fp32 scores (device helper shared by the stream
// scan's threshold pass, stream16.hip, and the matrix-core coarse ranking, coarse.hip).
#pragma once

// The score_key (kernels.h, order-preserving u32) of the K-th largest of v[0 .. n), 1 <= K <= n,
// 8-bit digits over 4 passes, counted in `hist` (256 ints of LDS owned by this wave).  CACHE values
// per lane are loaded at once (all independent, one memory latency per chunk), and kept in registers
// across the passes when the row fits (n <= 64 CACHE).  cv returns those cached values.
template <int CACHE>
__device__ __forceinline__ uint32_t wave_kth_key(const float *v, int n, int K, int *hist, int lane,
                                                 float (&cv)[CACHE]) {
  const bool cached = n <= 64 * CACHE;
  if (cached) {
#pragma unroll
    for (int u = 0; u < CACHE; ++u) cv[u] = lane + 64 * u < n ? v[lane + 64 * u] : 0.0f;
  }
  uint32_t prefix = 0u, pmask = 0u;
  int rem = K;
  for (int shift = 24; shift >= 0; shift -= 8) {
#pragma unroll
    for (int i = 0; i < 4; ++i) hist[lane + 64 * i] = 0;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    auto count = [&](const float (&x)[CACHE], int base) {
#pragma unroll
      for (int u = 0; u < CACHE; ++u) {
        if (base + lane + 64 * u >= n) break;
        const uint32_t k = score_key(x[u]);
        if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
      }
    };
    if (cached) {
      count(cv, 0);
    } else {
      for (int base = 0; base < n; base += 64 * CACHE) {
        float x[CACHE];
#pragma unroll
        for (int u = 0; u < CACHE; ++u) x[u] = base + lane + 64 * u < n ? v[base + lane + 64 * u] : 0.0f;
        count(x, base);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // lane l holds bins 4l .. 4l+3; above(l) = values in the bins of higher lanes
    int h4[4], s4 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      h4[i] = hist[4 * lane + i];
      s4 += h4[i];
    }
    int incl = s4;  // suffix sum over lanes >= l
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_down(incl, off);
      if (lane + off < 64) incl += o;
    }
    const int above = incl - s4;
    int bin = -1, before = 0;
    if (above < rem && incl >= rem) {
      int acc = above;
      for (int i = 3; i >= 0; --i) {
        if (acc + h4[i] >= rem) {
          bin = 4 * lane + i;
          before = acc;
          break;
        }
        acc += h4[i];
      }
    }
    const uint64_t m = __builtin_amdgcn_ballot_w64(bin >= 0);
    const int src = m ? (int)__builtin_ctzll(m) : 0;  // exactly one lane found it (K <= n)
    bin = __shfl(bin, src);
    before = __shfl(before, src);
    prefix |= (uint32_t)bin << shift;
    pmask |= 255u << shift;
    rem -= before;
    __builtin_amdgcn_wave_barrier();
  }
  return prefix;
}

__device__ __forceinline__ uint32_t wsort32_desc(uint32_t v, int lane) {  // bitonic, 64 lanes
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j >= 1; j >>= 1) {
      const uint32_t o = (uint32_t)__shfl_xor((int)v, j);
      const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == desc) ? (v > o ? v : o) : (v < o ? v : o);
    }
  return v;
}

// The same K-th largest key (K <= 64) without histograms (the radix passes' LDS atomics serialise when a
// row's keys share their top bytes, as scores of one query do): L = the K-th largest of the 64 lanes'
// maxima bounds the answer from below (K distinct values reach it), every key >= L is gathered (`buf`:
// 64 ints of LDS owned by this wave) and sorted when there are at most 64 of them -- typically about K;
// otherwise the radix select above.  Two streaming reads of the row, or none beyond the first when it
// fits the CACHE registers per lane.
template <int CACHE>
__device__ __forceinline__ uint32_t wave_kth_key_lm(const float *v, int n, int K, int *hist, int *buf, int lane,
                                                    float (&cv)[CACHE]) {
  const bool cached = n <= 64 * CACHE;
  uint32_t mk = 0u;
  if (cached) {
#pragma unroll
    for (int u = 0; u < CACHE; ++u) {
      cv[u] = lane + 64 * u < n ? v[lane + 64 * u] : 0.0f;
      if (lane + 64 * u < n) mk = max(mk, score_key(cv[u]));
    }
  } else {
    for (int base = 0; base < n; base += 64 * CACHE) {
      float x[CACHE];
#pragma unroll
      for (int u = 0; u < CACHE; ++u) x[u] = base + lane + 64 * u < n ? v[base + lane + 64 * u] : 0.0f;
#pragma unroll
      for (int u = 0; u < CACHE; ++u)
        if (base + lane + 64 * u < n) mk = max(mk, score_key(x[u]));
    }
  }
  const uint32_t L = (uint32_t)__shfl((int)wsort32_desc(mk, lane), K - 1);
  int cnt = 0;
  auto gather = [&](uint32_t k, bool in) {
    const bool p = in && k >= L;
    const uint64_t m = __builtin_amdgcn_ballot_w64(p);
    const int pos = cnt + (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    if (p && pos < 64) buf[pos] = (int)k;
    cnt += (int)__builtin_popcountll(m);
  };
  if (cached) {
#pragma unroll
    for (int u = 0; u < CACHE; ++u)
      if (64 * u < n) gather(score_key(cv[u]), lane + 64 * u < n);
  } else {
    for (int i = 0; i < n; i += 64) {
      const bool in = i + lane < n;
      gather(in ? score_key(v[i + lane]) : 0u, in);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if (cnt > 64) return wave_kth_key<CACHE>(v, n, K, hist, lane, cv);
  const uint32_t mine = lane < cnt ? (uint32_t)buf[lane] : 0u;
  __builtin_amdgcn_wave_barrier();
  return (uint32_t)__shfl((int)wsort32_desc(mine, lane), K - 1);
}
