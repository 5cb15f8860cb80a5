// candmerge.h -- the stream scans' per-query candidate merge, shared by cand_merge_kernel (sample16.hip) and
// the fused merge + certified refine (filter.hip).  Internal; include inside an anonymous namespace of a
// .hip file's pyr namespace, after <hip/hip_runtime.h> and kernels.h.
#pragma once

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}
// rank key: score desc, then storage key asc (~key); 0 = no entry
__device__ __forceinline__ uint64_t pack_cand(float s, uint32_t k) { return ((uint64_t)score_key(s) << 32) | (uint32_t)~k; }

__device__ __forceinline__ uint64_t sort64_desc(uint64_t v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j >= 1; j >>= 1) {
      const uint64_t o = shfl_xor64(v, j);
      const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
      v = (lower == desc) ? (v > o ? v : o) : (v < o ? v : o);
    }
  return v;
}
__device__ __forceinline__ uint64_t merge64_desc(uint64_t v, int lane) {  // v bitonic -> sorted desc
#pragma unroll
  for (int j = 32; j >= 1; j >>= 1) {
    const uint64_t o = shfl_xor64(v, j);
    v = (lane & j) == 0 ? (v > o ? v : o) : (v < o ? v : o);
  }
  return v;
}


// Query q's emitted rows (m.cand, query-major) merged with KO copies of its floor placeholder
// max(T_q, floor) (KEY_FLOOR): lane j returns the j-th best rank key (score bound desc, storage key asc;
// 0 = none).  Every row left out scores at most the KO-th.
template <int KO>
__device__ __forceinline__ uint64_t cand_merge_wave(const CandMergeArgs &m, int64_t q, int lane) {
  const int tot = min(m.cand_n[q], m.cap);
  const uint32_t fk = m.cand_f[q];
  float F = m.thr ? m.thr[q] : -INFINITY;
  if (fk != 0u) F = fmaxf(F, key_score(fk));
  const uint2 *cq = m.cand + (size_t)q * m.cap;
  uint64_t cur = F > -INFINITY ? pack_cand(F, KEY_FLOOR) : 0ull;
  for (int base = 0; base < tot; base += 64) {
    const int idx = base + lane;
    uint64_t v = 0ull;
    if (idx < tot) {
      const uint2 e = cq[idx];
      v = pack_cand(__uint_as_float(e.x), e.y);
    }
    const uint64_t kth = shfl64(cur, KO - 1);
    if (!__builtin_amdgcn_ballot_w64(v > kth)) continue;
    v = sort64_desc(v, lane);
    const uint64_t r = shfl64(v, 63 - lane);
    cur = cur > r ? cur : r;
    cur = merge64_desc(cur, lane);
  }
  return cur;
}
