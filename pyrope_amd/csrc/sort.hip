// sort.hip -- the k-means / list-layout grouping sort (sort_by_key, kernels.h): hipcub radix sort and
// exclusive scan.  Its own translation unit: rocPRIM's configuration instantiations dominate a file's
// compile time, and here they build in parallel with the kernels.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace pyr {
namespace {

unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

__global__ void iota_kernel(int32_t *p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (int32_t)i;
}
__global__ void hist_kernel(const int32_t *keys, int64_t n, int32_t *counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&counts[keys[i]], 1);
}

}  // namespace

static int key_bits(int32_t k) {
  int b = 1;
  while ((1 << b) < k) ++b;
  return b;
}

size_t sort_temp_bytes(int64_t n, int32_t k) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const int32_t *)nullptr, (int32_t *)nullptr,
                                           (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, key_bits(k));
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t *)nullptr, (int32_t *)nullptr, k + 1);
  return (a > b ? a : b) + 256;
}

void sort_by_key(const int32_t *keys, int64_t n, int32_t k, int32_t *keys_tmp, int32_t *idx_in, int32_t *members,
                 int32_t *counts, int32_t *coff, void *temp, size_t temp_bytes, hipStream_t st) {
  hipLaunchKernelGGL(iota_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, idx_in, n);
  size_t tb = temp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(temp, tb, keys, keys_tmp, idx_in, members, (int)n, 0, key_bits(k), st);
  (void)hipMemsetAsync(counts, 0, sizeof(int32_t) * (k + 1), st);
  hipLaunchKernelGGL(hist_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, keys, n, counts);
  tb = temp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(temp, tb, counts, coff, k + 1, st);
}

}  // namespace pyr
