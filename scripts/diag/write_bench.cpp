// Single-row adds through the C ABI, timed natively (no Python): the per-call cost of the small-batch write
// path, and the HIP calls it is made of, each timed alone.  Build + run (GPU box):
//   hipcc -O2 -Iinclude scripts/diag/write_bench.cpp -Lpyrope_amd -lpyrope_hip -Wl,-rpath,$PWD/pyrope_amd -o /tmp/wb
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "pyrope_ann.h"

struct Big {
  void *p[16];
  float f[8];
  int i[8];
};
__global__ void small_k(int *p) {
  if (p && threadIdx.x == 0) p[0] = 1;
}
__global__ void big_k(Big b) {
  if (b.p[0] && threadIdx.x == 0) static_cast<int *>(b.p[0])[0] = 1;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const int D = 128, base = 200000, adds = 50000;
  pyr_index_desc d{};
  d.kind = PYR_FLAT;
  d.dim = D;
  d.metric = 0;
  pyr_index *ix = nullptr;
  if (pyr_index_create(&d, &ix)) return printf("create: %s\n", pyr_last_error()), 1;
  std::vector<float> x((size_t)(base + adds) * D);
  for (size_t i = 0; i < x.size(); ++i) x[i] = (float)((i * 2654435761u) % 1000) / 1000.0f;
  std::vector<int64_t> lab(base + adds);
  for (int i = 0; i < base + adds; ++i) lab[i] = i;
  pyr_index_reserve(ix, base + adds);
  pyr_index_add(ix, x.data(), base, lab.data());
  double t = now();
  for (int i = base; i < base + adds; ++i)
    if (pyr_index_add(ix, x.data() + (size_t)i * D, 1, lab.data() + i)) return printf("add: %s\n", pyr_last_error()), 1;
  const double ta = now() - t;
  hipDeviceSynchronize();
  const double tb = now() - t;
  printf("single-row adds: %.1f us per call (%.0f/s), %.1f us per add including the device drain\n", 1e6 * ta / adds,
         adds / ta, 1e6 * tb / adds);
  // the HIP calls alone
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int N = 20000;
  t = now();
  for (int i = 0; i < N; ++i) hipEventRecord(ev, st);
  printf("hipEventRecord: %.2f us\n", 1e6 * (now() - t) / N);
  t = now();
  for (int i = 0; i < N; ++i) hipSetDevice(0);
  printf("hipSetDevice: %.2f us\n", 1e6 * (now() - t) / N);
  t = now();
  for (int i = 0; i < N; ++i) hipEventQuery(ev);
  printf("hipEventQuery: %.2f us\n", 1e6 * (now() - t) / N);
  hipStreamSynchronize(st);
  t = now();
  for (int i = 0; i < N; ++i) hipEventSynchronize(ev);
  printf("hipEventSynchronize (complete): %.2f us\n", 1e6 * (now() - t) / N);
  int *dp;
  hipMalloc(&dp, 64);
  t = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(small_k, dim3(1), dim3(64), 0, st, dp);
  printf("launch (8-B arg): %.2f us\n", 1e6 * (now() - t) / N);
  Big b{};
  b.p[0] = dp;
  t = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(big_k, dim3(1), dim3(64), 0, st, b);
  printf("launch (192-B arg): %.2f us\n", 1e6 * (now() - t) / N);
  hipStreamSynchronize(st);
  std::vector<char> hb(1024);
  void *hp;
  hipHostMalloc(&hp, 4096, hipHostMallocMapped);
  t = now();
  for (int i = 0; i < N; ++i) hipMemcpyAsync(dp, hp, 64, hipMemcpyHostToDevice, st);
  printf("hipMemcpyAsync pinned 64 B: %.2f us\n", 1e6 * (now() - t) / N);
  hipStreamSynchronize(st);
  pyr_index_destroy(ix);
  return 0;
}
