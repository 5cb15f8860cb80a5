// ldsdma_bw.hip -- measurement only: HBM -> LDS streaming rate of the list-scan tile ring shape.
//
// Every block streams its own contiguous chunk of 8 KiB tiles (the fp16 h16 tiles of D = 128) into
// an NST-slot LDS ring by global_load_lds_dwordx4 (one 1 KiB piece per loading wave per tile), with
// the list scan's counted vmcnt wait + one barrier per STEP tiles, and nothing else.  Compared with
// the same stream into registers (global_load_dwordx4).  Prints GB/s for each shape.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ldsdma_bw scripts/diag/ldsdma_bw.hip && /tmp/ldsdma_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void *g, uint32_t lds_addr) {
  int keep;
  const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

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

constexpr int TB = 8192;  // tile bytes

// NW waves, the first NL of them load (TB / NL bytes each per tile: 1 KiB pieces), NST ring slots
template <int NW, int NL, int NST, int STEP>
__global__ __launch_bounds__(64 * NW) void ring_kernel(const char *src, int64_t tiles_per_block, float *out) {
  constexpr int PPW = TB / 1024 / NL;  // pieces per loading wave per tile
  __shared__ __attribute__((aligned(16))) char ring[NST * TB];
  const uint32_t base = (uint32_t)(size_t)(lds_void *)ring;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char *chunk = src + (size_t)blockIdx.x * tiles_per_block * TB;
  const int nt = (int)tiles_per_block;
  auto issue = [&](int t) {
    if (w < NL)
#pragma unroll
      for (int p = 0; p < PPW; ++p) {
        const int piece = w * PPW + p;
        glds16(chunk + (size_t)t * TB + piece * 1024 + lane * 16, base + (t % NST) * TB + piece * 1024);
      }
  };
  for (int t = 0; t < NST - STEP && t < nt; ++t) issue(t);
  float acc = 0.0f;
  for (int st = 0; st < nt; st += STEP) {
    const int last = min(st + STEP, nt) - 1;
    if (w < NL) wait_vm_le<64>(PPW * max(0, min(NST - 2 * STEP, nt - 1 - last)));
    __builtin_amdgcn_s_barrier();
    for (int u = 0; u < STEP; ++u)
      if (st + NST - STEP + u < nt) issue(st + NST - STEP + u);
    for (int u = 0; u < STEP && st + u < nt; ++u) acc += reinterpret_cast<const float *>(ring + ((st + u) % NST) * TB)[lane];
  }
  if (acc == 12345.0f) out[blockIdx.x] = acc;
}

// the same stream into registers: each wave loads its 1 KiB piece per tile, UNR tiles in flight
template <int NW, int UNR>
__global__ __launch_bounds__(64 * NW) void reg_kernel(const char *src, int64_t tiles_per_block, float *out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char *chunk = src + (size_t)blockIdx.x * tiles_per_block * TB;
  float acc = 0.0f;
  for (int64_t t = 0; t < tiles_per_block; t += UNR) {
    float4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      v[u] = t + u < tiles_per_block ? *reinterpret_cast<const float4 *>(chunk + (size_t)(t + u) * TB + (w % 8) * 1024 + lane * 16)
                                     : float4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u].x;
  }
  if (acc == 12345.0f) out[blockIdx.x] = acc;
}

template <class F>
double timeit(F f, double bytes) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return bytes * 5 / (ms * 1e-3) / 1e9;
}

int main() {
  const int64_t total = int64_t(2600) << 20;  // ~2.6 GiB, the I1 fp16 tile bytes
  char *src;
  float *out;
  CHK(hipMalloc(&src, total));
  CHK(hipMalloc(&out, 1 << 20));
  CHK(hipMemset(src, 1, total));
  const int64_t tiles = total / TB;
  for (int blocks : {256, 512, 1024, 2048}) {
    const int64_t tpb = tiles / blocks;
    const double bytes = (double)tpb * blocks * TB;
#define RUN(NW, NL, NST, STEP)                                                                                   \
  printf("blocks %5d ring NW=%2d NL=%d NST=%2d STEP=%d: %7.0f GB/s\n", blocks, NW, NL, NST, STEP,                \
         timeit([&] { hipLaunchKernelGGL((ring_kernel<NW, NL, NST, STEP>), dim3(blocks), dim3(64 * NW), 0, 0, src, \
                                         tpb, out); }, bytes));
    RUN(8, 8, 4, 2)
    RUN(8, 8, 8, 2)
    RUN(8, 8, 16, 2)
    RUN(8, 4, 8, 2)
    RUN(8, 2, 8, 2)
    RUN(8, 1, 8, 2)
    RUN(16, 8, 8, 2)
    RUN(4, 4, 8, 2)
    RUN(4, 4, 16, 4)
    printf("blocks %5d reg  NW=8 UNR=4: %7.0f GB/s\n", blocks,
           timeit([&] { hipLaunchKernelGGL((reg_kernel<8, 4>), dim3(blocks), dim3(512), 0, 0, src, tpb, out); }, bytes));
    printf("blocks %5d reg  NW=8 UNR=8: %7.0f GB/s\n", blocks,
           timeit([&] { hipLaunchKernelGGL((reg_kernel<8, 8>), dim3(blocks), dim3(512), 0, 0, src, tpb, out); }, bytes));
    fflush(stdout);
  }
  return 0;
}
