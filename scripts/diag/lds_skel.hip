// Microbenchmark (diagnostic): the stream16 MAIN loop's LDS operand traffic alone -- 8 waves per block,
// one block per CU, 128 KiB of LDS operands, per group 1 record + 4 x ds_read_b128, read one group ahead
// (as the production loop).  Prints cycles per group per wave.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <bool MFMA, bool EPI, bool LOAD>
__global__ __launch_bounds__(512, 1) void skel(int groups, int iters, float *out, unsigned long long *cyc, const h8v *tiles, long ntiles) {
  __shared__ __attribute__((aligned(16))) char bl[32 * 4 * 1024];
  __shared__ float4 qr[512];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15;
  for (int i = tid; i < 32 * 4 * 1024 / 4; i += 512) reinterpret_cast<float *>(bl)[i] = 0.001f * (i & 7);
  for (int i = tid; i < 512; i += 512) qr[i] = make_float4(1.0f, 2.0f, 3.0f, 4.0f);
  __syncthreads();
  h8v A[4][2];
  for (int s = 0; s < 4; ++s) for (int b = 0; b < 2; ++b) for (int e = 0; e < 8; ++e) A[s][b][e] = (_Float16)(0.01f * (lane + s + b + e));
  f4v acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  float sink = 0.0f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // LOAD: the wave's A tile (8 KiB: 8 x 16 B per lane) streamed from HBM once per `groups` groups,
  // prefetched one tile ahead as the production loop does (tile t + 8 of a persistent walk)
  h8v An[4][2];
  long tix = (long)blockIdx.x * 8 + (tid >> 6);
  auto ld = [&](long t, h8v (&X)[4][2]) {
    const h8v *tp = tiles + (t % ntiles) * 512 + (lane & 15) + 16 * (lane >> 4);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      X[s2][0] = tp[s2 * 128];
      X[s2][1] = tp[s2 * 128 + 64];
    }
  };
  if (LOAD) ld(tix, A);
  for (int it = 0; it < iters; ++it) {
    if (LOAD) {
      tix += (long)gridDim.x * 8;
      ld(tix, An);
    }
    h8v b0[4], b1[4];
    auto rd = [&](int j, h8v (&B)[4]) {
      const char *bp = bl + j * 4 * 1024 + lane * 16;
#pragma unroll
      for (int s = 0; s < 4; ++s) B[s] = *reinterpret_cast<const h8v *>(bp + s * 1024);
    };
    rd(0, b0);
    rd(1, b1);
    for (int j = 0; j < groups; j += 2) {
      const float4 rp = qr[16 * j + c];
      if (MFMA) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][0], b0[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][1], b0[s], acc[1], 0, 0, 0);
        }
      } else {
        sink += (float)b0[0][0] + (float)b0[3][7];
      }
      rd(min(j + 2, groups - 1), b0);
      if (EPI) {  // the production epilogue: y = f acc + meta, max, compare, ballot (branch never taken)
        float y[8], mx;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i) y[4 * b + i] = fmaf(rp.x, acc[b][i], rp.z + i);
        mx = fmaxf(fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])), fmaxf(fmaxf(y[4], y[5]), fmaxf(y[6], y[7])));
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(mx >= rp.w * 1e30f) != 0ull, 0)) sink += mx;
      }
      sink += rp.x;
      const float4 rj = qr[16 * (j + 1) + c];
      if (MFMA) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][0], b1[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][1], b1[s], acc[1], 0, 0, 0);
        }
      } else {
        sink += (float)b1[0][0] + (float)b1[3][7];
      }
      rd(min(j + 3, groups - 1), b1);
      if (EPI) {
        float y[8], mx;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i) y[4 * b + i] = fmaf(rj.x, acc[b][i], rj.z + i);
        mx = fmaxf(fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])), fmaxf(fmaxf(y[4], y[5]), fmaxf(y[6], y[7])));
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(mx >= rj.w * 1e30f) != 0ull, 0)) sink += mx;
      }
      sink += rj.y;
    }
    if (LOAD) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        A[s2][0] = An[s2][0];
        A[s2][1] = An[s2][1];
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + tid] = sink + acc[0][0] + acc[1][1];
  if (lane == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
  int cus = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) cus = p.multiProcessorCount;
  float *out;
  unsigned long long *cyc, h;
  hipMalloc(&out, sizeof(float) * cus * 512);
  hipMalloc(&cyc, 8);
  const int groups = 20, iters = 200;
  h8v *tiles;
  const long ntiles = 2 * 1024 * 1024 / 8;  // 2 GiB of tiles (8 KiB each), far beyond the caches
  hipMalloc(&tiles, ntiles * 8192);
  hipMemset(tiles, 0, ntiles * 8192);
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipMemset(cyc, 0, 8);
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      if (mode == 3) hipLaunchKernelGGL((skel<true, true, true>), dim3(cus), dim3(512), 0, 0, groups, iters, out, cyc, tiles, ntiles);
      else if (mode == 2) hipLaunchKernelGGL((skel<true, true, false>), dim3(cus), dim3(512), 0, 0, groups, iters, out, cyc, tiles, ntiles);
      else if (mode == 1) hipLaunchKernelGGL((skel<true, false, false>), dim3(cus), dim3(512), 0, 0, groups, iters, out, cyc, tiles, ntiles);
      else hipLaunchKernelGGL((skel<false, false, false>), dim3(cus), dim3(512), 0, 0, groups, iters, out, cyc, tiles, ntiles);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      const double per = (double)h / (cus * 8.0) / (iters * (double)groups);
      printf("%s: %.3f ms, %.1f cycles (s_memtime) per group per wave\n", mode == 3 ? "LDS reads + 8 MFMA + epilogue + HBM tile stream" : mode == 2 ? "LDS reads + 8 MFMA + epilogue" : (mode ? "LDS reads + 8 MFMA" : "LDS reads only"), ms, per);
    }
  }
  return 0;
}
