// Diagnostic: how fast can the [N x 107] f32 obs stream be written?  Variants of
// a write-only kernel (65536 envs, 28 MB per launch): tile size per workgroup,
// persistent grid, store cache policy.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/write_probe tools/diag/write_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kD = 107;
typedef float v4f __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if (POL == 0) *p = v;
  else if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// ENVS envs per tile, THREADS threads, TILES tiles per workgroup (grid-stride)
template <int ENVS, int THREADS, int POL>
__global__ __launch_bounds__(THREADS) void wprobe(float* __restrict__ obs, int n) {
  const int ntiles = n / ENVS;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    v4f* d4 = reinterpret_cast<v4f*>(obs + (int64_t)t * ENVS * kD);
    for (int k = threadIdx.x; k < ENVS * kD / 4; k += THREADS) {
      const float f = (float)(k & 1023);
      st<POL>(d4 + k, v4f{f, f + 1.f, f + 2.f, f + 3.f});
    }
  }
}

template <int ENVS, int THREADS, int POL>
float run(float* obs, int n, int grid, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((wprobe<ENVS, THREADS, POL>), dim3(grid), dim3(THREADS), 0, 0, obs, n);
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((wprobe<ENVS, THREADS, POL>), dim3(grid), dim3(THREADS), 0, 0, obs, n);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int n = 65536, reps = 500;
  float* obs;
  (void)hipMalloc(&obs, (size_t)n * kD * 4);
  printf("{\"envs\": %d, \"MB\": %.1f, \"us_per_launch\": {", n, n * kD * 4 / 1e6);
  printf("\"t64x256_plain\": %.3f, ", run<64, 256, 0>(obs, n, n / 64, reps));
  printf("\"t64x256_sc1\": %.3f, ", run<64, 256, 1>(obs, n, n / 64, reps));
  printf("\"t64x256_nt\": %.3f, ", run<64, 256, 2>(obs, n, n / 64, reps));
  printf("\"t64x256_sc0sc1nt\": %.3f, ", run<64, 256, 3>(obs, n, n / 64, reps));
  printf("\"t128x512_sc1\": %.3f, ", run<128, 512, 1>(obs, n, n / 128, reps));
  printf("\"t64x64_sc1\": %.3f, ", run<64, 64, 1>(obs, n, n / 64, reps));
  printf("\"t64x256_sc1_persist512\": %.3f, ", run<64, 256, 1>(obs, n, 512, reps));
  printf("\"t64x256_sc1_persist256\": %.3f, ", run<64, 256, 1>(obs, n, 256, reps));
  printf("\"t64x1024_sc1\": %.3f, ", run<64, 1024, 1>(obs, n, n / 64, reps));
  printf("\"empty_grid1024\": %.3f}}\n", run<64, 256, 1>(obs, 0, n / 64, reps));
  return 0;
}
