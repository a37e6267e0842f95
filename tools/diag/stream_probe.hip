// Diagnostic: the floor of a one-round step design.  Per workgroup of 64 envs:
// read RB bytes of contiguous per-env state (coalesced 16-B loads into LDS), write
// 16 B of state back per env and the [64 x 107] f32 obs tile (sc1 16-B stores,
// as pe_step_quad).  No env semantics -- only the memory pattern.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/stream_probe tools/diag/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kD = 107;

template <int RB>
__global__ __launch_bounds__(256) void probe(const uint4* __restrict__ state, uint4* __restrict__ scal_out,
                                             float* __restrict__ obs, int n) {
  __shared__ __attribute__((aligned(16))) float tile[64 * kD + 4];
  __shared__ uint4 img[RB > 0 ? 64 * RB / 16 : 1];
  const int64_t e0 = (int64_t)blockIdx.x * 64;
  constexpr int per_env = RB / 16;
  if (RB > 0) {
    const uint4* src = state + e0 * per_env;
    for (int k = threadIdx.x; k < 64 * per_env; k += 256) img[k] = src[k];
  }
  __syncthreads();
  // each thread builds part of the tile from the image (keeps the loads live)
  for (int k = threadIdx.x; k < 64 * kD; k += 256) {
    const int env = k / kD;
    uint32_t v = (uint32_t)k;
    if (RB > 0) {
      const uint4 w = img[env * per_env + (k % per_env)];
      v ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    tile[k] = (float)(v & 1023u) * (1.0f / 1024.0f);
  }
  if (threadIdx.x < 64 && RB > 0) {
    const uint4 w = img[threadIdx.x * per_env];
    scal_out[e0 + threadIdx.x] = make_uint4(w.x + 1u, w.y, w.z, w.w);
  }
  __syncthreads();
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f* sv = reinterpret_cast<const v4f*>(tile);
  v4f* d4 = reinterpret_cast<v4f*>(obs + e0 * kD);
  for (int k = threadIdx.x; k < 64 * kD / 4; k += 256) {
    const v4f v = sv[k];
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(d4 + k), "v"(v) : "memory");
  }
}

template <int RB>
float run(int n, const uint4* state, uint4* scal, float* obs, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(probe<RB>, dim3(n / 64), dim3(256), 0, 0, state, scal, obs, n);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(probe<RB>, dim3(n / 64), dim3(256), 0, 0, state, scal, obs, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int n = 65536, reps = 500;
  uint4* state;
  uint4* scal;
  float* obs;
  hipMalloc(&state, (size_t)n * 512);
  hipMalloc(&scal, (size_t)n * 16);
  hipMalloc(&obs, (size_t)n * kD * 4);
  hipMemset(state, 1, (size_t)n * 512);
  printf("{\"envs\": %d, \"us_per_launch\": {", n);
  printf("\"read0\": %.3f, ", run<0>(n, state, scal, obs, reps));
  printf("\"read176\": %.3f, ", run<176>(n, state, scal, obs, reps));
  printf("\"read320\": %.3f, ", run<320>(n, state, scal, obs, reps));
  printf("\"read480\": %.3f}}\n", run<480>(n, state, scal, obs, reps));
  return 0;
}
