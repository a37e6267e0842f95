// Diagnostic: does overlapping the obs-tile store of one chunk with the state
// loads of the next pay?  Memory pattern only (no env semantics), 64 envs per
// chunk, [64 x 107] f32 obs tile stored with sc1 16-B stores as pe_step_quad.
//
//   flat<RB>          one chunk per workgroup (4 waves): load RB B/env into LDS,
//                     build the tile, store it (= stream_probe.hip)
//   flat2<RB>         same, but two dependent rounds: 16 B of scalars, then RB
//                     bytes at an offset read from the scalars (gather-like)
//   ws<RB, K, TWO>    persistent, wave-specialised: 4 "compute" waves only load
//                     (+ build the tile in LDS), 4 "store" waves only store the
//                     previous chunk's tile (double-buffered), K chunks per
//                     workgroup; gfx9 counts loads and stores in one vmcnt, so
//                     the split keeps the loaders' waits free of the stores
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/pipe_probe tools/diag/pipe_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kD = 107;
constexpr int kBlk = 512;  // per-env state block in the probe's buffer (bytes)

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store_sc1(float* dst, const float* tile, int t, int nt) {
  const v4f* sv = reinterpret_cast<const v4f*>(tile);
  v4f* d4 = reinterpret_cast<v4f*>(dst);
  for (int k = t; k < 64 * kD / 4; k += nt) {
    const v4f v = sv[k];
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(d4 + k), "v"(v) : "memory");
  }
}

template <int RB>
__device__ __forceinline__ void build_tile(float* tile, const uint4* img, int t, int nt) {
  constexpr int per_env = RB / 16 > 0 ? RB / 16 : 1;
  for (int k = t; k < 64 * kD; k += nt) {
    const int env = k / kD;
    uint32_t v = (uint32_t)k;
    if (RB > 0) {
      const uint4 w = img[env * per_env + (k % per_env)];
      v ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    tile[k] = (float)(v & 1023u) * (1.0f / 1024.0f);
  }
}

// round-2 offset of env e's block, from its scalars (always 0 in the buffer,
// but the compiler cannot know: the second round depends on the first)
__device__ __forceinline__ int off_from(uint4 s) { return (int)(s.x & 0x10u); }

template <int RB, bool TWO>
__global__ __launch_bounds__(256) void flat(const uint4* __restrict__ state, const uint4* __restrict__ scal,
                                            uint4* __restrict__ scal_out, float* __restrict__ obs) {
  __shared__ __attribute__((aligned(16))) float tile[64 * kD + 4];
  __shared__ uint4 img[RB > 0 ? 64 * RB / 16 : 1];
  __shared__ int offs[64];
  const int64_t e0 = (int64_t)blockIdx.x * 64;
  constexpr int per_env = RB / 16;
  uint4 s = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < 64) s = scal[e0 + threadIdx.x];
  if (TWO) {
    if (threadIdx.x < 64) offs[threadIdx.x] = off_from(s);
    __syncthreads();
  }
  if (RB > 0) {
    for (int k = threadIdx.x; k < 64 * per_env; k += 256) {
      const int env = k / per_env, j = k % per_env;
      const int o = TWO ? offs[env] : 0;
      img[k] = state[(e0 + env) * (kBlk / 16) + j + o];
    }
  }
  __syncthreads();
  build_tile<RB>(tile, img, threadIdx.x, 256);
  if (threadIdx.x < 64) scal_out[e0 + threadIdx.x] = make_uint4(s.x + 1u, s.y, s.z, s.w);
  __syncthreads();
  store_sc1(obs + e0 * kD, tile, threadIdx.x, 256);
}

// ws: waves 0-3 load chunk i and build tile[i&1]; waves 4-7 store tile[(i-1)&1]
// and the previous chunk's scalars.  Two barriers per iteration.
template <int RB, int K, bool TWO>
__global__ __launch_bounds__(512) void ws(const uint4* __restrict__ state, const uint4* __restrict__ scal,
                                          uint4* __restrict__ scal_out, float* __restrict__ obs, int nchunks) {
  __shared__ __attribute__((aligned(16))) float tile[2][64 * kD + 4];
  __shared__ uint4 img[RB > 0 ? 64 * RB / 16 : 1];
  __shared__ uint4 lsc[2][64];
  __shared__ int offs[64];
  constexpr int per_env = RB / 16;
  const int t = threadIdx.x;
  const bool loader = t < 256;
  for (int i = 0; i <= K; ++i) {
    const int c = blockIdx.x + i * gridDim.x;      // chunk of this iteration (loaders)
    const int cp = blockIdx.x + (i - 1) * gridDim.x;  // previous chunk (storers)
    if (loader) {
      if (i < K && c < nchunks) {
        const int64_t e0 = (int64_t)c * 64;
        uint4 s = make_uint4(0, 0, 0, 0);
        if (t < 64) s = scal[e0 + t];
        if (TWO) {
          if (t < 64) offs[t] = off_from(s);
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): ds_write visible to the team
          __builtin_amdgcn_s_barrier();          // (storers: matching barrier below)
        }
        if (RB > 0) {
          for (int k = t; k < 64 * per_env; k += 256) {
            const int env = k / per_env, j = k % per_env;
            const int o = TWO ? offs[env] : 0;
            img[k] = state[(e0 + env) * (kBlk / 16) + j + o];
          }
        }
        if (t < 64) lsc[i & 1][t] = make_uint4(s.x + 1u, s.y, s.z, s.w);
      } else if (TWO) {
        __builtin_amdgcn_s_barrier();
      }
    } else {
      if (TWO) __builtin_amdgcn_s_barrier();
      if (i > 0 && cp < nchunks) {
        const int64_t e0 = (int64_t)cp * 64;
        store_sc1(obs + e0 * kD, tile[(i - 1) & 1], t - 256, 256);
        if (t - 256 < 64) scal_out[e0 + t - 256] = lsc[(i - 1) & 1][t - 256];
      }
    }
    __syncthreads();  // img complete (loaders); tile[(i-1)&1] read into VGPRs (storers)
    if (loader && i < K && c < nchunks) build_tile<RB>(tile[i & 1], img, t, 256);
    __syncthreads();  // tile[i&1] complete; img free
  }
}

template <typename F>
float timeit(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int n = 65536, reps = 400, nch = n / 64;
  uint4 *state, *scal, *scal_out;
  float* obs;
  hipMalloc(&state, (size_t)n * kBlk + 4096);
  hipMalloc(&scal, (size_t)n * 16);
  hipMalloc(&scal_out, (size_t)n * 16);
  hipMalloc(&obs, (size_t)n * kD * 4);
  hipMemset(state, 1, (size_t)n * kBlk + 4096);
  hipMemset(scal, 0, (size_t)n * 16);
  printf("{\"envs\": %d, \"us_per_launch\": {", n);
#define FLAT(RB, TWO)                                                                                   \
  printf("\"flat%s_%d\": %.3f, ", TWO ? "2" : "", RB, timeit([&] {                                      \
           hipLaunchKernelGGL((flat<RB, TWO>), dim3(nch), dim3(256), 0, 0, state, scal, scal_out, obs); \
         }, reps))
#define WS(RB, K, TWO)                                                                                         \
  printf("\"ws%s_%d_k%d\": %.3f, ", TWO ? "2" : "", RB, K, timeit([&] {                                       \
           hipLaunchKernelGGL((ws<RB, K, TWO>), dim3((nch + K - 1) / K), dim3(512), 0, 0, state, scal, scal_out, \
                              obs, nch);                                                                       \
         }, reps))
  FLAT(0, false);
  FLAT(176, false);
  FLAT(320, false);
  FLAT(176, true);
  FLAT(320, true);
  WS(0, 2, false);
  WS(176, 2, false);
  WS(320, 2, false);
  WS(176, 2, true);
  WS(320, 2, true);
  WS(176, 4, true);
  WS(320, 4, true);
  WS(320, 8, true);
  printf("\"end\": 0}}\n");
  return 0;
}
