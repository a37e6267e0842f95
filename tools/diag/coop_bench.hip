// Diagnostic: latency of the wave-cooperative reset pieces (pe_coop.hpp) for ONE
// env on one wave (256 workgroups of one wave, each resetting K envs in a row).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/coop_bench tools/diag/coop_bench.hip
#include <hip/hip_runtime.h>
#define PE_COOP_TIMING 1
#include <cstdio>
#include <cstring>
#include "../../rl-env_amd/csrc/pe_coop.hpp"
using namespace pe;

constexpr int K = 16;

template <int MODE>
__global__ __launch_bounds__(64) void k_coop(Geo g, Rules rl, const Tables* tab, uint32_t* out) {
  __shared__ Tables lt;
  __shared__ float row[400];
  __shared__ uint64_t scr[64 * 4];
  __shared__ signed char ldx[96], ldy[96];
  if (threadIdx.x == 0) lt = *tab;
  for (int k = threadIdx.x; k < 96; k += 64) {
    ldx[k] = (signed char)((k % 6) - 3);
    ldy[k] = (signed char)((k % 5) - 2);
  }
  __syncthreads();
  const int lane = threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < K; ++i) {
    const uint32_t env = blockIdx.x * K + i;
    if (MODE == 0) {  // coop_gen_map
      Row4<1> rw;
      Scal s = coop_gen_map<1>(g, rl, &lt, rw, env, 0, lane, scr);
      acc += s.x * 31 + s.y + (uint32_t)rw.w0;
    } else if (MODE == 1) {  // the rng draws alone (uniform)
      WaveStream r;
      r.init(rl.seed, env, 0, lane);
      for (int q = 0; q < 60; ++q) acc += r.next(lane);
    } else if (MODE == 2) {  // 3 wave scans + 1 wave sum
      int v = (int)(lane + env);
      for (int q = 0; q < 3; ++q) v = wave_incl_scan(v, lane);
      acc += wave_sum(v);
    } else if (MODE == 4) {  // the bench's own overhead (empty env loop)
      acc += env * 3u;
    } else if (MODE == 5) {  // 60 draws with the wave's cycle counter read around them
      WaveStream r;
      const uint64_t t0 = __builtin_readcyclecounter();
      r.init(rl.seed, env, 0, lane);
      for (int q = 0; q < 60; ++q) acc += r.next(lane);
      acc += (uint32_t)(__builtin_readcyclecounter() - t0) * 0u;
      if (lane == 0 && i == K - 1) out[256 * 64 + blockIdx.x] = (uint32_t)(__builtin_readcyclecounter() - t0);
    } else if (MODE == 3) {  // gen + fresh obs
      Row4<1> rw;
      Scal s = coop_gen_map<1>(g, rl, &lt, rw, env, 0, lane, scr);
      coop_fresh_obs(g, rw, s, row, lt.dist, lt.pos, lt.vis, ldx, ldy, lane);
      acc += __float_as_uint(row[lane]);
    }
  }
  out[blockIdx.x * 64 + lane] = acc;
}

int main() {
  Geo g;
  memset(&g, 0, sizeof(g));
  g.G = 20; g.R = 6; g.C = 16; g.GG = 400; g.WPR = 1; g.D = 107; g.NW = 4;
  Rules rl;
  memset(&rl, 0, sizeof(rl));
  rl.p_thirsty = 0.7; rl.P = 10; rl.O = 12; rl.seed = 0;
  Tables tab;
  memset(&tab, 0, sizeof(tab));
  for (int p = 0; p < 32; ++p) {
    if (p < 6 || p >= 26) tab.grid_pad[0] |= 1ull << (2 * p); else tab.grid_real[0] |= 1ull << (2 * p);
  }
  for (int r = 0; r <= 6; ++r) tab.dist[r] = (float)r / 6.f;
  Tables* dtab; uint32_t* dout;
  hipMalloc(&dtab, sizeof(tab)); hipMalloc(&dout, (256 * 64 + 256) * 4);
  hipMemcpy(dtab, &tab, sizeof(tab), hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  printf("{");
  auto run = [&](auto kern, const char* name) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(64), 0, 0, g, rl, dtab, dout);
    hipEventRecord(a);
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(64), 0, 0, g, rl, dtab, dout);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("\"%s_us_per_env\": %.2f, ", name, ms * 1000 / 5 / K);
  };
  run(k_coop<0>, "coop_gen_map");
  {
    unsigned long long t[8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_coop_t), sizeof(t));
    const char* nm[6] = {"init", "clusters", "count_scan", "sample", "thirsty", "rover"};
    for (int k = 0; k < 6; ++k) printf("\"cyc_%s\": %.0f, ", nm[k], (double)(t[k + 1] - t[k]) / (7.0 * K));
  }
  run(k_coop<1>, "rng_60_draws");
  run(k_coop<2>, "scans");
  run(k_coop<3>, "gen_plus_obs");
  run(k_coop<4>, "empty");
  run(k_coop<5>, "rng_60_draws_timed");
  uint32_t cyc[256];
  hipMemcpy(cyc, dout + 256 * 64, sizeof(cyc), hipMemcpyDeviceToHost);
  printf("\"rng_60_draws_cycles_block0\": %u, ", cyc[0]);
  printf("\"K\": %d}\n", K);
  return 0;
}
