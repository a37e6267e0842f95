// Diagnostic micro-benchmark of the device map generator (pe_device.hpp gen_map):
// 65536 envs, one lane each, grid images in LDS; variants isolate the parts.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/genmap_bench tools/diag/genmap_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../../rl-env_amd/csrc/pe_device.hpp"
using namespace pe;

template <int MODE>
__global__ __launch_bounds__(64) void k_gen(Geo g, Rules rl, const Tables* tab, uint32_t* out) {
  __shared__ uint64_t img[64][40];
  __shared__ Tables lt;
  if (threadIdx.x == 0) lt = *tab;
  __syncthreads();
  const uint32_t e = blockIdx.x * 64 + threadIdx.x;
  uint64_t* sg = img[threadIdx.x];
  uint16_t* picks = reinterpret_cast<uint16_t*>(sg + 32);
  uint32_t acc = 0;
  if (MODE == 0) {  // full gen_map
    Scal s = gen_map(g, rl, &lt, sg, picks, e, 0);
    acc = s.x * 31 + s.y + s.total;
  } else if (MODE == 1) {  // rng only: same number of draws, no scans
    Stream r;
    r.init(rl.seed, e, 0);
    for (int i = 0; i < 60; ++i) acc += r.next();
  } else if (MODE == 2) {  // scans only: 11 nth_cell on an empty image
    for (int row = 0; row < g.G; ++row) sg[row] = lt.grid_pad[0];
    for (int i = 0; i < 11; ++i) acc += img_nth_cell(sg, g, &lt, (int)((e * 7 + i * 37) % 300), 0);
  }
  out[e] = acc;
}

int main() {
  Geo g;
  memset(&g, 0, sizeof(g));
  g.G = 20; g.R = 6; g.C = 16; g.GG = 400; g.WPR = 1;
  Rules rl;
  memset(&rl, 0, sizeof(rl));
  rl.p_thirsty = 0.7; rl.P = 10; rl.O = 12; rl.seed = 0;
  Tables tab;
  memset(&tab, 0, sizeof(tab));
  for (int p = 0; p < 32; ++p) {
    if (p < 6 || p >= 26) tab.grid_pad[0] |= 1ull << (2 * p); else tab.grid_real[0] |= 1ull << (2 * p);
  }
  Tables* dtab; uint32_t* dout;
  hipMalloc(&dtab, sizeof(tab)); hipMalloc(&dout, 65536 * 4);
  hipMemcpy(dtab, &tab, sizeof(tab), hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](auto kern, const char* name) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(1024), dim3(64), 0, 0, g, rl, dtab, dout);
    hipEventRecord(a);
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, dim3(1024), dim3(64), 0, 0, g, rl, dtab, dout);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("{\"variant\": \"%s\", \"us\": %.1f}\n", name, ms * 1000 / 5);
  };
  run(k_gen<0>, "gen_map");
  run(k_gen<1>, "rng_60_draws");
  run(k_gen<2>, "11_scans");
  return 0;
}
