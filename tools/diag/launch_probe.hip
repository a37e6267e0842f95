// Diagnostic: fixed per-launch cost of back-to-back dependent kernels (empty
// kernels), direct launches vs hipGraph replay, by grid size.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/launch_probe tools/diag/launch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void empty_k(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

float direct(int grid, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, 0, nullptr);
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, 0, nullptr);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

float graph(int grid, int per_graph, int replays) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < per_graph; ++i) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, s, nullptr);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int i = 0; i < 5; ++i) (void)hipGraphLaunch(ge, s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, s);
  for (int i = 0; i < replays; ++i) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / (replays * per_graph);
}

int main() {
  printf("{\"us_per_kernel\": {");
  const int grids[] = {1, 256, 1024, 4096};
  for (int gi = 0; gi < 4; ++gi) {
    const int gsz = grids[gi];
    printf("\"direct_grid%d\": %.3f, \"graph64_grid%d\": %.3f%s", gsz, direct(gsz, 2000), gsz, graph(gsz, 64, 40),
           gi < 3 ? ", " : "");
  }
  printf("}}\n");
  return 0;
}
