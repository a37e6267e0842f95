// Diagnostic: is the block -> XCD mapping of a repeated launch stable?
// Launches a 1024-block grid (the headline step geometry: 256 threads, ~38 KB
// LDS) back to back and records each block's XCC_ID per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(256) void k(unsigned* out, int launch) {
  extern __shared__ float lds[];
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  lds[threadIdx.x] = (float)x;
  __syncthreads();
  if (threadIdx.x == 0) out[launch * 1024 + blockIdx.x] = (unsigned)lds[5] & 7u;
}
int main() {
  const int L = 20;
  unsigned* d;
  hipMalloc(&d, L * 1024 * 4);
  for (int l = 0; l < L; ++l) hipLaunchKernelGGL(k, dim3(1024), dim3(256), 38 * 1024, 0, d, l);
  hipDeviceSynchronize();
  std::vector<unsigned> h(L * 1024);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  int same_as_prev = 0, rr = 0;
  for (int l = 0; l < L; ++l) {
    int off = (h[l * 1024] + 8 - 0) % 8, ok = 1;
    for (int b = 0; b < 1024; ++b) ok &= (h[l * 1024 + b] == (unsigned)((b + off) % 8));
    rr += ok;
    if (l) {
      int s = 1;
      for (int b = 0; b < 1024; ++b) s &= h[l * 1024 + b] == h[(l - 1) * 1024 + b];
      same_as_prev += s;
    }
    printf("launch %d: block0 xcc %u, round-robin %s\n", l, h[l * 1024], ok ? "yes" : "no");
  }
  printf("{\"launches\": %d, \"round_robin\": %d, \"identical_to_previous\": %d}\n", L, rr, same_as_prev);
  return 0;
}
