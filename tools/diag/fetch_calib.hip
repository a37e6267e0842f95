// FETCH_SIZE calibration on gfx950 for the access shapes of the step kernel
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact ×½ only for wide coalesced streaming
// reads; "calibrate on a known byte count in your own access pattern").  Each kernel
// reads a KNOWN number of bytes exactly once from a 1 GiB buffer (beyond the 256 MiB
// Infinity Cache) and writes one word per workgroup (a checksum, against dead-code
// elimination).  Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and compare
// FETCH_SIZE x 1024 with the bytes printed here.
//   stream16: lane i reads 16 B at i (coalesced, 1 KiB per wave-instruction)
//   stream4:  lane i reads 4 B at i (coalesced, 256 B per wave-instruction)
//   seg64:    4 lanes read one 64-B segment, segments at random 64-B-aligned places
//             (the sector kernel's round-1 loader shape: 4 threads x 16 B per env row)
//   gather16: every lane reads 16 B at a random 16-B-aligned place (window rows)
//   gather8:  every lane reads 8 B at a random 8-B-aligned place (multi-word rows)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__device__ __forceinline__ void sink(uint32_t v, uint32_t* out) {
  v = __reduce_xor_sync(0xFFFFFFFFFFFFFFFFull, v);
  if ((threadIdx.x & 63) == 0) atomicXor(out + blockIdx.x % 1024, v);
}

__global__ void stream16(const uint4* src, uint32_t* out) {
  const uint4 v = src[(size_t)blockIdx.x * blockDim.x + threadIdx.x];
  sink(v.x ^ v.y ^ v.z ^ v.w, out);
}
__global__ void stream4(const uint32_t* src, uint32_t* out) {
  sink(src[(size_t)blockIdx.x * blockDim.x + threadIdx.x], out);
}
__global__ void seg64(const uint4* src, const uint32_t* idx, uint32_t* out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 v = src[(size_t)idx[t >> 2] * 4 + (t & 3)];
  sink(v.x ^ v.y ^ v.z ^ v.w, out);
}
__global__ void gather16(const uint4* src, const uint32_t* idx, uint32_t* out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 v = src[idx[t]];
  sink(v.x ^ v.y ^ v.z ^ v.w, out);
}
__global__ void gather8(const uint2* src, const uint32_t* idx, uint32_t* out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint2 v = src[idx[t]];
  sink(v.x ^ v.y, out);
}

int main() {
  const size_t buf = 1ull << 30;  // 1 GiB
  const size_t n = 1u << 22;      // reads per kernel (4M lanes)
  void* src;
  uint32_t *out, *idx;
  CK(hipMalloc(&src, buf));
  CK(hipMemset(src, 0x5A, buf));
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMemset(out, 0, 4096 * 4));
  CK(hipMalloc(&idx, n * 4));
  std::vector<uint32_t> h(n);
  uint64_t x = 88172645463325252ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  // distinct random places: a stride walk over a prime-sized ring (no repeats)
  auto fill = [&](size_t units) {
    const uint64_t p = 1000003ull, off = rnd() % units;
    for (size_t i = 0; i < n; ++i) h[i] = (uint32_t)((off + i * p) % units);
  };
  const dim3 blk(256), grd((unsigned)(n / 256));
  hipLaunchKernelGGL(stream16, grd, blk, 0, 0, (const uint4*)src, out);
  hipLaunchKernelGGL(stream4, grd, blk, 0, 0, (const uint32_t*)src, out);
  fill(buf / 64);
  CK(hipMemcpy(idx, h.data(), (n / 4) * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(seg64, grd, blk, 0, 0, (const uint4*)src, idx, out);
  fill(buf / 16);
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(gather16, grd, blk, 0, 0, (const uint4*)src, idx, out);
  fill(buf / 8);
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(gather8, grd, blk, 0, 0, (const uint2*)src, idx, out);
  CK(hipDeviceSynchronize());
  std::printf("{\"reads\": %zu, \"bytes\": {\"stream16\": %zu, \"stream4\": %zu, \"seg64\": %zu, \"gather16\": %zu, "
              "\"gather8\": %zu}, \"idx_bytes\": {\"seg64\": %zu, \"gather16\": %zu, \"gather8\": %zu}}\n",
              n, n * 16, n * 4, n * 16, n * 16, n * 8, (n / 4) * 4, n * 4, n * 4);
  return 0;
}
