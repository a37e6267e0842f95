// Diagnostic: coop_gen_map (pe_coop.hpp, one wave per env) vs gen_map
// (pe_device.hpp, one lane per env) on the same Philox streams; prints the first
// differing env/row and which codes differ.  64x64 (100 plants, 120 obstacles)
// and 20x20 geometries.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o build/coop_check tools/diag/coop_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../rl-env_amd/csrc/pe_coop.hpp"
using namespace pe;

constexpr int kEnvs = 256;

template <int MAXW>
__global__ void k_coop(Geo g, Rules rl, const Tables* tab, uint64_t* rows, int* scal) {
  extern __shared__ uint64_t scr[];
  const int lane = threadIdx.x & 63, e = blockIdx.x;
  Row4<MAXW> rw;
  const Scal s = coop_gen_map<MAXW>(g, rl, tab, rw, e, 0, lane, scr);
  if (lane < g.G)
    for (int w = 0; w < g.WPR; ++w) rows[(e * g.G + lane) * g.WPR + w] = rw.get(w);
  if (lane == 0) {
    scal[e * 4] = s.x;
    scal[e * 4 + 1] = s.y;
    scal[e * 4 + 2] = s.total;
    scal[e * 4 + 3] = (int)s.flags;
  }
}

__global__ void k_lane(Geo g, Rules rl, const Tables* tab, uint64_t* rows, int* scal, uint16_t* picks) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kEnvs) return;
  const Scal s = gen_map(g, rl, tab, rows + (size_t)e * g.G * g.WPR, picks + e * 256, e, 0);
  scal[e * 4] = s.x;
  scal[e * 4 + 1] = s.y;
  scal[e * 4 + 2] = s.total;
  scal[e * 4 + 3] = (int)s.flags;
}

// cluster triples: coop_clusters vs the sequential Stream (clusters_original's draws)
__global__ void k_cl_coop(Geo g, int clusters, int* out) {
  extern __shared__ uint64_t scr[];
  const int lane = threadIdx.x & 63, e = blockIdx.x;
  for (int k = lane; k < g.G * g.WPR; k += 64) scr[k] = 0;
  WaveStream rng;
  rng.init(77, e, 0, lane);
  coop_clusters(g, clusters, rng, scr, lane, out + e * 3 * clusters);
}
__global__ void k_cl_seq(Geo g, int clusters, int* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kEnvs) return;
  Stream rng;
  rng.init(77, e, 0);
  for (int q = 0; q < clusters; ++q) {
    out[(e * clusters + q) * 3] = 2 + (int)rng.below((uint32_t)(g.G - 4));
    out[(e * clusters + q) * 3 + 1] = 2 + (int)rng.below((uint32_t)(g.G - 4));
    out[(e * clusters + q) * 3 + 2] = 2 + (int)rng.below(2u);
  }
}
void check_clusters(int G, int clusters, int R) {
  Geo g;
  memset(&g, 0, sizeof(g));
  g.G = G; g.R = R; g.GG = G * G; g.WPR = (2 * (G + 2 * R) + 63) / 64;
  int *a, *b;
  const size_t n = (size_t)kEnvs * clusters * 3;
  hipMalloc(&a, n * 4 + 4096); hipMalloc(&b, n * 4);
  hipMemset(a, 0xff, n * 4 + 4096);
  hipLaunchKernelGGL(k_cl_coop, dim3(kEnvs), dim3(64), (size_t)G * g.WPR * 8, 0, g, clusters, a);
  hipLaunchKernelGGL(k_cl_seq, dim3(kEnvs / 64), dim3(64), 0, 0, g, clusters, b);
  hipDeviceSynchronize();
  std::vector<int> ha(n + 1024), hb(n);
  hipMemcpy(ha.data(), a, n * 4 + 4096, hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int e = 0; e < kEnvs && bad < 3; ++e)
    for (int q = 0; q < clusters; ++q) {
      const int* x = &ha[(e * clusters + q) * 3];
      const int* y = &hb[(e * clusters + q) * 3];
      if (x[0] != y[0] || x[1] != y[1] || x[2] != y[2]) {
        printf("clusters G=%d env %d q=%d: coop (%d,%d,%d) seq (%d,%d,%d)\n", G, e, q, x[0], x[1], x[2], y[0], y[1], y[2]);
        ++bad;
        break;
      }
    }
  printf("clusters G=%d n=%d: %s\n", G, clusters, bad ? "MISMATCH" : "ok");
  if (bad) {
    printf("env0 coop:");
    for (int q = 0; q < clusters; ++q) printf(" (%d,%d,%d)", ha[q * 3], ha[q * 3 + 1], ha[q * 3 + 2]);
    printf("\ndbg:");
    for (int k = 0; k < 0; ++k) printf(" %d", ha[3 * clusters + k]);
    printf("\nenv0 seq: ");
    for (int q = 0; q < clusters; ++q) printf(" (%d,%d,%d)", hb[q * 3], hb[q * 3 + 1], hb[q * 3 + 2]);
    printf("\n");
  }
}

template <int MAXW>
void check(int G, int P, int O, int R) {
  Geo g;
  memset(&g, 0, sizeof(g));
  g.G = G; g.R = R; g.GG = G * G; g.WPR = (2 * (G + 2 * R) + 63) / 64;
  Rules rl;
  memset(&rl, 0, sizeof(rl));
  rl.p_thirsty = 0.7; rl.P = P; rl.O = O; rl.seed = 77;
  Tables tab;
  memset(&tab, 0, sizeof(tab));
  for (int p = 0; p < G + 2 * R; ++p) {
    int w = (2 * p) / 64, b = (2 * p) % 64;
    if (p < R || p >= G + R) tab.grid_pad[w] |= 1ull << b; else tab.grid_real[w] |= 1ull << b;
  }
  Tables* dtab; uint64_t *r1, *r2; int *s1, *s2; uint16_t* pk;
  const size_t nrow = (size_t)kEnvs * G * g.WPR;
  hipMalloc(&dtab, sizeof(tab)); hipMalloc(&r1, nrow * 8); hipMalloc(&r2, nrow * 8);
  hipMalloc(&s1, kEnvs * 16); hipMalloc(&s2, kEnvs * 16); hipMalloc(&pk, kEnvs * 512);
  hipMemcpy(dtab, &tab, sizeof(tab), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_coop<MAXW>, dim3(kEnvs), dim3(64), (size_t)G * g.WPR * 8, 0, g, rl, dtab, r1, s1);
  hipLaunchKernelGGL(k_lane, dim3(kEnvs / 64), dim3(64), 0, 0, g, rl, dtab, r2, s2, pk);
  hipDeviceSynchronize();
  std::vector<uint64_t> a(nrow), b(nrow);
  std::vector<int> sa(kEnvs * 4), sb(kEnvs * 4);
  hipMemcpy(a.data(), r1, nrow * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), r2, nrow * 8, hipMemcpyDeviceToHost);
  hipMemcpy(sa.data(), s1, kEnvs * 16, hipMemcpyDeviceToHost);
  hipMemcpy(sb.data(), s2, kEnvs * 16, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int e = 0; e < kEnvs && bad < 5; ++e) {
    bool diff = memcmp(&sa[e * 4], &sb[e * 4], 16) != 0;
    int cnt[4][4] = {};
    for (int r = 0; r < G; ++r)
      for (int c = 0; c < G; ++c) {
        const int bit = 2 * (c + R);
        const size_t k = ((size_t)e * G + r) * g.WPR + bit / 64;
        const int ca = (a[k] >> (bit % 64)) & 3, cb = (b[k] >> (bit % 64)) & 3;
        if (ca != cb) { cnt[cb][ca]++; diff = true; }
      }
    if (diff) {
      ++bad;
      printf("G=%d env %d: coop (x,y,total,flags)=(%d,%d,%d,%d) lane=(%d,%d,%d,%d) code lane->coop diffs:", G, e,
             sa[e * 4], sa[e * 4 + 1], sa[e * 4 + 2], sa[e * 4 + 3], sb[e * 4], sb[e * 4 + 1], sb[e * 4 + 2], sb[e * 4 + 3]);
      for (int x = 0; x < 4; ++x) for (int y = 0; y < 4; ++y) if (cnt[x][y]) printf(" %d->%d:%d", x, y, cnt[x][y]);
      printf("\n");
    }
  }
  printf("G=%d P=%d O=%d R=%d: %d differing envs (of %d, first 5 listed)\n", G, P, O, R, bad, kEnvs);
}

int main() {
  check_clusters(20, 4, 6);
  check_clusters(64, 40, 6);
  check_clusters(64, 20, 6);
  check<1>(20, 10, 12, 6);
  check<4>(64, 100, 120, 6);
  check<4>(32, 20, 30, 9);
  check<4>(64, 10, 12, 6);
  check<4>(64, 100, 12, 6);
  check<4>(64, 10, 120, 6);
  return 0;
}
