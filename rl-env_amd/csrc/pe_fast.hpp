// pe_fast.hpp -- the specialized fused step kernel (compile-time C, R).
//
// Latency structure (one wave per SIMD at the headline batch, so every dependent
// HBM round trip is exposed): each lane issues its env's loads in TWO rounds.
//   round 1: packed scalars, action, episode return           (env index only)
//   round 2: the 2R+3 grid rows and 7 visit rows around the rover, the exact visit
//            count and explored words of the move target      (position + action)
// Everything after that -- collision test, watering, visit/explored update,
// reward, LIDAR ray-march and the 5x5 slice for the post-move position -- runs
// out of registers; state updates are plain stores.  The obs row is assembled in
// LDS and streamed as one contiguous tile per workgroup.
#pragma once
#include "pe_device.hpp"

namespace pe {

// Branch-free 3-way select by d in {-1,0,1}.  Written with masks on purpose: a
// ternary between two array elements is folded by InstCombine into a load through
// a selected address, which defeats register promotion of the window (scratch).
template <class T>
__device__ __forceinline__ T sel3(int d, T m1, T z, T p1) {
  const T am = (T)0 - (T)(d < 0), ap = (T)0 - (T)(d > 0), az = (T)0 - (T)(d == 0);
  return (m1 & am) | (z & az) | (p1 & ap);
}

template <int R, bool ONEWORD>
struct Window {
  static_assert(ONEWORD || R <= 14, "funnel-shifted window row must hold 2R+5 cells");
  static constexpr int NR = 2 * R + 3;  // grid rows x-R-1 .. x+R+1
  uint64_t rows[NR];                    // padded 2-bit codes, column base yb
  uint64_t clo, chi;                    // raw words of the centre row (watering)
  uint32_t vlo[7], vhi[7];              // raw visit words, rows x-3 .. x+3
  int yb, ybv;                          // grid / visit column bases

  __device__ __forceinline__ void load(const State& st, const Geo& g, int64_t e, uint32_t ep, int x, int y) {
    const uint64_t* gb = st.grid + e * g.gstride;
    yb = ONEWORD ? 0 : (y > 0 ? y - 1 : 0);
    const int w0 = (2 * yb) >> 6, o = (2 * yb) & 63;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int xr = x - R - 1 + k;
      uint64_t v = kEven64;  // off-map row: obstacles
      if (xr >= 0 && xr < g.G) {
        if constexpr (ONEWORD) {
          v = gb[xr];
          if (k == R + 1) clo = v;
        } else {
          const uint64_t* p = gb + (int64_t)xr * g.WPR + w0;
          uint64_t lo = p[0];
          uint64_t hi = (w0 + 1 < g.WPR) ? p[1] : 0ull;
          if (k == R + 1) {
            clo = lo;
            chi = hi;
          }
          v = o ? ((lo >> o) | (hi << (64 - o))) : lo;
        }
      }
      rows[k] = v;
    }
    ybv = y > 0 ? y - 1 : 0;
    const int vw = (4 * ybv) >> 5;
    const uint32_t* vb = vis_env(st, g, e, ep) + vw;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int xr = x - 3 + k;
      uint32_t lo = 0xAAAAAAAAu, hi = 0xAAAAAAAAu;  // off-map row: visit 10 (reads 1.0)
      if (xr >= 0 && xr < g.G) {
        lo = vb[(int64_t)xr * g.NW];
        hi = vb[(int64_t)xr * g.NW + 1];
      }
      vlo[k] = lo;
      vhi[k] = hi;
    }
  }

  // grid row (window-relative index k) funnel-shifted to padded column yb
  __device__ __forceinline__ void refresh_centre() {
    if constexpr (ONEWORD) {
      rows[R + 1] = clo;
    } else {
      const int o = (2 * yb) & 63;
      rows[R + 1] = o ? ((clo >> o) | (chi << (64 - o))) : clo;
    }
  }

  // 2-bit code of real cell (row x + dr, column c), dr in {-1,0,1}
  __device__ __forceinline__ int code(int dr, int c) const {
    const uint64_t r = sel3<uint64_t>(dr, rows[R], rows[R + 1], rows[R + 2]);
    return (int)((r >> (2 * (c + R - yb))) & 3u);
  }

  __device__ __forceinline__ uint32_t vis32(int k) const {
    const int o = (4 * ybv) & 31;
    return o ? ((vlo[k] >> o) | (vhi[k] << (32 - o))) : vlo[k];
  }
};

template <int C, int R, bool ONEWORD>
__device__ __forceinline__ void obs_from_window(const Window<R, ONEWORD>& w, int G, int dxv, int x, int y,
                                                float* row, const float* tpos, const float* tvis) {
  constexpr int W = 2 * R + 1;
  uint64_t win[W];
  const int sh = 2 * (y - w.yb);
#pragma unroll
  for (int j = 0; j < W; ++j) {
    win[j] = sel3<uint64_t>(dxv, w.rows[j], w.rows[j + 1], w.rows[j + 2]) >> sh;
  }
  using T = LidarTab<C, R>;
#pragma unroll
  for (int i = 0; i < C; ++i) {
    float dist = 1.0f;  // float(R/R): nothing hit, plantos_env.py:262
    int ent = EMPTY;
#pragma unroll
    for (int r = R; r >= 1; --r) {
      const int dx = T::dx[i][r - 1], dy = T::dy[i][r - 1];
      const int cd = (int)((win[dx + R] >> (2 * (dy + R))) & 3u);
      if (cd != EMPTY) {
        dist = (float)((double)r / (double)R);  // folded to float(r/R), plantos_env.py:288
        ent = cd;
      }
    }
    row[5 * i] = dist;
    row[5 * i + 1] = ent == 0 ? 1.0f : 0.0f;
    row[5 * i + 2] = ent == 1 ? 1.0f : 0.0f;
    row[5 * i + 3] = ent == 2 ? 1.0f : 0.0f;
    row[5 * i + 4] = ent == 3 ? 1.0f : 0.0f;
  }
  row[5 * C] = tpos[x];
  row[5 * C + 1] = tpos[y];
  const int vs = 4 * (y - w.ybv);
#pragma unroll
  for (int lx = 0; lx < 5; ++lx) {
    // visit row x'-2+lx is row lx+1+dxv of the x-3 .. x+3 block
    const uint32_t v = sel3<uint32_t>(dxv, w.vis32(lx), w.vis32(lx + 1), w.vis32(lx + 2)) >> vs;
#pragma unroll
    for (int ly = 0; ly < 5; ++ly) row[5 * C + 2 + 5 * lx + ly] = tvis[(v >> (4 * ly)) & 15u];
  }
}

}  // namespace pe
