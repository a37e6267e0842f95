// pe_quad.hpp -- the quadrant-split fused step kernel (compile-time C, R).
//
// One workgroup = NW waves (4 or 8) = 64 envs; lane l of every wave works on env
// e0+l, and wave w owns LIDAR rays [w*C/NW, (w+1)*C/NW) -- one compass sector --
// so the per-wave ray code is fully unrolled with compile-time offsets and the
// wave index is the only branch (wave-uniform: no divergence).  At NW=8 this is
// 8 waves per SIMD at the headline batch instead of 1 (one lane per env), so the
// load latency of one workgroup hides behind the work of the others.
//
//   round 1  every wave: packed scalars + action of its 64 envs (same addresses
//            in all 4 waves: one fetch, L1 hits after)
//   round 2  the 2R+3 grid rows and 7 visit rows around the rover are split over
//            the waves (row k loaded by wave k%NW) and parked in LDS, [row][env];
//            the commit wave (NW-1) also fetches what the state commit needs (raw
//            target visit word, u16 overflow slot, explored words in bitmap mode,
//            raw centre grid word for watering)
//   barrier
//   every wave re-derives the transition from LDS (cheap, identical), wave NW-1
//   commits the state; each wave ray-marches its sector over the post-move
//   window read from LDS at a per-lane row offset, and writes its slice of the
//   obs row into the LDS obs tile
//   barrier (+ auto-reset slow path in the commit wave if any env is done)
//   the 64*NW threads stream the [64 x D] obs tile to HBM with 16-B stores.
#pragma once
#include <type_traits>

#include "pe_coop.hpp"
#include "pe_device.hpp"

namespace pe {

constexpr int kQuadEnvs = 64;  // envs per workgroup (one per lane of every wave)

// compile-time extent of the dx offsets of rays [i0, i1)
template <int C, int R>
constexpr int ray_dx_min(int i0, int i1) {
  int m = 0;
  for (int i = i0; i < i1; ++i)
    for (int r = 0; r < R; ++r) m = LidarTab<C, R>::dx[i][r] < m ? LidarTab<C, R>::dx[i][r] : m;
  return m;
}
template <int C, int R>
constexpr int ray_dx_max(int i0, int i1) {
  int m = 0;
  for (int i = i0; i < i1; ++i)
    for (int r = 0; r < R; ++r) m = LidarTab<C, R>::dx[i][r] > m ? LidarTab<C, R>::dx[i][r] : m;
  return m;
}

// Grid row xr as a 64-bit window of padded 2-bit codes starting at padded column
// yb (w0 = word, o = bit offset of yb); off-map rows read as obstacles.
template <bool ONEWORD>
__device__ __forceinline__ uint64_t quad_row(const uint64_t* gb, const Geo& g, int xr, int w0, int o) {
  if (xr < 0 || xr >= g.G) return kEven64;
  if constexpr (ONEWORD) {
    return gb[xr];
  } else {
    const uint64_t* p = gb + (int64_t)xr * g.WPR + w0;
    const uint64_t lo = p[0];
    const uint64_t hi = (w0 + 1 < g.WPR) ? p[1] : 0ull;
    return o ? ((lo >> o) | (hi << (64 - o))) : lo;
  }
}

// LDS table words the sector rays read (in the tables' dist[] region, which holds
// dist[0..R]): dist[R+1] = 1.0 (nothing hit), and at kOneHotF the one-hot rows of
// the 4 entity codes as float4 (16-B aligned).
constexpr int kOneHotF = 48;

// Rays [W*C/NW, (W+1)*C/NW) of one env (the sector of wave W): first hit over the
// post-move window rows read from LDS (row k of the [row][env] block = grid row
// x-R-1+k), written as obs[5i .. 5i+4] (plantos_env.py:260-292).  Per ray the R
// probe codes are packed 2 bits each (probe r at bits 2(r-1)), so the first hit is
// one find-first-set over their nonzero bits (a sentinel at bit 2R: nothing hit,
// range R, entity EMPTY), and its distance and one-hot come from LDS tables:
// ~3 VALU per probe instead of a compare-and-select chain per probe and per float.
// OT: float (an f32 tile row) or uint8_t (a byte-coded tile row, pe_coop.hpp ObsW).
template <int C, int R, int NW, int W, typename OT>
__device__ __forceinline__ void quad_rays(const uint64_t* lrow, int lane, int kc, int sh, bool watered, OT* row,
                                          const float* tdist) {
  constexpr int I0 = W * C / NW, I1 = (W + 1) * C / NW;
  constexpr int LO = ray_dx_min<C, R>(I0, I1), HI = ray_dx_max<C, R>(I0, I1);
  static_assert(2 * R + 1 <= 31, "packed probe codes + sentinel fit 32 bits");
  // the window cells yp-R .. yp+R of a row: 2(2R+1) bits (32-bit words up to R = 7)
  using WT = typename std::conditional<(4 * R + 2 <= 32), uint32_t, uint64_t>::type;
  WT win[HI - LO + 1];
#pragma unroll
  for (int j = 0; j <= HI - LO; ++j) win[j] = (WT)(lrow[(kc + LO + j) * kQuadEnvs + lane] >> sh);
  if constexpr (LO <= 0 && HI >= 0) {
    // watering turned the rover's cell thirsty -> hydrated (code 3 -> 2)
    if (watered) win[-LO] &= ~((WT)1 << (2 * R));
  }
  constexpr uint32_t kNZ = 0x55555555u & ((1u << (2 * R)) - 1u);
  const float4* tone = reinterpret_cast<const float4*>(tdist + kOneHotF);
  using T = LidarTab<C, R>;
  // f32 rows: every table read of the sector first, then the row writes -- in program
  // order a table read after a row write cannot be hoisted above it (the compiler
  // cannot tell the tile from the tables), which made each ray wait out two LDS
  // round trips (read -> lgkmcnt(0) -> write) in turn
  constexpr bool kF32 = std::is_same<OT, float>::value;
  float dv[kF32 ? I1 - I0 : 1];
  float4 ov[kF32 ? I1 - I0 : 1];
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    uint32_t pk = 0u;
#pragma unroll
    for (int r = 1; r <= R; ++r) {
      const int dx = T::dx[i][r - 1], dy = T::dy[i][r - 1];
      pk |= (uint32_t)((win[dx - LO] >> (2 * (dy + R))) & 3u) << (2 * (r - 1));
    }
    const uint32_t nz = ((pk | (pk >> 1)) & kNZ) | (1u << (2 * R));
    const int f = __builtin_ctz(nz);         // 2(r-1) of the first hit, 2R if none
    const int ent = (int)((pk >> f) & 3u);   // its code (EMPTY if none)
    if constexpr (kF32) {
      dv[i - I0] = tdist[(f >> 1) + 1];      // float(r / R), plantos_env.py:288 (R/R if none)
      ov[i - I0] = tone[ent];
    } else {
      row[5 * i] = (uint8_t)((f >> 1) + 1);  // code r = dist[r] (R+1: 1.0, nothing hit)
      const uint32_t oh = (uint32_t)(R + 1) << (8 * ent);  // one-hot as codes {0, R+1}
      row[5 * i + 1] = (uint8_t)oh;
      row[5 * i + 2] = (uint8_t)(oh >> 8);
      row[5 * i + 3] = (uint8_t)(oh >> 16);
      row[5 * i + 4] = (uint8_t)(oh >> 24);
    }
  }
  if constexpr (kF32) {
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      row[5 * i] = dv[i - I0];
      row[5 * i + 1] = ov[i - I0].x;
      row[5 * i + 2] = ov[i - I0].y;
      row[5 * i + 3] = ov[i - I0].z;
      row[5 * i + 4] = ov[i - I0].w;
    }
  }
}

// Runtime-(C, R) sector rays: the ray march of pe_step_quad<0, 0, ...> (the table-
// driven sector kernel of geometries with no compile-time specialization, C <= 64,
// 2 <= R <= 14).  Wave wv's rays [wv*C/NW, (wv+1)*C/NW); the probes are wave-uniform
// u32 entries of an LDS table (pe_create, round 5): the probe's LDS byte offset from the
// lane's rover row (dx * 64 envs * 8 B, int16) | its bit shift in the funnel-shifted row
// word (2(dy+R)) << 16 -- 4 probes per 16-B LDS read at a wave-uniform address, unrolled
// by 8; a probe is one address add, one LDS read, one shift add, the 64-bit shift and the
// 2-bit pack (plantos_env.py:260-292; first hit by one find-first-set).  The watered
// rover cell (code 3 -> 2) is fixed per ray, not per probe: it is the ray's first probe
// (r = 1 at (0, 0), the only radius where int(r cos) = int(r sin) = 0), a hit either way,
// so only that ray's entity changes (round 4's per-probe mask: ~10 VALU per probe).
template <typename OT>
__device__ __forceinline__ void quad_rays_rt(const uint64_t* lrow, const uint32_t* ltab, int i0, int i1, int R,
                                             int lane, int kc, int sh, bool watered, OT* row, const float* tdist) {
  const int RP = (R + 7) & ~7;
  const uint32_t kNZ = 0x55555555u & ((1u << (2 * R)) - 1u);  // R <= 14
  const float4* tone = reinterpret_cast<const float4*>(tdist + kOneHotF);
  const char* base = reinterpret_cast<const char*>(lrow + kc * kQuadEnvs + lane);  // the lane's rover row
  const uint32_t origin = (uint32_t)(2 * R) << 16;  // the entry of probe (0, 0)
  for (int i = i0; i < i1; ++i) {
    const uint4* o4 = reinterpret_cast<const uint4*>(ltab + i * RP);  // (16-B aligned: RP is a multiple of 8)
    uint32_t pk = 0u;
    auto probe = [&](uint32_t v, int r) {
      const uint64_t w = *reinterpret_cast<const uint64_t*>(base + (int)(int16_t)(v & 0xFFFFu));
      pk |= (uint32_t)((w >> (sh + (int)(v >> 16))) & 3u) << (2 * r);  // (r < R <= 14)
    };
    uint32_t first = 0u;
    int r0 = 0;
    for (; r0 + 8 <= R; r0 += 8) {  // whole chunks: 8 probes unrolled, their LDS reads in flight together
      const uint4 qa = o4[r0 >> 2], qb = o4[(r0 >> 2) + 1];
      const uint32_t qw[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
      if (r0 == 0) first = qa.x;
#pragma unroll
      for (int j = 0; j < 8; ++j) probe(qw[j], r0 + j);
    }
    if (r0 < R) {  // the last R % 8 probes (padded probes not marched: profiles/r4m)
      const uint4 qa = o4[r0 >> 2], qb = o4[(r0 >> 2) + 1];
      if (r0 == 0) first = qa.x;
      for (int j = 0; j < R - r0; ++j) {
        const uint32_t qj = j < 4 ? (j < 2 ? (j == 0 ? qa.x : qa.y) : (j == 2 ? qa.z : qa.w))
                                  : (j < 6 ? (j == 4 ? qb.x : qb.y) : (j == 6 ? qb.z : qb.w));
        probe(qj, r0 + j);
      }
    }
    const uint32_t nz = ((pk | (pk >> 1)) & kNZ) | (1u << (2 * R));
    const int f = __builtin_ctz(nz);        // 2r of the first hit, 2R if none
    int ent = (int)((pk >> f) & 3u);        // its code (EMPTY if none)
    if (watered && f == 0 && first == origin) ent &= 2;  // the watered rover cell: THIRSTY -> HYD
    if constexpr (std::is_same<OT, float>::value) {
      const float dv = tdist[(f >> 1) + 1];
      const float4 ov = tone[ent];
      row[5 * i] = dv;
      row[5 * i + 1] = ov.x;
      row[5 * i + 2] = ov.y;
      row[5 * i + 3] = ov.z;
      row[5 * i + 4] = ov.w;
    } else {  // byte codes (pe_coop.hpp ObsW<uint8_t>), as quad_rays
      row[5 * i] = (uint8_t)((f >> 1) + 1);  // code r = dist[r] (R+1: 1.0, nothing hit)
      const uint32_t oh = (uint32_t)(R + 1) << (8 * ent);  // one-hot as codes {0, R+1}
      row[5 * i + 1] = (uint8_t)oh;
      row[5 * i + 2] = (uint8_t)(oh >> 8);
      row[5 * i + 3] = (uint8_t)(oh >> 16);
      row[5 * i + 4] = (uint8_t)(oh >> 24);
    }
  }
}

// Runtime-(C, R) sector rays from a register window (round 6): the wave's sector rows
// dx in [LO, LO + NROWS) -- at most kRtRegRows, at most 16 columns dy in [DLO, DLO + 15]
// -- each read once from LDS and shifted by the lane's column offset into one 32-bit
// word (window column dy - DLO at bits 2(dy - DLO)); a probe is then the word at a
// wave-uniform index (VGPR indexing: s_set_gpr_idx_on + v_mov), one v_bfe at a uniform
// bit offset and one v_lshl_or into the packed codes -- 3 VALU instead of ~5.5 (an
// address add, a shift-amount add, the LDS read, a 64-bit shift, the mask and the pack).
// The probe entries (row index | bit offset << 8) and the sector header {LO, DLO,
// NROWS, ok} come through the scalar cache (constant address space: s_load), so their
// decode is SALU.  pe_create builds both; a sector whose rows or columns do not fit
// (ok == 0, e.g. uneven sectors of some C not a multiple of 4) takes quad_rays_rt.
constexpr int kRtRegRows = 15;  // R + 1 rows of a quadrant at R <= 14
typedef const __attribute__((address_space(4))) uint32_t* rt_cptr;
template <typename OT>
__device__ __forceinline__ void quad_rays_rt_reg(const uint64_t* lrow, rt_cptr hdr, rt_cptr ent, int i0, int i1,
                                                 int R, int lane, int kc, int sh, bool watered, OT* row,
                                                 const float* tdist) {
  const int RP = (R + 7) & ~7;
  const int LO = (int)hdr[0], DLO = (int)hdr[1], NR = (int)hdr[2];
  const uint32_t kNZ = 0x55555555u & ((1u << (2 * R)) - 1u);  // R <= 14
  const float4* tone = reinterpret_cast<const float4*>(tdist + kOneHotF);
  const int shw = sh + 2 * (DLO + R);  // the lane's bit of window column DLO in its LDS row word (< 64)
  uint32_t w[kRtRegRows];
#pragma unroll
  for (int j = 0; j < kRtRegRows; ++j) {  // (rows past NR: the last row again, never probed)
    const int jj = j < NR ? j : NR - 1;
    w[j] = (uint32_t)(lrow[(kc + LO + jj) * kQuadEnvs + lane] >> shw);
  }
  const uint32_t origin = (uint32_t)(-LO) | ((uint32_t)(-2 * DLO) << 8);  // the entry of probe (0, 0)
  for (int i = i0; i < i1; ++i) {
    rt_cptr e = ent + i * RP;
    uint32_t pk = 0u;
    int r0 = 0;
    for (; r0 + 8 <= R; r0 += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t v = e[r0 + j];
        pk |= __builtin_amdgcn_ubfe(w[v & 31u], (v >> 8) & 31u, 2) << (2 * (r0 + j));
      }
    }
    for (; r0 < R; ++r0) {
      const uint32_t v = e[r0];
      pk |= __builtin_amdgcn_ubfe(w[v & 31u], (v >> 8) & 31u, 2) << (2 * r0);
    }
    const uint32_t nz = ((pk | (pk >> 1)) & kNZ) | (1u << (2 * R));
    const int f = __builtin_ctz(nz);        // 2r of the first hit, 2R if none
    int ent_code = (int)((pk >> f) & 3u);   // its code (EMPTY if none)
    if (watered && f == 0 && e[0] == origin) ent_code &= 2;  // the watered rover cell: THIRSTY -> HYD
    if constexpr (std::is_same<OT, float>::value) {
      const float dv = tdist[(f >> 1) + 1];
      const float4 ov = tone[ent_code];
      row[5 * i] = dv;
      row[5 * i + 1] = ov.x;
      row[5 * i + 2] = ov.y;
      row[5 * i + 3] = ov.z;
      row[5 * i + 4] = ov.w;
    } else {
      row[5 * i] = (uint8_t)((f >> 1) + 1);
      const uint32_t oh = (uint32_t)(R + 1) << (8 * ent_code);
      row[5 * i + 1] = (uint8_t)oh;
      row[5 * i + 2] = (uint8_t)(oh >> 8);
      row[5 * i + 3] = (uint8_t)(oh >> 16);
      row[5 * i + 4] = (uint8_t)(oh >> 24);
    }
  }
}

// Wave-uniform dispatch of the sector code (wv comes from readfirstlane).
template <int C, int R, int NW, int W = 0, typename T>
__device__ __forceinline__ void sector_rays(int wv, const uint64_t* lrow, int lane, int kc, int sh, bool watered,
                                            T* row, const float* tdist) {
  if constexpr (W < NW) {
    if (wv == W)
      quad_rays<C, R, NW, W, T>(lrow, lane, kc, sh, watered, row, tdist);
    else
      sector_rays<C, R, NW, W + 1, T>(wv, lrow, lane, kc, sh, watered, row, tdist);
  }
}

// One row lx of the 5x5 visit slice (plantos_env.py:298-313) from the LDS visit
// rows (row k = visit row x-3+k, 8 nibbles from padded column ybv).
template <typename T>
__device__ __forceinline__ void quad_slice_row(const uint32_t* lvis, int lane, int lx, int dxv, int vs, bool bump,
                                               uint32_t nib, int C, T* row, const float* tvis) {
  uint32_t v = lvis[(dxv + 1 + lx) * kQuadEnvs + lane] >> vs;
  if (lx == 2 && bump) v = (v & ~0xF00u) | (nib << 8);  // the move's own visit (:203)
  if constexpr (std::is_same<T, float>::value) {
    float t[5];  // table reads first, then the writes (see quad_rays)
#pragma unroll
    for (int ly = 0; ly < 5; ++ly) t[ly] = tvis[(v >> (4 * ly)) & 15u];
#pragma unroll
    for (int ly = 0; ly < 5; ++ly) row[5 * C + 2 + 5 * lx + ly] = t[ly];
  } else {
#pragma unroll
    for (int ly = 0; ly < 5; ++ly) row[5 * C + 2 + 5 * lx + ly] = (uint8_t)(kCodeVis + ((v >> (4 * ly)) & 15u));
  }
}

}  // namespace pe
