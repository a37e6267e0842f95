// plantos_batch.hip -- MI355X (gfx950) batched PlantOSEnv step/reset + C-ABI.
//
// One lane owns one env (no cross-env writes, so no atomics on state).  The fused
// step kernel does, per env: action decode, move/collide or water, visit/explored
// update, f64 reward (cast once), terminated/truncated, optional auto-reset, LIDAR
// ray-march, position, 5x5 visit slice; each lane assembles its obs row in LDS and
// the workgroup streams the contiguous [BLOCK x D] obs tile to HBM with 16-byte
// stores.  C-ABI: include/plantos_batch.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/plantos_batch.h"
#include "lidar_tables.inc"
#include "pe_device.hpp"
#include "pe_fast.hpp"
#include "pe_coop.hpp"
#include "pe_quad.hpp"

using namespace pe;

namespace {

constexpr int kBlock = 64;      // envs per workgroup (one wave)
constexpr int kTabFloats = (int)(sizeof(Tables) / sizeof(float));  // whole Tables struct in LDS
static_assert(sizeof(Tables) % 16 == 0, "LDS regions after the tables stay 16-B aligned");

struct StepArgs {
  State st;
  Geo g;
  Rules rl;
  int n;
  int autoreset;
  int act_bytes;
  int coop_max_done;  // step kernel: wave-cooperative resets up to this many done envs per block
  const void* actions;
  float* obs;
  uint8_t* obs_codes;   // byte-coded tile kernels: the obs as codes (pe_step_codes) instead of obs
  float* reward;
  uint8_t* term;
  uint8_t* trunc;
  float* tobs;
  double* ep_ret_out;
  int32_t* ep_len_out;
  int32_t* tinfo;       // terminal _get_info rows of done envs (may be NULL)
  Prefetch pf;          // prefetched resets (pe_coop.hpp); pf.scal == NULL: off
  int stagger;          // sector kernel: start delay per block quarter, units of 512 cycles
  const uint8_t* mask;  // reset kernel
};

// ------------------------------------------------------------------ obs builders
// _get_lidar_obs, plantos_env.py:251-315, into one LDS row.

// Generic: runtime (G, C, R), LIDAR offsets from the handle's table.
__device__ __forceinline__ void build_obs_generic(const StepArgs& a, int64_t e, uint32_t ep, int x, int y, float* row,
                                                  const float* tdist, const float* tpos, const float* tvis,
                                                  const signed char* ldx, const signed char* ldy) {
  const Geo& g = a.g;
  const int R = g.R, C = g.C;
  for (int i = 0; i < C; ++i) {
    int dist = R, ent = EMPTY;
    for (int r = 1; r <= R; ++r) {
      int cx = x + ldx[i * R + r - 1];
      int cy = y + ldy[i * R + r - 1];
      int code = (cx >= 0 && cx < g.G) ? grid_code(a.st, g, e, cx, cy + R) : OBST;  // :271-284
      if (code != EMPTY) {
        dist = r;
        ent = code;
        break;
      }
    }
    row[5 * i] = tdist[dist];
    row[5 * i + 1] = ent == 0 ? 1.0f : 0.0f;
    row[5 * i + 2] = ent == 1 ? 1.0f : 0.0f;
    row[5 * i + 3] = ent == 2 ? 1.0f : 0.0f;
    row[5 * i + 4] = ent == 3 ? 1.0f : 0.0f;
  }
  row[5 * C] = tpos[x];
  row[5 * C + 1] = tpos[y];
  for (int lx = 0; lx < 5; ++lx) {
    int xr = x + lx - 2;
    uint32_t win = (xr >= 0 && xr < g.G) ? vis_window(a.st, g, e, ep, xr, y) : 0xAAAAAu;
    for (int ly = 0; ly < 5; ++ly) row[5 * C + 2 + 5 * lx + ly] = tvis[(win >> (4 * ly)) & 15u];
  }
}

// obs of a freshly reset env (all visits 0 but the rover's 1) from its grid image
// sg, written to `out` (HBM).  Same values as build_obs_generic on that state.
__device__ inline void build_obs_fresh(const StepArgs& a, const uint64_t* sg, const Scal& s, float* out,
                                       const float* tdist, const float* tpos, const float* tvis,
                                       const signed char* ldx, const signed char* ldy) {
  const Geo& g = a.g;
  const int R = g.R, C = g.C, x = s.x, y = s.y;
  for (int i = 0; i < C; ++i) {
    int dist = R, ent = EMPTY;
    for (int r = 1; r <= R; ++r) {
      const int cx = x + ldx[i * R + r - 1];
      const int cy = y + ldy[i * R + r - 1];
      const int code = (cx >= 0 && cx < g.G) ? img_code(sg, g, cx, cy + R) : OBST;  // :271-284
      if (code != EMPTY) {
        dist = r;
        ent = code;
        break;
      }
    }
    out[5 * i] = tdist[dist];
    out[5 * i + 1] = ent == 0 ? 1.0f : 0.0f;
    out[5 * i + 2] = ent == 1 ? 1.0f : 0.0f;
    out[5 * i + 3] = ent == 2 ? 1.0f : 0.0f;
    out[5 * i + 4] = ent == 3 ? 1.0f : 0.0f;
  }
  out[5 * C] = tpos[x];
  out[5 * C + 1] = tpos[y];
  for (int lx = 0; lx < 5; ++lx)
    for (int ly = 0; ly < 5; ++ly) {
      const int gx = x + lx - 2, gy = y + ly - 2;
      const bool in = gx >= 0 && gx < g.G && gy >= 0 && gy < g.G;       // :307-311
      const bool rover = lx == 2 && ly == 2 && !(s.flags & F_NOROOM);
      out[5 * C + 2 + 5 * lx + ly] = !in ? tvis[10] : (rover ? tvis[1] : tvis[0]);
    }
}

// The same obs as byte codes (pe_coop.hpp ObsW<uint8_t>: dist r -> r, one-hot 0 / 1 ->
// 0 / R+1, vis v -> kCodeVis + v, pos x -> kCodePos + x).
__device__ inline void build_obs_fresh_codes(const StepArgs& a, const uint64_t* sg, const Scal& s, uint8_t* out,
                                             const signed char* ldx, const signed char* ldy) {
  const Geo& g = a.g;
  const int R = g.R, C = g.C, x = s.x, y = s.y;
  for (int i = 0; i < C; ++i) {
    int dist = R, ent = EMPTY;
    for (int r = 1; r <= R; ++r) {
      const int cx = x + ldx[i * R + r - 1];
      const int cy = y + ldy[i * R + r - 1];
      const int code = (cx >= 0 && cx < g.G) ? img_code(sg, g, cx, cy + R) : OBST;  // :271-284
      if (code != EMPTY) {
        dist = r;
        ent = code;
        break;
      }
    }
    out[5 * i] = (uint8_t)dist;
    for (int k = 0; k < 4; ++k) out[5 * i + 1 + k] = (uint8_t)(ent == k ? R + 1 : 0);
  }
  out[5 * C] = (uint8_t)(kCodePos + x);
  out[5 * C + 1] = (uint8_t)(kCodePos + y);
  for (int lx = 0; lx < 5; ++lx)
    for (int ly = 0; ly < 5; ++ly) {
      const int gx = x + lx - 2, gy = y + ly - 2;
      const bool in = gx >= 0 && gx < g.G && gy >= 0 && gy < g.G;       // :307-311
      const bool rover = lx == 2 && ly == 2 && !(s.flags & F_NOROOM);
      out[5 * C + 2 + 5 * lx + ly] = (uint8_t)(kCodeVis + (!in ? 10 : (rover ? 1 : 0)));
    }
}


__device__ __forceinline__ void load_tables(float* smem, const Tables* tab) {
  const float* src = reinterpret_cast<const float*>(tab);
  for (int k = threadIdx.x; k < kTabFloats; k += blockDim.x) smem[k] = src[k];
}

// The tables the step reads: dist[0..R], pos[0..G), vis[0..16) (hot path) and the
// pad masks (floats 344.., reset paths: read from LDS there, never from global
// memory under the obs stores' traffic).
__device__ __forceinline__ void load_tables_hot(float* smem, const Tables* tab, int G, int R) {
  const float* src = reinterpret_cast<const float*>(tab);
  const int n = (R + 1) + G + 16 + (kTabFloats - 344);
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const int f = k <= R ? k : (k < R + 1 + G ? 72 + (k - R - 1) : (k < R + 1 + G + 16 ? 328 + (k - R - 1 - G)
                                                                                      : 344 + (k - R - 1 - G - 16)));
    smem[f] = src[f];
  }
}

// The rest (pad masks, read by map generation / info): loaded on the rare reset path.
__device__ __forceinline__ void load_tables_cold(float* smem, const Tables* tab) {
  const float* src = reinterpret_cast<const float*>(tab);
  for (int k = 344 + (int)threadIdx.x; k < kTabFloats; k += blockDim.x) smem[k] = src[k];
}

// Stream the block's [valid x D] obs tile (LDS rows of stride DS) to HBM.
// t0 / nt: this thread's index among the nt storing threads (default: the block).
#ifndef PE_TILE_BATCH
#define PE_TILE_BATCH 1  // obs tile store: 16-B chunks per thread read from LDS ahead of their stores (f32 20x20: 3 same, 9 slower)
#endif
#ifndef PE_TILE_BATCH_CODES
#define PE_TILE_BATCH_CODES 4  // the same for the byte-coded tile (64x64: 25.6 -> 23.0 us; 2: 23.2, 6: 23.6)
#endif
__device__ __forceinline__ void store_tile(const float* rows, float* dst, int valid, int D, int DS,
                                           int t0 = -1, int nt = 0) {
  const int total = valid * D;
  const int tid = t0 < 0 ? (int)threadIdx.x : t0;
  const int nth = t0 < 0 ? (int)blockDim.x : nt;
  if (DS == D) {
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
      const int n4 = total >> 2;
      const float4* s4 = reinterpret_cast<const float4*>(rows);
      float4* d4 = reinterpret_cast<float4*>(dst);
#if !defined(PE_OBS_STORE_ASM) && !defined(PE_OBS_STORE_NT) && !defined(PE_TEMPORAL_OBS)
#define PE_OBS_STORE_ASM "sc1"
#endif
#if defined(PE_OBS_STORE_ASM)
      // the obs stream (28 MB per step at the headline batch) is written with sc1
      // (write-through; the line is dropped from the XCD's L2) so it does not evict
      // the envs' state from L2 / the Infinity Cache: plain stores 12.8 us, nt 11.4,
      // sc1 11.1 us per step (profiles/r1i_store_policy.json).  Inline asm: the
      // compiler does not count these in vmcnt; the reset path waits explicitly.
      typedef float v4f __attribute__((ext_vector_type(4)));
      const v4f* sv = reinterpret_cast<const v4f*>(rows);
      // PE_TILE_BATCH chunks per thread read from LDS before their stores are issued:
      // the asm's memory clobber keeps a later LDS read below an earlier store, so
      // one chunk at a time would wait out an LDS round trip per store
      constexpr int TB = PE_TILE_BATCH;
      for (int k0 = tid; k0 < n4; k0 += TB * nth) {
        v4f v[TB];
#pragma unroll
        for (int b = 0; b < TB; ++b)
          if (k0 + b * nth < n4) v[b] = sv[k0 + b * nth];
#pragma unroll
        for (int b = 0; b < TB; ++b)
          if (k0 + b * nth < n4)
            // s_nop 1: a 128-bit store reads its data VGPRs after issue; nothing inside
            // the asm pads that hazard for hipcc's next write of them
            asm volatile("global_store_dwordx4 %0, %1, off " PE_OBS_STORE_ASM "\n\ts_nop 1" ::"v"(d4 + k0 + b * nth),
                         "v"(v[b])
                         : "memory");
      }
#elif defined(PE_OBS_STORE_NT)
      typedef float v4f __attribute__((ext_vector_type(4)));
      const v4f* sv = reinterpret_cast<const v4f*>(rows);
      v4f* dv = reinterpret_cast<v4f*>(dst);
      for (int k = tid; k < n4; k += nth) __builtin_nontemporal_store(sv[k], &dv[k]);
#else
      for (int k = tid; k < n4; k += nth) d4[k] = s4[k];
#endif
      for (int k = (n4 << 2) + tid; k < total; k += nth) dst[k] = rows[k];
    } else {
      for (int k = tid; k < total; k += nth) dst[k] = rows[k];
    }
  } else {
    for (int k = tid; k < total; k += nth) {
      int r = k / D, c = k - r * D;
      dst[k] = rows[r * DS + c];
    }
  }
}

// Stream the block's byte-coded [valid x D] obs tile (contiguous codes, pe_coop.hpp
// ObsW<uint8_t>) to HBM as floats: 4 codes per thread and step expanded through the
// LDS code table ctab[256] into one 16-B store (same store policy as store_tile).
__device__ __forceinline__ void store_tile_codes(const uint8_t* codes, const float* ctab, float* dst, int valid, int D,
                                                 int t0, int nt) {
  const int total = valid * D;
  if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
    const int n4 = total >> 2;
    const uint32_t* c4 = reinterpret_cast<const uint32_t*>(codes);
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f* d4 = reinterpret_cast<v4f*>(dst);
    constexpr int TB = PE_TILE_BATCH_CODES;  // chunks per thread expanded before their stores (see store_tile)
    for (int k0 = t0; k0 < n4; k0 += TB * nt) {
      uint32_t c[TB];
#pragma unroll
      for (int b = 0; b < TB; ++b) c[b] = k0 + b * nt < n4 ? c4[k0 + b * nt] : 0u;
      v4f v[TB];
#pragma unroll
      for (int b = 0; b < TB; ++b) {
        v[b].x = ctab[c[b] & 255u];
        v[b].y = ctab[(c[b] >> 8) & 255u];
        v[b].z = ctab[(c[b] >> 16) & 255u];
        v[b].w = ctab[c[b] >> 24];
      }
#pragma unroll
      for (int b = 0; b < TB; ++b)
        if (k0 + b * nt < n4) {
#if defined(PE_OBS_STORE_ASM)
          asm volatile("global_store_dwordx4 %0, %1, off " PE_OBS_STORE_ASM "\n\ts_nop 1" ::"v"(d4 + k0 + b * nt),
                       "v"(v[b])
                       : "memory");
#else
          d4[k0 + b * nt] = v[b];
#endif
        }
    }
    for (int k = (n4 << 2) + t0; k < total; k += nt) dst[k] = ctab[codes[k]];
  } else {
    for (int k = t0; k < total; k += nt) dst[k] = ctab[codes[k]];
  }
}

// The byte-coded tile as it is (pe_step_codes): [valid x D] codes, 16-B sc1 stores
// where the destination allows, bytes for the rest.
__device__ __forceinline__ void store_tile_bytes(const uint8_t* codes, uint8_t* dst, int valid, int D, int t0,
                                                 int nt) {
  const int total = valid * D;
  int head = 0;
  if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
    const int n16 = total >> 4;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u* sv = reinterpret_cast<const v4u*>(codes);
    v4u* d4 = reinterpret_cast<v4u*>(dst);
    for (int k = t0; k < n16; k += nt) {
      const v4u v = sv[k];
      asm volatile("global_store_dwordx4 %0, %1, off " PE_OBS_STORE_ASM "\n\ts_nop 1" ::"v"(d4 + k), "v"(v) : "memory");
    }
    head = n16 << 4;
  }
  for (int k = head + t0; k < total; k += nt) dst[k] = codes[k];
}

// Cache-policy operand of the buffer-store builtin: bit 4 = sc1 on gfx950 (write-through,
// the line dropped from the XCD's L2 -- the obs stream must not evict the envs' state).
constexpr int kBufSc1 = 16;
constexpr int kBufRsrcWord3 = 0x00020000;  // raw buffer, 32-bit data format (range-checked)

// Stream a full block's [64 x D] f32 obs tile (LDS) to dst: thread t0 of nt stores the
// 16-B chunks t0, t0 + nt, ...; every chunk index past the tile is dropped by the
// buffer's range check, so each wave issues exactly NI stores (a count the compiler's
// wait for earlier loads relies on).
template <int D, int NT>
__device__ __forceinline__ void store_tile_buf(const float* rows, float* dst, int t0) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr int N4 = kQuadEnvs * D / 4, NI = (N4 + NT - 1) / NT;
  static_assert((kQuadEnvs * D) % 4 == 0, "whole 16-B chunks");
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, N4 * 16, kBufRsrcWord3);
  const v4f* sv = reinterpret_cast<const v4f*>(rows);
  v4f v[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int k = t0 + NT * j;
    v[j] = sv[k < N4 ? k : N4 - 1];
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) __builtin_amdgcn_raw_buffer_store_b128(v[j], rs, (t0 + NT * j) * 16, 0, kBufSc1);
}

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] |
// vmcnt[5:4] at [15:14]) waiting on vmcnt alone
constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }
constexpr int kVmcnt0 = vmcnt_imm(0);
// the store instructions store_tile_buf issues per wave
template <int D, int NT>
constexpr int tile_buf_stores() { return (kQuadEnvs * D / 4 + NT - 1) / NT; }
static_assert(vmcnt_imm(0) == 0x0F70, "s_waitcnt vmcnt(0)");

// ------------------------------------------------------------------ kernels
// Specialized fused step (compile-time C, R): two load rounds per lane, the rest
// from registers (pe_fast.hpp).  Same semantics as pe_step_wave.
template <int C, int R, bool ONEWORD>
__global__ __launch_bounds__(kBlock) void pe_step_fast(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  float* rows = smem + kTabFloats;
  const Geo& g = a.g;
  const Rules& rl = a.rl;
  const State& st = a.st;
  const int64_t e0 = (int64_t)blockIdx.x * kBlock;
  const int64_t e = e0 + threadIdx.x;
  const bool live = e < a.n;
  float* row = rows + threadIdx.x * g.DS;
  // ---- round 1: env-indexed loads
  uint4 sw = make_uint4(0u, 0u, 0u, 0u);
  int64_t action = 0;
  double ret = 0.0;
  if (live) {
    sw = st.scal[e];
    action = a.act_bytes == 8 ? reinterpret_cast<const int64_t*>(a.actions)[e]
                              : (int64_t)reinterpret_cast<const int32_t*>(a.actions)[e];
    ret = st.ep_ret[e];
  }
  load_tables(smem, st.tab);
  const Tables* ltab = reinterpret_cast<const Tables*>(smem);
  __syncthreads();
  if (live) {
    Scal s = unpack(sw);
    s.step = s.step < 65535 ? s.step + 1 : 65535;                  // plantos_env.py:162
    bool mv = false, water = false;
    int dxm = 0, dym = 0;
    if (action < 4) {                                              // :166
      const int64_t ai = action < 0 ? action + 4 : action;         // Python negative index
      if (ai < 0) {
        s.flags |= F_POISON_ACT;                                   // reference IndexError
        atomicOr(st.err_bits, F_POISON_ACT);
      } else {
        mv = true;                                                 // :186 N,E,S,W
        dxm = ai == 0 ? -1 : (ai == 2 ? 1 : 0);
        dym = ai == 1 ? 1 : (ai == 3 ? -1 : 0);
      }
    } else {
      water = true;
    }
    const int nx = s.x + dxm, ny = s.y + dym;
    const bool inb = mv && nx >= 0 && nx < g.G && ny >= 0 && ny < g.G;
    // ---- round 2: position-indexed loads
    Window<R, ONEWORD> w;
    w.load(st, g, e, s.episode, s.x, s.y);
    const int cell_o = s.x * g.G + s.y, cell_n = nx * g.G + ny;
    uint32_t* ep_o = st.expl + e * g.estride + (cell_o >> 5);
    uint32_t* ep_n = st.expl + e * g.estride + ((inb ? cell_n : cell_o) >> 5);
    const bool bitmap = (s.flags & F_EXPL_BITMAP) != 0u;
    uint32_t eo = 0u, en = 0u;
    if (inb) {
      if (bitmap) {
        eo = *ep_o;
        en = *ep_n;
      }
    }
    double h = 0.0;
    int dxv = 0;
    if (mv) {
      const bool ok = inb && w.code(dxm, ny) != OBST;              // :193-195
      if (ok) {
        const uint32_t n = (sel3<uint32_t>(dxm, w.vis32(2), w.vis32(3), w.vis32(4)) >> (4 * (ny + 2 - w.ybv))) & 15u;
        const bool never = n == 0u;                                // :197
        const uint32_t nib = n < 15u ? n + 1u : 15u;               // :203
        visit_bump_exact(st, g, e, cell_n, n);
        const int pb = 4 * (ny + 2) - 32 * ((4 * w.ybv) >> 5);
        uint32_t* vrow = vis_env(st, g, e, s.episode) + (int64_t)nx * g.NW + ((4 * w.ybv) >> 5);
#pragma unroll
        for (int k = 2; k <= 4; ++k) {
          if (k == 3 + dxm) {
            if (pb < 32) {
              w.vlo[k] = (w.vlo[k] & ~(0xFu << pb)) | (nib << pb);
              vrow[0] = w.vlo[k];
            } else {
              w.vhi[k] = (w.vhi[k] & ~(0xFu << (pb - 32))) | (nib << (pb - 32));
              vrow[1] = w.vhi[k];
            }
          }
        }
        if (bitmap) {
          const uint32_t bo = 1u << (cell_o & 31), bn = 1u << (cell_n & 31);
          if ((cell_o >> 5) == (cell_n >> 5)) {                    // explored[old]=1, [new]=2 (:198-200)
            uint32_t wv = eo;
            if (!(wv & bo)) { wv |= bo; s.expl++; }
            if (!(wv & bn)) { wv |= bn; s.expl++; }
            if (wv != eo) *ep_o = wv;
          } else {
            if (!(eo & bo)) { *ep_o = eo | bo; s.expl++; }
            if (!(en & bn)) { *ep_n = en | bn; s.expl++; }
          }
        } else if (never) {
          s.expl++;                                                // derived explored mode
        }
        s.x = nx;                                                  // :199
        s.y = ny;
        dxv = dxm;
        h = never ? rl.r_exploration : rl.r_revisit;               // :204-207
      } else {
        s.flags |= F_COLLIDED;                                     // :209
        s.coll = s.coll < 65535 ? s.coll + 1 : 65535;              // :210
        h = rl.r_invalid;                                          // :211
      }
    } else if (water) {
      const int cd = w.code(0, s.y);
      if (cd == THIRSTY) {                                         // fork plantos_env_new.py:237-240
        const int pb = 2 * (s.y + R) - 64 * ((2 * w.yb) >> 6);
        uint64_t* grow = st.grid + e * g.gstride + (int64_t)s.x * g.WPR + ((2 * w.yb) >> 6);
        if (pb < 64) {
          w.clo &= ~(1ull << pb);                                  // code 3 -> 2: clear the low bit
          grow[0] = w.clo;
        } else {
          w.chi &= ~(1ull << (pb - 64));
          grow[1] = w.chi;
        }
        w.refresh_centre();
        h = rl.r_goal;
      } else if (cd == HYD) {                                      // fork :241-242 (root raises)
        h = rl.r_mistake;
        if (!(s.flags & F_POISON_HYD)) atomicOr(st.err_bits, F_POISON_HYD);
        s.flags |= F_POISON_HYD;
      } else {
        h = rl.r_water_empty;                                      // :221-222
      }
    }
    double rew = rl.r_step;                                        // :164
    rew += h;
    bool term = s.expl >= s.total;                                 // :176, 244-246, 331
    const bool trunc = s.step >= rl.max_steps;                     // :177
    if (term && !(s.flags & F_BONUS)) {                            // :179-181
      rew += rl.r_complete;
      s.flags |= F_BONUS;
    }
    ret += rew;
    if (st.cur) term = curriculum_hit(st.cur, e, st.cur[e].thr, s.expl, s.total, rl.cur_term) || term;
    a.reward[e] = (float)rew;
    a.term[e] = term;
    a.trunc[e] = trunc;
    if (term || trunc) {                                           // ended: terminal outputs
      if (a.tobs) {
        obs_from_window<C, R, ONEWORD>(w, g.G, dxv, s.x, s.y, row, tpos, tvis);
        float* t = a.tobs + e * g.D;
        for (int k = 0; k < g.D; ++k) t[k] = row[k];
      }
      if (a.ep_ret_out) a.ep_ret_out[e] = ret;
      if (a.ep_len_out) a.ep_len_out[e] = s.step;
      if (a.tinfo) write_info(a.st, a.g, ltab, e, s, a.tinfo + e * PE_NINFO);
    }
    if ((term || trunc) && a.autoreset) {                          // DummyVecEnv auto-reset
      s = reset_env(st, g, rl, ltab, e, s.episode);
      st.ep_ret[e] = 0.0;
      st.scal[e] = pack(s);
      build_obs_fresh(a, st.grid + e * g.gstride, s, row, smem, tpos, tvis, a.st.ldx, a.st.ldy);  // rare path
    } else {
      st.ep_ret[e] = ret;
      st.scal[e] = pack(s);
      obs_from_window<C, R, ONEWORD>(w, g.G, dxv, s.x, s.y, row, tpos, tvis);
    }
  }
  __syncthreads();
  const int64_t valid = a.n - e0 < kBlock ? a.n - e0 : kBlock;
  store_tile(rows, a.obs + e0 * g.D, (int)valid, g.D, g.DS);
}

// (The round-1 phase ablations and the round-2 timing probes -- PE_ABLATE, PE_PROBE_*,
// PE_VIS_R1 -- were separate libraries built from this file; their results are in
// DESIGN.md §8 and profiles/r1d_ablation.json, profiles/r2ag_*; the probes are gone.)
#ifndef PE_GRID_R1
#define PE_GRID_R1 1  // one-word sector kernel: the grid block in round 1 (A/B: -DPE_GRID_R1=0)
#endif
#ifndef PE_WAVE_ROWSTORE_MIN
// pe_step_wave's obs row of D >= this many floats as 16-B stores (shorter: one float per
// lane): 64x64/C64/R32 93.8 -> 90.4 us, 40x40/C48/R8 76.7 -> 75.0, but 8x8/C16/R20
// 68.0 -> 70.2 (sc1 16-B stores: 90.8 / 76.7 / 70.4; profiles/r3x/)
#define PE_WAVE_ROWSTORE_MIN 200
#endif
#ifndef PE_QUAD_TILE_BUF
#define PE_QUAD_TILE_BUF 0  // sector kernel's f32 tile: asm sc1 stores (0); A/B: buffer stores (1, 2)
#endif
#ifndef PE_BT_DV
#define PE_BT_DV 1  // the byte-coded C16R6 kernel defers its overflow writes as the f32 one (A/B: 0)
#endif
#ifndef PE_BT_EARLY
#define PE_BT_EARLY 1  // the byte-coded one-word kernel loads a predicted single truncation's record early (A/B: 0)
#endif
#ifndef PE_REG_STAGE
#define PE_REG_STAGE 0  // f32 kernels without the early record: a predicted single truncation's record
                        // register-staged into LDS during round 2 (round 6 A/B: not kept)
#endif
#ifndef PE_RT_REG
#define PE_RT_REG 1  // runtime sector kernel: rays from a per-wave register window (A/B: 0, the LDS-table form)
#endif
#ifndef PE_BT_INFO_REG
#define PE_BT_INFO_REG 1  // byte-coded LDS-DMA kernels: the info rows register-staged by the info wave (A/B: 0)
#endif
#ifndef PE_GR2
#define PE_GR2 0  // the two-word C16R6 kernel (G <= 28) loads the loader env's grid block in round 1 (A/B: not kept)
#endif
#ifndef PE_EARLY2
#define PE_EARLY2 0  // one-word early-record kernels: two predicted truncations' records by waves 0 and 1 (A/B: not kept)
#endif
#ifndef PE_REG_STAGE_SMALL
#define PE_REG_STAGE_SMALL 0  // ... and the 16 / 32-env small-batch shapes (A/B: 1)
#endif
#ifndef PE_DONE_BATCH
#define PE_DONE_BATCH 1  // done path: the terminal / fresh obs row copies as batched reads, then writes (A/B: 0)
#endif
#ifndef PE_DONE_ONEWAIT
// done path without the early record: every load (record, terminal-info rows, terminal obs)
// issued before any store, one wait, then the stores -- vmcnt counts stores too, in order, so
// a load consumed after a store waits for that store (A/B: 0; 2: in every kernel)
#define PE_DONE_ONEWAIT 1
#endif
#ifndef PE_BT_STAGE_MIN_C
#define PE_BT_STAGE_MIN_C 64  // byte-coded kernels stage the predicted record by LDS-DMA from this C on (A/B: 0)
#endif
#ifndef PE_STAGGER_GROUPS
#define PE_STAGGER_GROUPS 4  // sector kernel: the grid's start-delay groups (A/B: -DPE_STAGGER_GROUPS=n)
#endif

// Diagnostic phase stamps (tools/stamps.py builds a SEPARATE library with
// -DPE_STAMPS): lane 0 of every wave of the sector kernel records s_memrealtime
// (100 MHz) at 8 points; pe_debug_stamps() copies them out.  Not in the product build.
#if defined(PE_STAMPS) || defined(PE_STAMPS_RESET)
__device__ uint64_t g_stamps[16384 * 8];
#define PE_STAMP_RAW(k)                                                                     \
  do {                                                                                      \
    uint64_t _t;                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const int _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                     \
    if ((threadIdx.x & 63) == 0 && _w < 16384) g_stamps[_w * 8 + (k)] = _t;                \
  } while (0)
#endif
#ifdef PE_STAMPS
#define PE_STAMP(k) PE_STAMP_RAW(k)
// done-path stamps of the wave running a block's auto-reset (per block)
__device__ uint64_t g_dstamps[16384 * 8];
#define PE_DSTAMP(k)                                                                        \
  do {                                                                                      \
    uint64_t _t;                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 16384) g_dstamps[blockIdx.x * 8 + (k)] = _t; \
  } while (0)
#else
#define PE_DSTAMP(k) \
  do {               \
  } while (0)
#define PE_STAMP(k) \
  do {              \
  } while (0)
#endif
#ifdef PE_STAMPS_RESET
#define PE_RSTAMP(k) PE_STAMP_RAW(k)
#else
#define PE_RSTAMP(k) \
  do {               \
  } while (0)
#endif

// Quadrant-split fused step (pe_quad.hpp): 4 waves x 64 envs per workgroup.
// Same semantics as pe_step_wave.
template <int R>
constexpr int quad_tile_off() {
  return (kTabFloats + (2 * R + 3) * kQuadEnvs * 2 + 7 * kQuadEnvs + 3) & ~3;
}
// the runtime sector kernel (pe_step_quad<0, 0, ...>): maxima and its layout -- C up to
// 32 with the f32 tile, up to 64 with the byte-coded one (the f32 tile of 64 rays holds
// the kernel to one workgroup per CU)
constexpr int kRtCMax = 32, kRtCMaxBT = 64, kRtRMax = 14;
__host__ __device__ constexpr int quad_tile_off_rt(int R) {
  return (kTabFloats + (2 * R + 3) * kQuadEnvs * 2 + 7 * kQuadEnvs + 3) & ~3;
}
// byte-coded tile (BT): the code table ctab[256] after the [64 x D] code tile
template <int R, int C>
constexpr int quad_ctab_off() {
  return quad_tile_off<R>() + ((kQuadEnvs * (5 * C + 27) + 15) / 16) * 4;
}
__host__ __device__ constexpr int quad_ctab_off_rt(int R, int C) {
  return quad_tile_off_rt(R) + ((kQuadEnvs * (5 * C + 27) + 15) / 16) * 4;
}
// offset (floats) from the tile to what follows it (+ the code table)
__host__ __device__ constexpr int quad_rtab_off(int C, bool bt) {
  return bt ? ((kQuadEnvs * (5 * C + 27) + 15) / 16) * 4 + 256 : kQuadEnvs * (5 * C + 27);
}
// the runtime sector kernel's probe table in LDS (floats; C rays x R rounded up to 8
// int16 entries), placed after the tile (+ code table) and before the staging region
__host__ __device__ constexpr int quad_rtab_floats(int C, int R) { return C * ((R + 7) & ~7); }  // u32 entries

// ---- pe_step_quad's auto-reset slow path (a block with a done env), out of line:
// kept in separate functions so that their register demand (map generation, the
// cooperative reset) does not raise the hot path's.  `ka` is the kernel's
// argument segment (StepArgs); LDS is the kernel's dynamic LDS (same layout).
// the kernel's argument segment as a generic pointer (constant and global
// addresses coincide in the flat space)
__device__ __forceinline__ const void* kernargs() {
  return reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(__builtin_amdgcn_kernarg_segment_ptr()));
}

__device__ __forceinline__ bool quad_coop(const StepArgs& a, int ndone) {
#ifdef PE_NO_COOP
  return false;
#else
  return a.autoreset && ndone <= a.coop_max_done;
#endif
}

// The single-done early record's terminal info by a second wave (round 5): the commit
// wave loads the record, the info wave (kQuadInfoWave) the env's current rows in round
// 2; at the done path the info wave reduces and stores the info while the commit wave
// takes the record -- the info's wave reductions off the one-done block's critical path.
// The commit wave parks the env's post-step scalars + wfix in free table words
// (dist[24..28]) before the done barrier.  A/B: -DPE_INFO_WAVE=0.
#ifndef PE_INFO_WAVE
#define PE_INFO_WAVE 1
#endif
constexpr int kQuadInfoWave = 2;  // (4-wave kernels; the slice / position wave)
constexpr int kInfoParkF = 24;    // floats 24..28 of dist[] (dist[0..R+1] and the one-hot rows at 48.. in use)
__device__ __forceinline__ bool el_info_hit(int64_t e_info, int64_t e0, const float* smem) {
  // the block's one done env (the done mask in dist[70..71]) is the info wave's early env
  const uint64_t dmw = reinterpret_cast<const uint64_t*>(smem)[35];
  return e_info >= 0 && e_info == e0 + (__ffsll((unsigned long long)dmw) - 1);
}

// BT: the obs tile holds byte codes (ctab: the LDS code table), see pe_step_quad.
// DB: the row copies batched (PE_DONE_BATCH) -- where the registers are there: rows of at most
// 128 values, or a path out of line (the far kernel's far_done); inlined into the C64 / runtime
// byte-tile kernels (KD = 6) it cost their hot path (64x64/C64 24.15 -> 25.0 us, profiles/r6h/)
template <int NW, bool ONEWORD, int KD, bool BT = false, bool DB = (KD <= 2)>  // one copy per kernel: each
                                                                              // inherits its kernel's register budget
__device__ __forceinline__ uint4 quad_done_path(const void* ka, int tile_off, int C, int R, int lane, int wv, int CW,
                                                int64_t e0, bool done, uint4 sp, double ret, int ndone, bool wfix,
                                                const float* ctab = nullptr, const float* stage = nullptr,
                                                bool stage_info = false, int64_t e_early = -1,
                                                const PfLoad<ONEWORD ? 1 : kCoopWPR, KD>* early = nullptr,
                                                const Row4<ONEWORD ? 1 : kCoopWPR>* early_rows = nullptr,
                                                int64_t e_info = -1, bool stage_reg = false, bool info_iw = false,
                                                const float* ipark = nullptr) {
  // stage_reg: `stage` was written by register-staged copies before the window barrier
  // (pe_step_quad kRegStage), not by LDS-DMA: nothing to wait for.  info_iw: the env's
  // terminal-info rows were register-staged into `stage` (after the record) by the info
  // wave (kQuadInfoWave), which writes the terminal info beside the commit wave's reset
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const StepArgs& a = *reinterpret_cast<const StepArgs*>(ka);
  const Geo& g = a.g;
  const Rules& rl = a.rl;
  const State& st = a.st;
  float* tdist = smem;
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  const Tables* ltab = reinterpret_cast<const Tables*>(smem);
  uint64_t* lrow = reinterpret_cast<uint64_t*>(smem + kTabFloats);
  using OT = typename std::conditional<BT, uint8_t, float>::type;
  OT* rows = reinterpret_cast<OT*>(smem + tile_off);
  OT* row = rows + lane * g.D;
  const int64_t e = e0 + lane;
  Scal s = unpack(sp);
  constexpr int MAXW = ONEWORD ? 1 : kCoopWPR;
  // the early record's terminal info is the info wave's (the kernel's kInfoW)
  constexpr bool kIW = PE_INFO_WAVE && NW == 4 && ONEWORD && KD <= 2;
  // loads before stores (PE_DONE_ONEWAIT): the one-word f32 kernels (1); every kernel with
  // batched row copies (2: the multi-word and byte-tile ones measured slower)
  constexpr bool kOneWait = PE_DONE_ONEWAIT && PE_DONE_BATCH && DB && (PE_DONE_ONEWAIT > 1 || (ONEWORD && !BT));
  // the table reads of the reset / info helpers as LDS reads of ltab (pe_coop.hpp LdsTables):
  // the one-word f32 kernels (the others measured slower with them, 64x64 +0.2 us desync)
  constexpr bool kLT = ONEWORD && !BT;
  // an obs tile value as a float (BT: expand the code)
  auto tval = [&](const OT* r, int k) -> float {
    if constexpr (BT) return ctab[r[k]];
    else return r[k];
  };
  // a prefetched record's fresh obs row into tile row `o` once taken (BT: codes)
  auto take = [&](int64_t el, uint32_t episode, const PfLoad<MAXW, KD>& pl, Row4<MAXW>& rw, Scal& ns, OT* o) -> bool {
    return coop_take_prefetched<MAXW, KD, OT>(a.pf, g, el, episode, pl, rw, ns, o, lane);
  };
  if (ndone == 1 && quad_coop(a, ndone)) {
    // One done env (the usual case with desynchronized episodes): the commit wave,
    // which holds its scalars, resets it alone -- no staging, one barrier.
    if (wv == CW) {
      PE_DSTAMP(0);
      const uint64_t dmw = reinterpret_cast<const uint64_t*>(smem)[35];
      const int l = __ffsll((unsigned long long)dmw) - 1;
      const int64_t el = e0 + l;
      OT* orow = rows + l * g.D;
      // early: the kernel loaded this env's record and rows behind the compute phase
      const bool early_hit = KD <= 2 && early != nullptr && el == e_early;
      if (early_hit) {
        // the record and the env's rows were loaded behind the compute phase (the
        // kernel's early record): every wait here is for loads issued ~1 us ago.
        // Terminal obs held in registers while the fresh row replaces it in the tile;
        // stores only after every load is consumed.
        const int wf = __builtin_amdgcn_readlane((int)wfix, l);
        const Scal sv = unpack(make_uint4((uint32_t)__builtin_amdgcn_readlane((int)sp.x, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.y, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.z, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.w, l)));
        float tv[KD];
#pragma unroll
        for (int j = 0; j < KD; ++j) tv[j] = lane + 64 * j < g.D ? tval(orow, lane + 64 * j) : 0.0f;
        PE_DSTAMP(1);
        // (the terminal info: the info wave's, below, when it loaded the env's rows)
        if (a.tinfo && !kIW) coop_info_store<MAXW, kLT>(st, g, *early_rows, sv, a.tinfo + el * PE_NINFO, lane, wf, ltab);
        PE_DSTAMP(2);
        Row4<MAXW> rw;
        Scal ns;
        asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
        if (take(el, sv.episode, *early, rw, ns, orow)) {
          ns = coop_apply_reset<MAXW, kLT>(st, g, el, ns, false, rw, lane, ltab, true);
        } else {  // the record is not this reset's (not generated yet): generate in place
          uint64_t* scr = reinterpret_cast<uint64_t*>(lrow) + 162 + wv * coop_scratch_words(g.G, g.WPR);
          ns = coop_reset_env<MAXW, kLT>(st, g, rl, el, sv.episode, false, rw, lane, scr, ltab);
          coop_fresh_obs<MAXW>(g, rw, ns, orow, tdist, tpos, tvis, st.ldx, st.ldy, lane);
        }
        PE_DSTAMP(3);
        if (a.tobs) {
          float* t = a.tobs + el * g.D;
#pragma unroll
          for (int j = 0; j < KD; ++j)
            if (lane + 64 * j < g.D) t[lane + 64 * j] = tv[j];
        }
        if (lane == 0) a.pf.flag[el] = 1;  // its next map goes into the next generating batch
        PE_DSTAMP(4);
        if (done) {  // lane l: program order after its commit stores
          s = ns;
          st.ep_ret[e] = 0.0;
          st.scal[e] = pack(s);
        }
        PE_DSTAMP(5);
      } else {
        // the record: staged into LDS before the done barrier (stage), or loaded now
        PfLoad<MAXW, KD> pl;
        if (a.pf.scal && !stage) coop_load_prefetched<MAXW, KD, OT>(a.pf, g, el, pl, lane);  // in flight from here on
        bool keep = false;
        if (done && st.cur) keep = curriculum_on_reset(st.cur, e, rl);  // A2C_training.py:56-95
        const bool kp = __builtin_amdgcn_readlane((int)keep, l) != 0;
        const int wf = __builtin_amdgcn_readlane((int)wfix, l);
        const Scal sv = unpack(make_uint4((uint32_t)__builtin_amdgcn_readlane((int)sp.x, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.y, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.z, l),
                                          (uint32_t)__builtin_amdgcn_readlane((int)sp.w, l)));
        if constexpr (kOneWait) {
          // loads first (the record above, the info rows, the terminal obs out of the
          // tile), one wait, then every store
          if (st.cur) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the commit's rows landed
          const bool iload = a.tinfo && !info_iw && !stage_info;
          Row4<MAXW> ir{0ull, 0ull, 0ull, 0ull};
          if (iload) ir = coop_info_rows<MAXW>(st, g, el, lane);
          float tv[KD];
#pragma unroll
          for (int j = 0; j < KD; ++j) tv[j] = a.tobs && lane + 64 * j < g.D ? tval(orow, lane + 64 * j) : 0.0f;
          __builtin_amdgcn_s_waitcnt(0x0F70);  // (tracked: no later wait for these loads; stage: the DMA)
          PE_DSTAMP(1);
          if (a.tinfo && !info_iw) {
            if (stage_info)
              coop_info_store<MAXW, kLT>(st, g,
                                    pf_stage_rows<MAXW>(reinterpret_cast<const uint64_t*>(
                                                            stage + 4 + 4 * pf_grid_units(g.G, g.WPR) + a.pf.ostride / 4),
                                                        g, lane),
                                    sv, a.tinfo + el * PE_NINFO, lane, wf, ltab);
            else
              coop_info_store<MAXW, kLT>(st, g, ir, sv, a.tinfo + el * PE_NINFO, lane, wf, ltab);
          }
          PE_DSTAMP(2);
          Row4<MAXW> rw;
          Scal ns;
          asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
          const bool took = stage ? pf_stage_take<MAXW, OT, KD>(stage, g, (int)a.pf.ostride, sv.episode, rw, ns, orow, lane)
                                  : (a.pf.scal && take(el, sv.episode, pl, rw, ns, orow));
          if (took) {
            ns = coop_apply_reset<MAXW, kLT>(st, g, el, ns, kp, rw, lane, ltab, true);
          } else {
            uint64_t* scr = reinterpret_cast<uint64_t*>(lrow) + 162 + wv * coop_scratch_words(g.G, g.WPR);
            ns = coop_reset_env<MAXW, kLT>(st, g, rl, el, sv.episode, kp, rw, lane, scr, ltab);
            coop_fresh_obs<MAXW>(g, rw, ns, orow, tdist, tpos, tvis, st.ldx, st.ldy, lane);
          }
          PE_DSTAMP(3);
          if (a.tobs) {
            float* t = a.tobs + el * g.D;
#pragma unroll
            for (int j = 0; j < KD; ++j)
              if (lane + 64 * j < g.D) t[lane + 64 * j] = tv[j];
          }
          if (a.pf.scal && lane == 0) a.pf.flag[el] = 1;  // its next map goes into the next generating batch
          PE_DSTAMP(4);
          if (done) {  // lane l: program order after its commit stores
            s = ns;
            st.ep_ret[e] = 0.0;
            st.scal[e] = pack(s);
          }
          PE_DSTAMP(5);
        } else {
          if (a.tobs) {  // (the row's reads first, then the stores: one LDS round trip, not one per 64 values)
            float* t = a.tobs + el * g.D;
            if constexpr (PE_DONE_BATCH && DB) {
              float tv[KD];
#pragma unroll
              for (int j = 0; j < KD; ++j) tv[j] = lane + 64 * j < g.D ? tval(orow, lane + 64 * j) : 0.0f;
#pragma unroll
              for (int j = 0; j < KD; ++j)
                if (lane + 64 * j < g.D) t[lane + 64 * j] = tv[j];
            } else {
              for (int k2 = lane; k2 < g.D; k2 += 64) t[k2] = tval(orow, k2);
            }
          }
          // with the curriculum the commit stored this env's rows: they must land before
          // the info reads them and the reset rewrites them
          if (st.cur || (stage && !stage_reg)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (stage: the LDS-DMA landed)
          PE_DSTAMP(1);
          if (a.tinfo && !info_iw) {  // (register-staged info rows: the info wave's)
            if (stage_info)  // the env's rows came with the record
              coop_info_store<MAXW, kLT>(st, g,
                                    pf_stage_rows<MAXW>(reinterpret_cast<const uint64_t*>(
                                                            stage + 4 + 4 * pf_grid_units(g.G, g.WPR) + a.pf.ostride / 4),
                                                        g, lane),
                                    sv, a.tinfo + el * PE_NINFO, lane, wf, ltab);
            else
              coop_write_info<MAXW, kLT>(st, g, el, sv, a.tinfo + el * PE_NINFO, lane, wf, ltab);
          }
          PE_DSTAMP(2);
          Row4<MAXW> rw;
          Scal ns;
          asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
          const bool took = stage ? pf_stage_take<MAXW, OT, PE_DONE_BATCH && DB ? KD : 0>(stage, g, (int)a.pf.ostride, sv.episode,
                                                                                    rw, ns, orow, lane)
                                  : (a.pf.scal && take(el, sv.episode, pl, rw, ns, orow));
          if (took) {
            ns = coop_apply_reset<MAXW, kLT>(st, g, el, ns, kp, rw, lane, ltab, true);
          } else {
            uint64_t* scr = reinterpret_cast<uint64_t*>(lrow) + 162 + wv * coop_scratch_words(g.G, g.WPR);
            ns = coop_reset_env<MAXW, kLT>(st, g, rl, el, sv.episode, kp, rw, lane, scr, ltab);
            coop_fresh_obs<MAXW>(g, rw, ns, orow, tdist, tpos, tvis, st.ldx, st.ldy, lane);
          }
          PE_DSTAMP(3);
          if (a.pf.scal && lane == 0) a.pf.flag[el] = 1;  // its next map goes into the next generating batch
          PE_DSTAMP(4);
          if (done) {  // lane l: program order after its commit stores
            s = ns;
            st.ep_ret[e] = 0.0;
            st.scal[e] = pack(s);
          }
          PE_DSTAMP(5);
        }
      }
    } else if (kIW && a.tinfo && wv == kQuadInfoWave && el_info_hit(e_info, e0, smem)) {
      // the terminal info of the early-record env (_get_info, plantos_env.py:317-336) by
      // the info wave, beside the commit wave's reset: the env's rows came with round 2,
      // its post-step scalars through LDS (quad_info_park)
      const float* pk = smem + kInfoParkF;
      const uint4 spk = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[0])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[1])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[2])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[3])));
      const int wf = __builtin_amdgcn_readfirstlane(__float_as_int(pk[4]));
      coop_info_store<MAXW, kLT>(st, g, *early_rows, unpack(spk), a.tinfo + e_info * PE_NINFO, lane, wf, ltab);
    } else if (info_iw && a.tinfo && wv == kQuadInfoWave) {
      // the terminal info of the staged env (the block's one done env: its truncation was
      // predicted) by the info wave from its rows register-staged in round 2 and its
      // post-step scalars parked by the commit wave (kInfoParkF; ipark: the far kernel's slot)
      const uint64_t dmw = reinterpret_cast<const uint64_t*>(smem)[35];
      const int64_t el = e0 + (__ffsll((unsigned long long)dmw) - 1);
      const float* pk = ipark ? ipark : smem + kInfoParkF;
      const uint4 spk = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[0])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[1])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[2])),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(pk[3])));
      const int wf = __builtin_amdgcn_readfirstlane(__float_as_int(pk[4]));
      coop_info_store<MAXW, kLT>(st, g,
                            pf_stage_rows<MAXW>(reinterpret_cast<const uint64_t*>(
                                                    stage + 4 + 4 * pf_grid_units(g.G, g.WPR) + a.pf.ostride / 4),
                                                g, lane),
                            unpack(spk), a.tinfo + el * PE_NINFO, lane, wf, ltab);
    }
    __syncthreads();  // the fresh obs row is in the tile
    __builtin_amdgcn_s_waitcnt(0x0F70);  // see the end of the path below
    return pack(s);
  }
  if (quad_coop(a, ndone)) {
    // A few done envs: wave-cooperative resets (pe_coop.hpp), spread over the
    // block's waves (the k-th done env to wave k % NW).  For each, the 64 lanes
    // copy the terminal obs row out, write the terminal info, generate the map,
    // write grid + visit rows and build the fresh obs into the env's tile row,
    // which the tile store then streams out with the others.  The commit wave
    // stages each done env's scalars in the (dead) window region of LDS and
    // stores the new ones afterwards: every store to an env's scalars stays in
    // its own lane, in program order.
    uint32_t* stage = reinterpret_cast<uint32_t*>(lrow);  // [64][5]: packed scalars, keep
    uint64_t* dmask = reinterpret_cast<uint64_t*>(stage + 5 * kQuadEnvs);
    const int NWv = blockDim.x >> 6;
    if (wv == CW) {
      bool keep = false;
      if (done) {
        if (st.cur) keep = curriculum_on_reset(st.cur, e, rl);  // A2C_training.py:56-95
        stage[5 * lane] = sp.x;
        stage[5 * lane + 1] = sp.y;
        stage[5 * lane + 2] = sp.z;
        stage[5 * lane + 3] = sp.w;
        stage[5 * lane + 4] = (uint32_t)keep | ((uint32_t)wfix << 1);
      }
      const uint64_t dm = __ballot(done);
      if (lane == 0) *dmask = dm;
      // with the curriculum, the commit's grid / visit stores of a done env
      // (watering, the carried visit) must land before other waves read its rows
      // (terminal info) and write new ones; otherwise it made none (see the commit)
      if (st.cur) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    {
      const uint64_t dml = *dmask;  // uniform: read into scalar registers
      uint64_t dm = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dml) |
                    ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(dml >> 32)) << 32);
      for (int k = 0; dm; ++k) {
        const int l = __ffsll((unsigned long long)dm) - 1;
        dm &= dm - 1;
        if (k % NWv != wv) continue;
        const int64_t el = e0 + l;
        OT* orow = rows + l * g.D;
        if constexpr (kOneWait) {
          // loads first (the record, the info rows, the terminal obs), one wait, then
          // every store (as the single-done path)
          const uint4 sl = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l]),
                                      (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 1]),
                                      (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 2]),
                                      (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 3]));
          const int kw = __builtin_amdgcn_readfirstlane((int)stage[5 * l + 4]);
          const bool kp = (kw & 1) != 0;
          const Scal sv = unpack(sl);
          const bool eh = KD <= 2 && early != nullptr && el == e_early;
          const bool erows = eh && (!kIW || e_info == el);  // (as below)
          PfLoad<MAXW, KD> pl;
          if (a.pf.scal && !eh) coop_load_prefetched<MAXW, KD, OT>(a.pf, g, el, pl, lane);
          Row4<MAXW> ir{0ull, 0ull, 0ull, 0ull};
          if (a.tinfo && !erows) ir = coop_info_rows<MAXW>(st, g, el, lane);
          float tv[KD];
#pragma unroll
          for (int j = 0; j < KD; ++j) tv[j] = a.tobs && lane + 64 * j < g.D ? tval(orow, lane + 64 * j) : 0.0f;
          __builtin_amdgcn_s_waitcnt(0x0F70);
          if (a.tinfo) coop_info_store<MAXW, kLT>(st, g, erows ? *early_rows : ir, sv, a.tinfo + el * PE_NINFO, lane, kw >> 1, ltab);
          Row4<MAXW> rw;
          Scal ns;
          asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
          if (a.pf.scal && take(el, sv.episode, eh ? *early : pl, rw, ns, orow)) {
            ns = coop_apply_reset<MAXW, kLT>(st, g, el, ns, kp, rw, lane, ltab, true);
          } else {
            uint64_t* scr = reinterpret_cast<uint64_t*>(lrow) + 162 + wv * coop_scratch_words(g.G, g.WPR);
            ns = coop_reset_env<MAXW, kLT>(st, g, rl, el, sv.episode, kp, rw, lane, scr, ltab);
            coop_fresh_obs<MAXW>(g, rw, ns, orow, tdist, tpos, tvis, st.ldx, st.ldy, lane);
          }
          if (a.tobs) {
            float* t = a.tobs + el * g.D;
#pragma unroll
            for (int j = 0; j < KD; ++j)
              if (lane + 64 * j < g.D) t[lane + 64 * j] = tv[j];
          }
          if (a.pf.scal && lane == 0) a.pf.flag[el] = 1;  // its next map goes into the next generating batch
          const uint4 np = pack(ns);
          if (lane == 0) {
            stage[5 * l] = np.x;
            stage[5 * l + 1] = np.y;
            stage[5 * l + 2] = np.z;
            stage[5 * l + 3] = np.w;
          }
          continue;
        }
        if (a.tobs) {  // (the row's reads first, then the stores: one LDS round trip, not one per 64 values)
          float* t = a.tobs + el * g.D;
          if constexpr (PE_DONE_BATCH && DB) {
            float tv[KD];
#pragma unroll
            for (int j = 0; j < KD; ++j) tv[j] = lane + 64 * j < g.D ? tval(orow, lane + 64 * j) : 0.0f;
#pragma unroll
            for (int j = 0; j < KD; ++j)
              if (lane + 64 * j < g.D) t[lane + 64 * j] = tv[j];
          } else {
            for (int k2 = lane; k2 < g.D; k2 += 64) t[k2] = tval(orow, k2);
          }
        }
        const uint4 sl = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l]),
                                    (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 1]),
                                    (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 2]),
                                    (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[5 * l + 3]));
        const int kw = __builtin_amdgcn_readfirstlane((int)stage[5 * l + 4]);
        const bool kp = (kw & 1) != 0;
        const Scal sv = unpack(sl);
        // the prefetched record's loads go out first, the terminal info's after them --
        // or both came with round 2 (the kernel's early record of this wave's env)
        const bool eh = KD <= 2 && early != nullptr && el == e_early;
        PfLoad<MAXW, KD> pl;
        if (a.pf.scal && !eh) coop_load_prefetched<MAXW, KD, OT>(a.pf, g, el, pl, lane);
        if (a.tinfo) {
          // (with the info wave the single early env's rows are that wave's, not this one's;
          // kEarly2's waves hold their env's rows themselves: e_info == e_early)
          if (eh && (!kIW || e_info == el))
            coop_info_store<MAXW, kLT>(st, g, *early_rows, sv, a.tinfo + el * PE_NINFO, lane, kw >> 1, ltab);
          else
            coop_write_info<MAXW, kLT>(st, g, el, sv, a.tinfo + el * PE_NINFO, lane, kw >> 1, ltab);
        }
        Row4<MAXW> rw;
        Scal ns;
        asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
        if (a.pf.scal && take(el, sv.episode, eh ? *early : pl, rw, ns, orow)) {
          ns = coop_apply_reset<MAXW, kLT>(st, g, el, ns, kp, rw, lane, ltab, true);
        } else {
          uint64_t* scr = reinterpret_cast<uint64_t*>(lrow) + 162 + wv * coop_scratch_words(g.G, g.WPR);
          ns = coop_reset_env<MAXW, kLT>(st, g, rl, el, sv.episode, kp, rw, lane, scr, ltab);
          coop_fresh_obs<MAXW>(g, rw, ns, orow, tdist, tpos, tvis, st.ldx, st.ldy, lane);
        }
        if (a.pf.scal && lane == 0) a.pf.flag[el] = 1;  // its next map goes into the next generating batch
        const uint4 np = pack(ns);
        if (lane == 0) {
          stage[5 * l] = np.x;
          stage[5 * l + 1] = np.y;
          stage[5 * l + 2] = np.z;
          stage[5 * l + 3] = np.w;
        }
      }
    }
    __syncthreads();  // fresh tile rows and new scalars complete
    if (wv == CW && done) {
      s = unpack(make_uint4(stage[5 * lane], stage[5 * lane + 1], stage[5 * lane + 2], stage[5 * lane + 3]));
      st.ep_ret[e] = 0.0;
      st.scal[e] = pack(s);
    }
    // vmcnt(0) as an instruction the compiler tracks (not asm): nothing of this path
    // is pending where it rejoins the hot path, so the tile store loop after it
    // carries no per-iteration wait (only the commit wave waits here, and it does
    // not take part in the tile store)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    return pack(s);
  }
  // Many done envs (a synchronized batch truncating together): one lane per env.
  // The done env's own obs-tile row is free once its terminal obs is copied out:
  // the new map is generated there when it can hold the grid image (LDS latency
  // for the rejection-sampling scans; the fresh obs row goes straight to HBM
  // after the tile store, quad_done_obs)
  // (BT: the tile row holds D bytes, never the image; the fresh obs of that case is
  // built from the env's grid in HBM after the tile store, quad_done_obs)
  const bool scratch_ok = !BT && reset_scratch_bytes(g.G, g.WPR, rl.P) <= 4 * g.D;
  // 8-B aligned start inside the row (rows is 16-B aligned, D is odd)
  uint64_t* sg = reinterpret_cast<uint64_t*>(reinterpret_cast<float*>(rows) + lane * g.D + ((lane * g.D) & 1));
  // LIDAR offsets for the reset-path obs builders, staged in the (now dead) window region
  const signed char* lldx = reinterpret_cast<const signed char*>(lrow);
  const signed char* lldy = lldx + C * R;
  PE_RSTAMP(0);
  load_tables_cold(smem, st.tab);
  for (int k = threadIdx.x; k < C * R; k += blockDim.x) {
    reinterpret_cast<signed char*>(lrow)[k] = st.ldx[k];
    reinterpret_cast<signed char*>(lrow)[C * R + k] = st.ldy[k];
  }
  __syncthreads();
  if (done) {
    if (a.tobs) {
      float* t = a.tobs + e * g.D;
      for (int k = 0; k < g.D; ++k) t[k] = tval(row, k);
    }
    PE_RSTAMP(1);
    if (a.tinfo) write_info(a.st, a.g, ltab, e, s, a.tinfo + e * PE_NINFO, wfix);
    PE_RSTAMP(2);
    if (!a.autoreset) {
    } else if (scratch_ok) {
      s = reset_env_scratch(st, g, rl, ltab, e, s.episode, sg);
      PE_RSTAMP(3);
    } else {
      s = reset_env(st, g, rl, ltab, e, s.episode);
      if constexpr (!BT) build_obs_fresh(a, st.grid + e * g.gstride, s, row, tdist, tpos, tvis, lldx, lldy);
    }
    if (a.autoreset) {
      st.ep_ret[e] = 0.0;
      st.scal[e] = pack(s);
    }
  }
  __syncthreads();
  return pack(s);
}

// The lane-per-env path's fresh obs, after the tile store (see quad_done_path).
template <int NW, bool BT = false>
__device__ __forceinline__ void quad_done_obs(const void* ka, int tile_off, int lane, int64_t e, bool done, uint4 sp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const StepArgs& a = *reinterpret_cast<const StepArgs*>(ka);
  const Geo& g = a.g;
  float* row = smem + tile_off + lane * g.D;
  // the grid image: the LDS scratch in the env's tile row, or (BT) the env's rows in HBM
  const uint64_t* sg = BT ? a.st.grid + e * g.gstride : reinterpret_cast<const uint64_t*>(row + ((lane * g.D) & 1));
  const signed char* lldx = reinterpret_cast<const signed char*>(smem + kTabFloats);
  PE_RSTAMP(4);
  if (done) {
    if (BT && a.obs_codes)
      build_obs_fresh_codes(a, sg, unpack(sp), a.obs_codes + e * g.D, lldx, lldx + g.C * g.R);
    else
      build_obs_fresh(a, sg, unpack(sp), a.obs + e * g.D, smem, smem + 72, smem + 328, lldx, lldx + g.C * g.R);
  }
  PE_RSTAMP(5);
}

// The action's move / watering decode (plantos_env.py:166, 186-195) and the window
// coordinates it implies, from the scalars before the step.
struct QuadMove {
  bool mv, water, bad, inb;      // move / water / reference IndexError / target in bounds
  int dxm, dym, nx, ny, nyc;     // direction, target, target column clamped to the map
  int yb, ybv, cell_o, cell_n;   // window's first padded grid / visit column, old / new cell
};
template <bool ONEWORD>
__device__ __forceinline__ QuadMove quad_move(const Scal& s, int64_t action, int G) {
  QuadMove m;
  m.mv = false;
  m.water = false;
  m.bad = false;
  m.dxm = 0;
  m.dym = 0;
  if (action < 4) {                                              // plantos_env.py:166
    const int64_t ai = action < 0 ? action + 4 : action;         // Python negative index
    if (ai < 0) {
      m.bad = true;                                              // reference IndexError
    } else {
      m.mv = true;                                               // :186 N,E,S,W
      m.dxm = ai == 0 ? -1 : (ai == 2 ? 1 : 0);
      m.dym = ai == 1 ? 1 : (ai == 3 ? -1 : 0);
    }
  } else {
    m.water = true;
  }
  m.nx = s.x + m.dxm;
  m.ny = s.y + m.dym;
  m.inb = m.mv && m.nx >= 0 && m.nx < G && m.ny >= 0 && m.ny < G;  // :193-195
  return m;
}
// (the window coordinates: separate, so that the kernels compute them where they did)
template <bool ONEWORD>
__device__ __forceinline__ void quad_move_cells(QuadMove& m, const Scal& s, int G) {
  m.nyc = m.inb ? m.ny : s.y;
  m.yb = ONEWORD ? 0 : (s.y > 0 ? s.y - 1 : 0);
  m.ybv = s.y > 0 ? s.y - 1 : 0;
  m.cell_o = s.x * G + s.y;
  m.cell_n = m.nx * G + m.nyc;
}

// The compute phase of the sector kernels (pe_step_quad, pe_step_pipe), between the
// window barrier and the done barrier: every wave re-derives the transition
// (plantos_env.py:160-222) from the LDS window, marches its sector of rays and writes
// its part of the env's obs row into the LDS tile; the commit wave (NW-1) stores the
// state.  done / wfix: the env ended this step / its last watering is not stored.
// eo / en / cthr: the explored-bitmap words (F_EXPL_BITMAP) and the CurriculumWrapper
// threshold, loaded by the caller with round 2, or (LX) here by the commit wave in the
// modes that need them -- the persistent kernel keeps other loads in flight here, and
// a wait for a value loaded one iteration earlier is a vmcnt(0).
template <int C, int R, bool ONEWORD, int NW, bool BT, bool RT, bool LX = false, bool DV = false>
__device__ __forceinline__ void quad_compute(const StepArgs& a, const uint64_t* lrow, const uint32_t* lvis,
                                             typename std::conditional<BT, uint8_t, float>::type* rows,
                                             const float* tdist, const float* tpos, const float* tvis, int lane,
                                             int wv, int64_t e, bool live, int Cr, int Rr, const QuadMove& m,
                                             uint32_t eo, uint32_t en, double cthr, uint32_t vp0, Scal& s,
                                             double& ret, bool& done, bool& wfix) {
  using OT = typename std::conditional<BT, uint8_t, float>::type;
  constexpr int LS = kQuadEnvs, CW = NW - 1;
  const Geo& g = a.g;
  // the rules by value: a per-lane choice between two fields of a referenced struct
  // became a per-lane address select and a VMEM load of the chosen double
  const Rules rl = a.rl;
  const State& st = a.st;
  const uint64_t* gb = st.grid + e * g.gstride;
  done = false;
  wfix = false;
  // DV: the previous step's deferred overflow write (pe_device.hpp vx_pending), issued
  // now by wave 0 (not the commit wave, the block's laggard; desynchronized 10.71 ->
  // 10.60 us with the compaction below, profiles/r4ad/): every load the wave waits for
  // has landed at the barrier.  (Ordered before a same-kernel lane-path reset of the env,
  // which uses vx as scratch, by that path's __syncthreads.)
  if constexpr (DV) {
    if (wv == 0 && live && vp0) vx_apply(st, g, e, vp0);
  }
  uint32_t np = 0u;
  s.step = s.step < 65535 ? s.step + 1 : 65535;                  // :162
  bool ok = false, watered = false, wet_hyd = false;
  uint32_t n = 0u;
  int dxv = 0;
  double h = 0.0;
  if (m.mv) {
    const uint64_t rt = lrow[(Rr + 1 + m.dxm) * LS + lane];
    ok = m.inb && ((rt >> (2 * (m.nyc + Rr - m.yb))) & 3u) != OBST;     // :193-195 (plants walkable)
    if (ok) {
      n = (lvis[(3 + m.dxm) * LS + lane] >> (4 * (m.nyc + 2 - m.ybv))) & 15u;
      h = n == 0u ? rl.r_exploration : rl.r_revisit;              // :197, 204-207
      dxv = m.dxm;
    } else {
      s.flags |= F_COLLIDED;                                      // :209
      s.coll = s.coll < 65535 ? s.coll + 1 : 65535;               // :210
      h = rl.r_invalid;                                           // :211
    }
  } else if (m.water) {
    const uint64_t rc = lrow[(Rr + 1) * LS + lane];
    const int cd = (int)((rc >> (2 * (s.y + Rr - m.yb))) & 3u);
    if (cd == THIRSTY) {                                          // fork plantos_env_new.py:237-240
      watered = true;
      h = rl.r_goal;
    } else if (cd == HYD) {                                       // fork :241-242 (root raises)
      wet_hyd = true;
      h = rl.r_mistake;
    } else {
      h = rl.r_water_empty;                                       // :221-222
    }
  }
  const int xp = s.x + dxv, yp = ok ? m.ny : s.y;
  const uint32_t nib = n < 15u ? n + 1u : 15u;                    // :203
  OT* row = rows + lane * g.D;
  if (live) {
    const int kc = dxv + Rr + 1;
    const int sh = 2 * (yp - m.yb);
    const int vs = 4 * (yp - m.ybv);
    if constexpr (RT) {
      // the register-window form where pe_create found the wave's sector fits it (its header's
      // ok word, after the LDS-form table in st.ldxy), else the LDS-table form
      const uint32_t* gt = reinterpret_cast<const uint32_t*>(st.ldxy) + Cr * ((Rr + 7) & ~7);
      const rt_cptr hdr = (rt_cptr)(gt + 4 * wv);
#if PE_RT_REG
      if (hdr[3]) {
        quad_rays_rt_reg<OT>(lrow, hdr, (rt_cptr)(gt + 16), wv * Cr / NW, (wv + 1) * Cr / NW, Rr, lane, kc, sh, watered,
                             row, tdist);
      } else
#endif
      {
        const uint32_t* ltab = reinterpret_cast<const uint32_t*>(reinterpret_cast<const float*>(rows) + quad_rtab_off(Cr, BT));
        quad_rays_rt<OT>(lrow, ltab, wv * Cr / NW, (wv + 1) * Cr / NW, Rr, lane, kc, sh, watered, row, tdist);
      }
    } else {
      sector_rays<C, R, NW>(wv, lrow, lane, kc, sh, watered, row, tdist);
    }
    // slice rows and position go to the non-commit waves (the commit wave is the laggard)
    if (wv != CW)
      for (int lx = wv; lx < 5; lx += NW - 1) quad_slice_row(lvis, lane, lx, dxv, vs, ok, nib, Cr, row, tvis);
    if (wv == (NW == 4 ? 2 : 5)) {                                // :294-296
      if constexpr (BT) {
        row[5 * Cr] = (uint8_t)(kCodePos + xp);
        row[5 * Cr + 1] = (uint8_t)(kCodePos + yp);
      } else {
        row[5 * Cr] = tpos[xp];
        row[5 * Cr + 1] = tpos[yp];
      }
    }
    if (wv == CW) {
      // ---- commit (plantos_env.py:160-222)
      uint32_t wo = eo, wn = en;  // explored-bitmap words after the move (bitmap mode)
      if (ok) {
        if (s.flags & F_EXPL_BITMAP) {                            // explored[old]=1, [new]=2 (:198-200)
          if constexpr (LX) {  // (loaded where used: a copy outside the branch would wait for it)
            eo = st.expl[e * g.estride + (m.cell_o >> 5)];
            en = st.expl[e * g.estride + (m.cell_n >> 5)];
            wo = eo;
            wn = en;
          }
          const uint32_t bo = 1u << (m.cell_o & 31), bn = 1u << (m.cell_n & 31);
          if ((m.cell_o >> 5) == (m.cell_n >> 5)) {
            if (!(wo & bo)) { wo |= bo; s.expl++; }
            if (!(wo & bn)) { wo |= bn; s.expl++; }
          } else {
            if (!(wo & bo)) { wo |= bo; s.expl++; }
            if (!(wn & bn)) { wn |= bn; s.expl++; }
          }
        } else if (n == 0u) {
          s.expl++;  // derived mode: explored[new] was 0 iff never visited
        }
      }
      if (m.bad) {
        s.flags |= F_POISON_ACT;
        atomicOr(st.err_bits, F_POISON_ACT);
      }
      if (wet_hyd && !(s.flags & F_POISON_HYD)) {
        s.flags |= F_POISON_HYD;
        atomicOr(st.err_bits, F_POISON_HYD);
      }
      const int ox = s.x;
      s.x = xp;                                                   // :199
      s.y = yp;
      double rew = rl.r_step;                                     // :164
      rew += h;
      bool term = s.expl >= s.total;                              // :176, 244-246, 331
      const bool trunc = s.step >= rl.max_steps;                  // :177
      if (term && !(s.flags & F_BONUS)) {                         // :179-181
        rew += rl.r_complete;
        s.flags |= F_BONUS;
      }
      if (st.cur) {
        if constexpr (LX) cthr = st.cur[e].thr;  // CurriculumWrapper threshold
        term = curriculum_hit(st.cur, e, cthr, s.expl, s.total, rl.cur_term) || term;  // A2C_training.py:101-103
      }
      done = term || trunc;  // terminal outputs; the reset itself only with autoreset
      // an env about to be auto-reset gets new grid and visit rows: its last move /
      // watering is not stored (the terminal info accounts for the watering), so no
      // store of this step can land after the reset's (unless the curriculum
      // carries the visits over)
      wfix = watered && done && a.autoreset && !st.cur;
      if (!(done && a.autoreset && !st.cur)) {
        if (ok) {
          // the byte holding the target's visit nibble (padded column p), rebuilt from
          // the window of row nx in LDS (padded nibbles ybv..ybv+7 hold both of its
          // nibbles): one byte store, no read of the word from memory
          const int p = m.ny + 2, b = p >> 1;
          const uint32_t wnew = (lvis[(3 + m.dxm) * LS + lane] & ~(0xFu << (4 * (p - m.ybv)))) | (nib << (4 * (p - m.ybv)));
#if defined(PE_PROBE_VISIDLE)  // (timing / traffic probe, wrong results: the byte into the idle slot)
          st_wt(reinterpret_cast<uint8_t*>(vis_env(st, g, e, s.episode ^ 1u) + (int64_t)m.nx * g.NW) + b,
                (uint8_t)(wnew >> (4 * (2 * b - m.ybv))));
#elif defined(PE_VIS_PLAIN)  // (A/B: a write-back byte store, merged into the L2 line round 2 read)
          *(reinterpret_cast<uint8_t*>(vis_env(st, g, e, s.episode) + (int64_t)m.nx * g.NW) + b) =
              (uint8_t)(wnew >> (4 * (2 * b - m.ybv)));
#else
          st_wt(reinterpret_cast<uint8_t*>(vis_env(st, g, e, s.episode) + (int64_t)m.nx * g.NW) + b,
                (uint8_t)(wnew >> (4 * (2 * b - m.ybv))));
#endif
          if constexpr (DV)
            np = vx_pending(m.cell_n, n);
          else
            visit_bump_exact(st, g, e, m.cell_n, n);
          if (s.flags & F_EXPL_BITMAP) {
            uint32_t* ep_o = st.expl + e * g.estride + (m.cell_o >> 5);
            uint32_t* ep_n = st.expl + e * g.estride + (m.cell_n >> 5);
            if (wo != eo) *ep_o = wo;
            if ((m.cell_o >> 5) != (m.cell_n >> 5) && wn != en) *ep_n = wn;
          }
        }
        if (watered) {
          const int bit = 2 * (s.y + Rr);
          if constexpr (ONEWORD) {
            st_wt(const_cast<uint64_t*>(gb) + ox, (uint64_t)(lrow[(Rr + 1) * LS + lane] & ~(1ull << bit)));  // code 3 -> 2
          } else {
            // the byte holding the cell's code (padded column c; its 4 cells lie in the
            // window of row x, padded columns yb..yb+31, for R >= 2)
            const int c = s.y + Rr, B = c >> 2;
            const uint64_t wr = lrow[(Rr + 1) * LS + lane] & ~(1ull << (2 * (c - m.yb)));  // code 3 -> 2
            st_wt(reinterpret_cast<uint8_t*>(const_cast<uint64_t*>(gb) + (int64_t)ox * g.WPR) + B,
                  (uint8_t)(wr >> (2 * (4 * B - m.yb))));
          }
        }
      }
      ret += rew;
#if !defined(PE_PROBE_NOOUT)
      st_wt(a.reward + e, (float)rew);
      st_wt(a.term + e, (uint8_t)term);
      st_wt(a.trunc + e, (uint8_t)trunc);
#endif
      if (done) {  // Monitor's episode return / length of the ended episode
        if (a.ep_ret_out) st_wt(a.ep_ret_out + e, ret);
        if (a.ep_len_out) st_wt(a.ep_len_out + e, (int32_t)s.step);
      }
      // an env about to be auto-reset: its reset path stores the new episode's scalars
#if !defined(PE_PROBE_NOSCAL)
      if (!(done && a.autoreset && !st.cur)) {
        st_wt(st.ep_ret + e, ret);
        st_wt(st.scal + e, pack(s));
      }
#endif
      if constexpr (DV) {
        if (vp0 | np) st_wt(st.vpend + e, np);
      }
    }
  }
}

// BT: byte-coded obs tile (pe_coop.hpp ObsW<uint8_t>): [64 x D] bytes instead of
// floats in LDS (64x64 / 64 rays: 22 KB instead of 89 KB), expanded through the LDS
// code table at the tile store -- the f32 tile held the kernel to one workgroup per CU.
// EPB: envs per workgroup (64; 16 / 32 for small batches: more workgroups, so that
// a batch of a few thousand envs spreads over every CU -- lanes >= EPB idle).  The
// LDS layout keeps the 64-env stride LS whatever EPB.
// GR2 (round 6): two-word rows (WPR == 2) of a grid small enough (G <= kGr2MaxG: 25x25, the
// training scripts' grid) that the loader env's whole block comes in round 1, as the one-word
// kernel's (kGridR1): round 2 then holds only the visit rows.
constexpr int kGr2MaxG = 28;
template <int C, int R, bool ONEWORD, int NW, bool BT = false, int EPB = kQuadEnvs, bool GR2 = false>
__global__ __launch_bounds__(64 * NW, NW == 8 ? (EPB < kQuadEnvs ? 2 : 8) : 4) void pe_step_quad(StepArgs a) {  // NW=8: <= 80 SGPRs (small-batch EPB: one workgroup per CU, no cap); NW=4: <= 128 VGPRs (4 workgroups per CU: G=25 13.1 -> 10.5 us; 1-word C16: 122 -> 104 VGPRs)
  // C == 0 (R == 0): the runtime-(C, R) sector kernel (quad_rays_rt): C, R from the
  // geometry (up to kRtCMax -- kRtCMaxBT with the byte-coded tile -- / kRtRMax), the LDS
  // layout sized at run time
  constexpr bool RT = C == 0;
  constexpr int CM = RT ? (BT ? kRtCMaxBT : kRtCMax) : C, RM = RT ? kRtRMax : R;
  static_assert(!RT || (R == 0 && NW == 4 && EPB == kQuadEnvs), "runtime sector kernel: 4 waves, 64 envs");
  const int Cr = RT ? a.g.C : C, Rr = RT ? a.g.R : R;
  constexpr int NR = 2 * RM + 3, NV = 7, LS = kQuadEnvs, CW = NW - 1;  // CW: commit wave
  const int NRL = RT ? 2 * Rr + 3 : NR;  // window rows (the LDS layout's)
  const int tile_off = RT ? quad_tile_off_rt(Rr) : quad_tile_off<RM>();
  // after the tile (+ code table): RT's probe table (quad_rtab_off), then the staging region
  const int tail_off = tile_off + quad_rtab_off(Cr, BT);
  static_assert(EPB == 16 || EPB == 32 || EPB == 64, "envs per workgroup");
  static_assert(!BT || EPB == kQuadEnvs, "the byte-coded kernel's LDS-DMA staging predicts over all 64 lanes");

  static_assert(RT || C >= NW, "every wave owns a sector of at least one ray");
  static_assert(ONEWORD || RM <= 14, "funnel-shifted window row must hold 2R+5 cells");
  static_assert(ONEWORD || RT || R >= 2, "the watered cell's byte must lie in the window row");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tdist = smem;
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  uint64_t* lrow = reinterpret_cast<uint64_t*>(smem + kTabFloats);  // [NR][LS]
  uint32_t* lvis = reinterpret_cast<uint32_t*>(lrow + NRL * LS);   // [NV][LS]
  using OT = typename std::conditional<BT, uint8_t, float>::type;
  OT* rows = reinterpret_cast<OT*>(smem + tile_off);                // [LS][D] floats or codes
  float* ctab = smem + (RT ? quad_ctab_off_rt(Rr, Cr) : quad_ctab_off<RM, CM>());  // BT: code -> float
  const Geo& g = a.g;
  const Rules& rl = a.rl;
  const State& st = a.st;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t e0 = (int64_t)blockIdx.x * EPB;
  const int64_t e = e0 + lane;
  const bool live = (EPB == LS || lane < EPB) && e < a.n;

  // ---- round 1: env-indexed loads (all waves).  Every thread also plays a LOADER
  // role for round 2: LT = 64 NW / EPB threads per env (env le < EPB, part sub), so
  // each load instruction reads LT consecutive rows of 64/LT envs instead of one row of 64.
  PE_STAMP(0);
  if (a.stagger) {  // de-phase the resident workgroups of a CU (speed only)
    const int q = (int)(blockIdx.x * PE_STAGGER_GROUPS / gridDim.x);
    for (int i = 0; i < q * a.stagger; ++i) __builtin_amdgcn_s_sleep(8);
  }
  constexpr int LT = NW * (LS / EPB);
  const int le = threadIdx.x / LT, sub = threadIdx.x % LT;
  const int64_t el = e0 + le;
  const bool llive = el < a.n;
  // Every round-1 load unconditional (indices clamped into the batch; the values of
  // lanes past its end are never used): a load inside a branch whose value merges
  // after it is waited for right there -- the 4-byte action load used to be, before
  // the loader scalars were even issued, i.e. two memory round trips instead of one.
  const int64_t ec = live ? e : (int64_t)a.n - 1, elc = llive ? el : (int64_t)a.n - 1;
  const uint4 sw = st.scal[ec];
  const int ash = a.act_bytes == 8 ? 1 : 0;  // 8-byte actions: two words, low first
  const int32_t* ap = reinterpret_cast<const int32_t*>(a.actions);
  const int32_t alo = ap[ec << ash], ahi = ap[(ec << ash) + ash];
  double ret = st.ep_ret[wv == CW ? ec : 0];  // (the commit wave's; the others read one shared word)
  // the deferred overflow write (pe_device.hpp vx_pending): the headline instantiation
  // only -- measured faster there (9.66 -> 9.52 us), slower in the constructor default's
  // multi-word C10R2 kernel (8.22 -> 8.69) and the 16-env small-batch shape (4.44 -> 4.61),
  // profiles/r4q/, r4v/
  // (round 5: the byte-coded twin of the headline kernel too -- config 5's codes step, A/B
  // PE_BT_DV=0)
  constexpr bool DV = C == 16 && R == 6 && ONEWORD && NW == 4 && (PE_BT_DV || !BT) && EPB == kQuadEnvs;
  const uint32_t vp0 = DV ? st.vpend[wv == CW || wv == 0 ? ec : 0] : 0u;  // (wave 0 applies, CW stores)
  // (Tried: the loader env's position by a bpermute from lane le of the wave instead of
  // this load -- 64x64 24.5 -> 25.2 us, 25x25 desync +0.4 us, the headline unchanged;
  // profiles/r3m_ab_*.jsonl.)
  const uint4 lw = st.scal[elc];
  // one-word rows (G <= 20): the loader env's whole grid block (gstride / 2 <= 10
  // 16-B units, contiguous, 3 per loader thread) comes in round 1 -- its address does
  // not depend on the position -- and only the visit rows are left for round 2
  static_assert(!GR2 || (!ONEWORD && !RT && NW == 4 && EPB == kQuadEnvs), "GR2: the two-word 64-env kernel");
  constexpr int JG1 = GR2 ? (kGr2MaxG + LT - 1) / LT : (10 + LT - 1) / LT;  // gstride / 2 <= 10 16-B units (one-word:
                                                                            // NW == 4, G <= 20); GR2: G <= kGr2MaxG rows
  constexpr bool kGridR1 = (ONEWORD && PE_GRID_R1) || GR2;
  uint4 qg1[kGridR1 ? JG1 : 1];
  if constexpr (kGridR1) {
    const uint4* lgq = reinterpret_cast<const uint4*>(st.grid + elc * g.gstride);
    const int nq = (int)(g.gstride >> 1);
#pragma unroll
    for (int j = 0; j < JG1; ++j) {
      const int q = sub + LT * j;
      qg1[j] = lgq[q < nq ? q : nq - 1];
    }
  }
  load_tables_hot(smem, st.tab, a.g.G, Rr);
  // the sector rays' tables (pe_quad.hpp quad_rays): dist[R+1] = 1.0, one-hot rows
  static_assert(RM + 2 <= kOneHotF && kOneHotF + 16 <= 70, "ray tables inside dist[], below the done mask");
  if (threadIdx.x < 16) smem[kOneHotF + threadIdx.x] = (threadIdx.x >> 2) == (threadIdx.x & 3) ? 1.0f : 0.0f;
  if (threadIdx.x == 16) smem[Rr + 1] = 1.0f;

  if constexpr (RT) {  // the probe table (st.ldxy) into LDS: read from global memory in the ray
                       // loop, each 8-probe chunk was a vector load waited out with vmcnt(0)
    // (the LDS form's table: the sectors the register window does not take; round 6: the
    // copy's loads issued with round 1's, one unit per thread, measured slower -- 32x32/C24/R9
    // 17.05 -> 17.39 us, 40x40/C48/R8 28.57 -> 29.1, profiles/r6c/)
    const uint4* src = reinterpret_cast<const uint4*>(st.ldxy);
    uint4* dst = reinterpret_cast<uint4*>(smem + tail_off);
    for (int k = threadIdx.x; k < Cr * ((Rr + 7) & ~7) / 4; k += blockDim.x) dst[k] = src[k];  // (u32 entries)
  }
  Scal s = unpack(sw);
#ifdef PE_STAMPS
  if ((int)(s.x + lw.x) == -12345) g_stamps[0] = 1;  // consume round 1 before the stamp
#endif
  PE_STAMP(1);
  const int64_t action = ash ? (int64_t)(((uint64_t)(uint32_t)ahi << 32) | (uint32_t)alo) : (int64_t)alo;
  QuadMove m = quad_move<ONEWORD>(s, action, g.G);
  // A block whose only env to truncate this step is known from its step count
  // (:177, the steady state of desynchronized episodes: ~6 % of the blocks each
  // step): that env's prefetched record -- and, small grids, its current rows for the
  // terminal info -- go into LDS by LDS-DMA now, in the same round trip as round 2,
  // so its auto-reset (quad_done_path) makes no memory round trip of its own
  // (pe_coop.hpp pf_stage_issue; the LDS-DMA needs no VGPRs).  A termination is not
  // predictable: a block with one then takes the unstaged path.  Byte-coded kernels
  // only (64x64 desynchronized: 36.6 -> 36.2 us): at 20x20 the waits hipcc places
  // around a possibly outstanding LDS-DMA (a vmcnt(0) at the next use of any load
  // result) serialize round 2 in every block (9.39 -> 10.0 us, desync 11.52 -> 12.29).
  float* stage = smem + tail_off + (RT ? quad_rtab_floats(Cr, Rr) : 0);
  // (C >= PE_BT_STAGE_MIN_C only: the byte-coded C16 kernel -- config 5's codes step --
  // pays the same round-2 serialization as the f32 one would)
  const bool stage_ok = BT && CM >= PE_BT_STAGE_MIN_C && a.pf.scal && quad_coop(a, 1) &&
                        e0 + EPB <= a.n;  // full block: every lane live
  const bool stage_info = !st.cur && a.tinfo && pf_stage_info_fits(g.G, g.WPR, (int)a.pf.ostride);
  // (issued right after round 2's own loads: hipcc drains every memory op in flight
  // before the first use of a load result while an LDS-DMA is outstanding, so issued
  // earlier it would put a round trip of its own ahead of round 2)
  int npred = 0;
  uint64_t pm = 0ull;
  if (stage_ok) {
    pm = __ballot(s.step + 1 >= rl.max_steps);
    npred = __popcll(pm);
  }
  // (round 6) the env's current grid rows for its terminal info, when they do not fit the
  // record's LDS-DMA instructions (64x64, the runtime kernel's larger grids): register-staged
  // by the info wave (two 16-B units per lane) into the staging region after the record,
  // so that the info wave writes the terminal info beside the commit wave's reset instead
  // of the commit wave loading them after the done barrier (a round trip on its path)
  const int ng_s = pf_grid_units(g.G, g.WPR);
  const bool info_reg = BT && PE_BT_INFO_REG && stage_ok && !stage_info && !st.cur && a.tinfo != nullptr && ng_s <= 128;
  uint4 iq0 = make_uint4(0u, 0u, 0u, 0u), iq1 = iq0;
  auto stage_issue = [&]() {
    if (BT && wv == CW && npred == 1)
      pf_stage_issue(a.pf, st, g, e0 + (__ffsll((unsigned long long)pm) - 1), stage, lane, stage_info);
    if (BT && info_reg && wv == kQuadInfoWave && npred == 1) {
      const uint4* src = reinterpret_cast<const uint4*>(st.grid + (e0 + (__ffsll((unsigned long long)pm) - 1)) * g.gstride);
      iq0 = src[lane < ng_s ? lane : ng_s - 1];
      iq1 = src[lane + 64 < ng_s ? lane + 64 : ng_s - 1];
    }
  };
  quad_move_cells<ONEWORD>(m, s, g.G);

  // Early record (one-word 64-env kernels): a block whose ONLY env to truncate this
  // step is known from its step count (:177; ~6 % of the blocks of a desynchronized
  // batch each step) has the commit wave load that env's prefetched record and its
  // grid rows (the terminal info) right before round 2's loads -- they land with them,
  // and the barrier after round 2 has waited for them -- so its auto-reset makes no
  // memory round trip of its own (quad_done_path).  Issued behind the compute phase
  // instead, the done path's first use waited for the commit's stores too (vmcnt
  // counts both, in order).  (The byte-coded kernel stages the same record by
  // LDS-DMA during round 2.)
  constexpr int KDQ = (5 * CM + 27 + 63) / 64, MAXWQ = ONEWORD ? 1 : kCoopWPR;
  // (one-word 64-env kernels only: the multi-word kernel is at its 128-VGPR cap and
  // spilled with it -- 25x25 desynchronized 14.0 -> 14.6 us -- and the 16-env shape of
  // small batches lost 2-5 % synchronized; profiles/r3c_ab_early_*.jsonl)
  // (round 5: the byte-coded one-word kernel too -- config 5's codes step; the record's
  // codes come in as 4-code words; A/B: -DPE_BT_EARLY=0)
  constexpr bool kEarlyRec = (!BT || PE_BT_EARLY) && ONEWORD && EPB == LS && KDQ <= 2;
  PfLoad<MAXWQ, KDQ> epl;
  Row4<MAXWQ> eir;
  int64_t e_early = -1, e_info = -1;
  constexpr bool kInfoW = kEarlyRec && PE_INFO_WAVE && NW == 4;
  static_assert(!kInfoW || (RM + 2 <= kInfoParkF && kInfoParkF + 5 <= kOneHotF), "info park words inside dist[]");
  if constexpr (kEarlyRec) {
    // (the commit wave only, for a block with exactly one: records for up to one
    // predicted env per wave took the desynchronized step 11.16 -> 11.06 us but the
    // synchronized one 9.42 -> 9.49, profiles/r3g_ab_*.jsonl; round 5: the env's rows
    // for its terminal info by the info wave)
    // (round 6, kEarly2: a block with exactly TWO predicted truncations -- ~2 of the 1024
    // blocks of a desynchronized 65536-env step, which the one-done blocks' early record left
    // as the step's last blocks -- has waves 0 and 1 load one env's record and rows each:
    // the cooperative path hands the k-th done env to wave k, so each finds its own)
    constexpr bool kEarly2 = PE_EARLY2 && NW == 4;
    if ((wv == CW || (kInfoW && wv == kQuadInfoWave) || (kEarly2 && wv < 2)) && a.pf.scal && a.autoreset && !st.cur) {
      const uint64_t pmk = __ballot(live && s.step + 1 >= rl.max_steps);
      const uint32_t plo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pmk),
                     phi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pmk >> 32));
      const uint64_t pmu = (uint64_t)plo | ((uint64_t)phi << 32);
      const int npk = __popcll(pmu);
      if (kEarly2 && npk == 2 && wv < 2) {
        const uint64_t lowb = pmu & (0ull - pmu);
        const int64_t ep = e0 + (__ffsll((unsigned long long)(wv == 0 ? lowb : (pmu ^ lowb))) - 1);
        e_early = ep;
        e_info = ep;
        coop_load_prefetched<MAXWQ, KDQ, OT>(a.pf, g, ep, epl, lane);
        eir = coop_info_rows<MAXWQ>(st, g, ep, lane);
      } else if (npk == 1 && wv >= 2) {
        const int64_t ep = e0 + (__ffsll((unsigned long long)pmu) - 1);
        if (wv == CW) {
          e_early = ep;
          coop_load_prefetched<MAXWQ, KDQ, OT>(a.pf, g, e_early, epl, lane);
          if constexpr (!kInfoW) eir = coop_info_rows<MAXWQ>(st, g, e_early, lane);
        } else {
          e_info = ep;
          eir = coop_info_rows<MAXWQ>(st, g, e_info, lane);
        }
      }
    }
  }
  // Register-staged record (round 6; the f32 kernels that have neither the early record
  // nor LDS-DMA staging: the multi-word rows -- 25x25, 21x21 -- the runtime-(C, R) f32
  // kernel and the 16 / 32-env small-batch shapes).  A block whose ONLY env to truncate
  // this step is known from its step count (:177) has the commit wave load that env's
  // prefetched record -- scalars, grid rows, obs row: one 16-B unit per lane, the layout
  // of pf_stage_issue -- and the info wave the env's current grid rows, right after round
  // 2's loads; both are written into the LDS staging region after round 2's LDS writes,
  // so they hold 4 VGPRs through round 2 only (the early record's registers live across
  // the compute phase spilled the multi-word kernel, at its 128-VGPR cap), and the single-
  // done path makes no memory round trip: the commit wave takes the staged record, the
  // info wave writes the terminal info from the staged rows beside it.
  // (not the 16 / 32-env small-batch shapes: 4096 envs synchronized 4.43 -> 4.62 us for
  // desynchronized 6.38 -> 6.30, profiles/r6c/)
  constexpr bool kRegStage =
      PE_REG_STAGE && !kEarlyRec && !BT && NW > kQuadInfoWave && (EPB == kQuadEnvs || PE_REG_STAGE_SMALL);
  // (the staging outcome goes to LDS -- kRsFlagF, written by the commit wave every launch --
  // and the done env's scalars are parked after the compute phase: no SGPRs live across it)
  constexpr int kRsFlagF = kInfoParkF + 5;
  static_assert(!(kRegStage || BT) || (RM + 2 <= kInfoParkF && kRsFlagF + 1 <= kOneHotF), "info park words inside dist[]");
  bool rs_on = false, rs_info = false;  // (wave-uniform; identical in the commit and the info wave)
  int64_t e_rs = -1;
  uint4 rq = make_uint4(0u, 0u, 0u, 0u);
  int rs_u = 0, rs_n = 0;  // this lane's staging unit, the wave's unit count
  if constexpr (kRegStage) {
    if ((wv == CW || wv == kQuadInfoWave) && a.pf.scal && a.autoreset && !st.cur && quad_coop(a, 1)) {
      const uint64_t pmk = __ballot(live && s.step + 1 >= rl.max_steps);
      const uint64_t pmu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pmk) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pmk >> 32)) << 32);
      const int ng = pf_grid_units(g.G, g.WPR), no = (int)a.pf.ostride / 16;
      if (__popcll(pmu) == 1 && 1 + ng + no <= 64) {
        rs_on = true;
        rs_info = a.tinfo != nullptr;
        e_rs = e0 + (__ffsll((unsigned long long)pmu) - 1);
        rs_n = wv == CW ? 1 + ng + no : (rs_info ? ng : 0);
        rs_u = (wv == CW ? 0 : 1 + ng + no) + (lane < rs_n ? lane : rs_n - 1);
      }
    }
  }
  auto rs_issue = [&]() {
    if (kRegStage && rs_n > 0) {
      const int ng = pf_grid_units(g.G, g.WPR);
      const int u = rs_u;
      const uint4* src;
      if (wv == CW)
        src = u == 0 ? reinterpret_cast<const uint4*>(a.pf.scal + e_rs)
                     : (u <= ng ? reinterpret_cast<const uint4*>(a.pf.grid + e_rs * g.gstride) + (u - 1)
                                : reinterpret_cast<const uint4*>(pf_obs_row(a.pf, e_rs)) + (u - 1 - ng));
      else
        src = reinterpret_cast<const uint4*>(st.grid + e_rs * g.gstride) + (u - (1 + ng + (int)a.pf.ostride / 16));
      rq = *src;
    }
  };
  // ---- round 2: window rows of env le -> LDS [row][env] (loader role)
  uint32_t eo = 0u, en = 0u;
  if (llive) {
    const int lx = (int)(lw.x & 0xFF), ly = (int)((lw.x >> 8) & 0xFF);
    const uint64_t* lgb = st.grid + el * g.gstride;
    const int base = lx - Rr - 1;  // grid row of LDS row 0
    // Every load first, then the LDS writes: the loads are unconditional (row
    // indices clamped into the map, off-map rows selected away afterwards), so the
    // compiler issues all of them back to back and waits once -- with the range
    // tests around the loads it waited after each (one memory round trip per row).
    if constexpr (ONEWORD) {
      // row pairs (16 B, aligned: env blocks are 16-B aligned, pairs start on even rows)
      const int ps = base & ~1;
      constexpr int NP = (NR + 2) / 2, JG = kGridR1 ? 1 : (NP + LT - 1) / LT, JV = (NV + LT - 1) / LT;
      const int gmax = g.G - 2 > 0 ? g.G - 2 : 0;
      uint4 qg[JG], qv[JV];
      if constexpr (!kGridR1) {
#pragma unroll
        for (int j = 0; j < JG; ++j) {
          const int ra = ps + 2 * (sub + LT * j);
          const int rc = ra < 0 ? 0 : (ra > gmax ? gmax : ra);
          qg[j] = *reinterpret_cast<const uint4*>(lgb + rc);
        }
      }
      const uint32_t* lvb = vis_env(st, g, el, lw.w);  // (lw.w: the loader env's episode)
      {
#pragma unroll
        for (int j = 0; j < JV; ++j) {
          const int kk = sub + LT * j;
          const int xr = lx - 3 + kk;
          const int xc = xr < 0 ? 0 : (xr >= g.G ? g.G - 1 : xr);
          qv[j] = *reinterpret_cast<const uint4*>(lvb + (int64_t)xc * 4);  // g.NW == 4
        }
      }
      stage_issue();
      rs_issue();  // (after round 2's loads: their waits stay as they were)
      if constexpr (kGridR1) {
        // the block's rows (pairs 2q, 2q+1) inside the window, then the off-map rows
        const int nq = (int)(g.gstride >> 1);
#pragma unroll
        for (int j = 0; j < JG1; ++j) {
          const int q = sub + LT * j, ka = 2 * q - base;
          if (q < nq) {
            const uint64_t lo = (uint64_t)qg1[j].x | ((uint64_t)qg1[j].y << 32);
            const uint64_t hi = (uint64_t)qg1[j].z | ((uint64_t)qg1[j].w << 32);
            if (ka >= 0 && ka < NRL) lrow[ka * LS + le] = lo;
            if (ka + 1 >= 0 && ka + 1 < NRL && 2 * q + 1 < g.G) lrow[(ka + 1) * LS + le] = hi;
          }
        }
#pragma unroll
        for (int j = 0; j < (NR + LT - 1) / LT; ++j) {
          const int k = sub + LT * j, xr = base + k;
          if (k < NRL && (xr < 0 || xr >= g.G)) lrow[k * LS + le] = kEven64;  // off-map rows: obstacles
        }
      }
#pragma unroll
      for (int j = 0; j < JG; ++j) {
        const int pp = sub + LT * j;
        if (!kGridR1 && pp < NP) {
          const int ra = ps + 2 * pp;
          const int rc = ra < 0 ? 0 : (ra > gmax ? gmax : ra);
          const uint64_t lo = (uint64_t)qg[j].x | ((uint64_t)qg[j].y << 32);
          const uint64_t hi = (uint64_t)qg[j].z | ((uint64_t)qg[j].w << 32);
          // off-map rows: obstacles
          const uint64_t va = (ra >= 0 && ra < g.G) ? (ra == rc ? lo : hi) : kEven64;
          const uint64_t vb2 = (ra + 1 >= 0 && ra + 1 < g.G) ? (ra + 1 == rc ? lo : hi) : kEven64;
          const int ka = ra - base;
          if (ka >= 0 && ka < NRL) lrow[ka * LS + le] = va;
          if (ka + 1 >= 0 && ka + 1 < NRL) lrow[(ka + 1) * LS + le] = vb2;
        }
      }
      // visit rows: one 16-B row per load, funnel-shifted to ybv
      const int lybv = ly > 0 ? ly - 1 : 0;
      const int vw = (4 * lybv) >> 5, vo = (4 * lybv) & 31;
#pragma unroll
      for (int j = 0; j < JV; ++j) {
        const int k = sub + LT * j;
        if (k < NV) {
          const int xr = lx - 3 + k;
          uint32_t lo = 0xAAAAAAAAu, hi = 0xAAAAAAAAu;  // off-map row: visit 10 (reads 1.0)
          if (xr >= 0 && xr < g.G) {
            const uint4 q = qv[j];
            lo = vw == 0 ? q.x : (vw == 1 ? q.y : q.z);
            hi = vw == 0 ? q.y : (vw == 1 ? q.z : q.w);
          }
          lvis[k * LS + le] = vo ? ((lo >> vo) | (hi << (32 - vo))) : lo;
        }
      }
    } else {
      const int lyb = ly > 0 ? ly - 1 : 0;
      const int w0 = (2 * lyb) >> 6, o = (2 * lyb) & 63;
      const int w1 = w0 + 1 < g.WPR ? w0 + 1 : w0;  // in bounds; its word is dropped when w0 is the last
      constexpr int JG = GR2 ? 1 : (NR + LT - 1) / LT, JV = (NV + LT - 1) / LT;
      uint64_t glo[JG], ghi[JG];
      uint32_t vlo[JV], vhi[JV];
      if constexpr (GR2) {
        // (the rows came with round 1: qg1, unit q = grid row q)
      } else if (g.WPR == 2) {  // (G <= 52, e.g. the training scripts' 25x25) a row is one aligned 16-B load
#pragma unroll
        for (int j = 0; j < JG; ++j) {
          const int xr = base + sub + LT * j;
          const int xc = xr < 0 ? 0 : (xr >= g.G ? g.G - 1 : xr);
          const uint4 q = *reinterpret_cast<const uint4*>(lgb + (int64_t)xc * 2);
          const uint64_t lo64 = (uint64_t)q.x | ((uint64_t)q.y << 32), hi64 = (uint64_t)q.z | ((uint64_t)q.w << 32);
          glo[j] = w0 ? hi64 : lo64;
          ghi[j] = hi64;
        }
      } else {
#pragma unroll
        for (int j = 0; j < JG; ++j) {
          const int xr = base + sub + LT * j;
          const int xc = xr < 0 ? 0 : (xr >= g.G ? g.G - 1 : xr);
          const uint64_t* p = lgb + (int64_t)xc * g.WPR;
          glo[j] = p[w0];
          ghi[j] = p[w1];
        }
      }
      const int lybv = ly > 0 ? ly - 1 : 0;
      const int vw = (4 * lybv) >> 5, vo = (4 * lybv) & 31;
      const uint32_t* vb = vis_env(st, g, el, lw.w) + vw;
#pragma unroll
      for (int j = 0; j < JV; ++j) {
        const int xr = lx - 3 + sub + LT * j;
        const int xc = xr < 0 ? 0 : (xr >= g.G ? g.G - 1 : xr);
        vlo[j] = vb[(int64_t)xc * g.NW];
        vhi[j] = vb[(int64_t)xc * g.NW + 1];  // vw + 1 < NW always (one spare word per row)
      }
      stage_issue();
      rs_issue();  // (after round 2's loads: their waits stay as they were)
      if constexpr (GR2) {
        // the loader env's rows inside the window, funnel-shifted to padded column yb, then
        // the off-map rows (obstacles)
#pragma unroll
        for (int j = 0; j < JG1; ++j) {
          const int q = sub + LT * j, k = q - base;
          if (q < g.G && k >= 0 && k < NRL) {
            const uint64_t lo64 = (uint64_t)qg1[j].x | ((uint64_t)qg1[j].y << 32);
            const uint64_t hi64 = (uint64_t)qg1[j].z | ((uint64_t)qg1[j].w << 32);
            const uint64_t lo = w0 ? hi64 : lo64, hi = w0 ? 0ull : hi64;
            lrow[k * LS + le] = o ? ((lo >> o) | (hi << (64 - o))) : lo;
          }
        }
#pragma unroll
        for (int j = 0; j < (NR + LT - 1) / LT; ++j) {
          const int k = sub + LT * j, xr = base + k;
          if (k < NRL && (xr < 0 || xr >= g.G)) lrow[k * LS + le] = kEven64;  // off-map rows: obstacles
        }
      }
#pragma unroll
      for (int j = 0; j < JG; ++j) {
        const int k = sub + LT * j;
        if (!GR2 && k < NRL) {
          const int xr = base + k;
          uint64_t v = kEven64;  // off-map rows read as obstacles
          if (xr >= 0 && xr < g.G) {
            const uint64_t hi = w0 + 1 < g.WPR ? ghi[j] : 0ull;
            v = o ? ((glo[j] >> o) | (hi << (64 - o))) : glo[j];
          }
          lrow[k * LS + le] = v;
        }
      }
#pragma unroll
      for (int j = 0; j < JV; ++j) {
        const int k = sub + LT * j;
        if (k < NV) {
          const int xr = lx - 3 + k;
          uint32_t lo = 0xAAAAAAAAu, hi = 0xAAAAAAAAu;
          if (xr >= 0 && xr < g.G) {
            lo = vlo[j];
            hi = vhi[j];
          }
          lvis[k * LS + le] = vo ? ((lo >> vo) | (hi << (32 - vo))) : lo;
        }
      }
    }
  } else {
    rs_issue();  // (a lane whose loader env is past the batch end: its staging unit all the same)
  }
  // the register-staged units into the LDS staging region (after round 2's LDS writes:
  // the wait for them is the last of the round)
  if (kRegStage && rs_n > 0 && lane < rs_n) reinterpret_cast<uint4*>(stage)[rs_u] = rq;
  if (kRegStage && wv == CW && lane == 0) smem[kRsFlagF] = __int_as_float((int)rs_on | ((int)rs_info << 1));
  if (BT && info_reg && wv == kQuadInfoWave && npred == 1) {
    uint4* d = reinterpret_cast<uint4*>(stage) + 1 + ng_s + (int)a.pf.ostride / 16;
    if (lane < ng_s) d[lane] = iq0;
    if (lane + 64 < ng_s) d[lane + 64] = iq1;
  }
  // what the state commit needs beyond the window rows (lane = env): only in the
  // curriculum / injected-state modes (the visit and grid words it rewrites are
  // rebuilt from the window rows, see the commit)
  double cthr = 0.0;
  if (live && wv == CW) {
    if (st.cur) cthr = st.cur[e].thr;  // CurriculumWrapper threshold
    if (m.inb && (s.flags & F_EXPL_BITMAP)) {
      eo = st.expl[e * g.estride + (m.cell_o >> 5)];
      en = st.expl[e * g.estride + (m.cell_n >> 5)];
    }
  }
#ifdef PE_STAMPS
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
  // the commit wave's early record landed with round 2: a wait the compiler tracks
  // (not asm), so that the done path's first use of it carries none -- otherwise it
  // waits vmcnt(0) there, i.e. for the commit's stores too (in-order counter)
  if constexpr (kEarlyRec) {
    if (wv == CW || (kInfoW && wv == kQuadInfoWave) || (PE_EARLY2 && NW == 4 && wv < 2))
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  PE_STAMP(2);
  __syncthreads();
  PE_STAMP(3);

  // ---- transition from LDS (every wave; wave 0 commits)
  // the commit wave is the block's laggard through this phase (its state stores come
  // on top of its sector): issue priority until the done barrier (same-box A/B: 9.73
  // -> 9.65 us synchronized, 12.88 -> 12.43 us desynchronized; for the whole kernel
  // it slowed the synchronized step)
  if (wv == CW) __builtin_amdgcn_s_setprio(2);
  // BT: the LDS code table from the LDS tables (complete at the barrier above; read after the
  // done barrier).  It was a per-code if-chain of global loads in round 1, each waited out
  // at once (three dependent round trips), then the candidate loads issued with round 1
  // (profiles/r5s/ab_code_table_*.txt)
  if constexpr (BT) {
    if (threadIdx.x < 256) ctab_from_lds(smem, ctab, Rr, g.G, (int)threadIdx.x, kOneHotF + 1);
  }
  // (Tried: the early record's state writes issued here, at the start of the compute
  // phase, instead of in the done path: the commit wave then waited for them before
  // re-using their data registers -- desynchronized 11.12 -> 12.05 us, synchronized
  // 9.47 -> 9.59; profiles/r3i_ab_*.jsonl.)
  bool done = false, wfix = false;
  quad_compute<C, R, ONEWORD, NW, BT, RT, false, DV>(a, lrow, lvis, rows, tdist, tpos, tvis, lane, wv, e, live, Cr,
                                                     Rr, m, eo, en, cthr, vp0, s, ret, done, wfix);
  if constexpr (kInfoW) {  // the early env's post-step scalars for the info wave (read after the done barrier)
    if (wv == CW && e_early >= 0 && e == e_early) {
      const uint4 pk = pack(s);
      smem[kInfoParkF] = __int_as_float((int)pk.x);
      smem[kInfoParkF + 1] = __int_as_float((int)pk.y);
      smem[kInfoParkF + 2] = __int_as_float((int)pk.z);
      smem[kInfoParkF + 3] = __int_as_float((int)pk.w);
      smem[kInfoParkF + 4] = __int_as_float((int)wfix);
    }
  }
  if constexpr (kRegStage || (BT && !kEarlyRec && NW > kQuadInfoWave)) {  // a block's one done env's post-step
                                                                           // scalars for the info wave (as kInfoW)
    if (wv == CW) {
      const uint64_t dm1 = __ballot(done);
      if (__popcll(dm1) == 1 && done) {
        const uint4 pk = pack(s);
        smem[kInfoParkF] = __int_as_float((int)pk.x);
        smem[kInfoParkF + 1] = __int_as_float((int)pk.y);
        smem[kInfoParkF + 2] = __int_as_float((int)pk.z);
        smem[kInfoParkF + 3] = __int_as_float((int)pk.w);
        smem[kInfoParkF + 4] = __int_as_float((int)wfix);
      }
    }
  }
  PE_STAMP(4);
  // ---- DummyVecEnv auto-reset (rare): commit wave, after the whole obs row is in LDS
  // any env of the block done (the usual answer: no)?  The commit wave's done mask
  // goes to an unused LDS table word (dist[70..71]) for the count the reset path needs.
  static_assert(RM < 70, "dist[70..71] holds the done mask");
  if (wv == CW) {
    const uint64_t dm = __ballot(done);
    if (lane == 0) reinterpret_cast<uint64_t*>(smem)[35] = dm;
  }
  // The block barrier (obs rows and the done mask complete in LDS) WITHOUT a memory
  // fence: __syncthreads() would make the commit wave wait for its state stores to
  // land first (s_waitcnt vmcnt(0)), although nothing in this launch reads them
  // back -- the reset path orders its own accesses (see quad_done_path).
  if (wv == CW) __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const uint64_t dmask = reinterpret_cast<const uint64_t*>(smem)[35];  // after the asm barrier ("memory")
  const uint64_t dmu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dmask) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(dmask >> 32)) << 32);
  const bool any_done = dmu != 0ull;
  const int ndone = __popcll(dmu);
  // (Tried: a single-done fast path -- the early record checked before the done barrier,
  // no barrier after the reset, the commit wave storing its env's chunks of the tile and
  // the other waves the rest at once: desync 11.14 -> 11.38 us, synchronized 9.46 -> 9.60;
  // profiles/r3n_ab_*.jsonl.)
  PE_STAMP(5);
  // auto-reset slow path, out of line (its registers stay off the hot path)
  // (RT: the region is sized by the actual R -- pe_create checks these at run time)
  static_assert(RT || 2 * C * R <= (NR * 8 + NV * 4) * LS, "LIDAR offset tables must fit the window region");
  static_assert(RT || 5 * 4 * LS + 8 <= (NR * 8 + NV * 4) * LS, "reset staging must fit the window region");
  const int64_t valid = a.n - e0 < EPB ? a.n - e0 : EPB;
  if (__builtin_expect(any_done, 0)) {  // cold: laid out after the hot path
    const bool staged = stage_ok && npred == 1 && ndone == 1;  // then the done env is the predicted one
    // (register-staged: the single done env is the predicted one likewise)
    const int rsf = kRegStage ? __builtin_amdgcn_readfirstlane(__float_as_int(smem[kRsFlagF])) : 0;
    const bool rstaged = kRegStage && (rsf & 1) && ndone == 1;
    const uint4 ns = quad_done_path<NW, ONEWORD, (5 * CM + 27 + 63) / 64, BT>(
        kernargs(), tile_off, Cr, Rr, lane, wv, CW, e0, done, pack(s), ret, ndone, wfix, ctab,
        (staged || rstaged) ? stage : nullptr, (staged && stage_info) || (rstaged && (rsf & 2)), e_early, &epl, &eir,
        e_info, rstaged, (rstaged && (rsf & 2)) || (staged && info_reg));
    s = unpack(ns);
  }
  // the obs tile goes out through the waves other than the commit wave: its state
  // stores are still in flight (no fence at the barrier above), and the compiler
  // would make every iteration of its store loop wait for them (s_waitcnt vmcnt(0)
  // before re-using a store's data registers)
  if constexpr (CM >= 64) {  // long rows: the commit wave's share pays for its wait (64x64: 33.2 -> 32.7 us)
    if (wv == CW) __builtin_amdgcn_s_waitcnt(0x0F70);  // tracked vmcnt(0): no wait inside the loop
    if constexpr (BT) {
      if (a.obs_codes)
        store_tile_bytes(rows, a.obs_codes + e0 * g.D, (int)valid, g.D, (int)threadIdx.x, (int)blockDim.x);
      else
        store_tile_codes(rows, ctab, a.obs + e0 * g.D, (int)valid, g.D, (int)threadIdx.x, (int)blockDim.x);
    } else
      store_tile(rows, a.obs + e0 * g.D, (int)valid, g.D, g.D);
  } else {
#if PE_QUAD_TILE_BUF
    // A/B (debug builds): the f32 tile as compiler-counted buffer stores (pe_pipe.hpp's
    // form), by the non-commit waves (1) or by every wave (2)
    constexpr int kTB = PE_QUAD_TILE_BUF;
    if constexpr (!BT && !RT && EPB == kQuadEnvs) {
      float* dst = a.obs + e0 * g.D;
      if (valid == LS && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        if (kTB == 2)
          store_tile_buf<5 * C + 27, 64 * NW>(rows, dst, (int)threadIdx.x);
        else if (wv != CW)
          store_tile_buf<5 * C + 27, 64 * (NW - 1)>(rows, dst, (int)threadIdx.x);
      } else if (wv != CW) {
        store_tile(rows, dst, (int)valid, g.D, g.D, (int)threadIdx.x, 64 * (NW - 1));
      }
    } else
#endif
    if (wv != CW) {
      if constexpr (BT) {
        if (a.obs_codes)
          store_tile_bytes(rows, a.obs_codes + e0 * g.D, (int)valid, g.D, (int)threadIdx.x, 64 * (NW - 1));
        else
          store_tile_codes(rows, ctab, a.obs + e0 * g.D, (int)valid, g.D, (int)threadIdx.x, 64 * (NW - 1));
      } else
        store_tile(rows, a.obs + e0 * g.D, (int)valid, g.D, g.D, (int)threadIdx.x, 64 * (NW - 1));
    }
  }
  if (any_done && a.autoreset && !quad_coop(a, ndone) && (BT || reset_scratch_bytes(g.G, g.WPR, rl.P) <= 4 * g.D)) {
    // the tile store above wrote stale values (scratch bytes / the terminal codes)
    // into the done rows: drain it, then overwrite those rows with the fresh obs built
    // from the grid image (LDS scratch, or BT: the env's rows in HBM)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    quad_done_obs<NW, BT>(kernargs(), tile_off, lane, e, done, pack(s));
  }
  PE_STAMP(6);
#ifdef PE_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  PE_STAMP(7);
}

#include "pe_far.hpp"  // pe_step_far<C, R>: the sector kernel of long LIDAR ranges (R > 14)

#ifdef PE_DEBUG_KNOBS  // the persistent pipelined kernel: a debug-build A/B only (measured slower)
#include "../../tools/diag/pe_pipe.hpp"  // (the closed A/B kernel lives with the diagnostics)
#endif

// ---------------------------------------------------------------- pe_step_wave
// The fused step for every geometry without a compile-time sector kernel (any
// G <= 128, C <= 120, R <= 64; e.g. SURVEY §8(d)'s 64x64 / 64 rays / R=32 stress
// variant): ONE WAVE PER ENV.  The rover's window -- grid rows x-R-1 .. x+R+1
// clipped to the map, one contiguous 16-B-aligned span of the env's block, and
// visit rows x-3 .. x+3 -- is staged into the wave's LDS region with coalesced
// loads in one round after the scalars; the transition and commit are wave-uniform
// (scalar loads of the env's scalars / action / return); lane i marches ray i
// (i+64, ... for C > 64) over LDS (plantos_env.py:260-292), lanes 0..26 build the
// position and the 5x5 visit slice, and the obs row goes out through LDS as
// contiguous stores.  A done env's auto-reset is the wave-cooperative one of the
// sector kernel (prefetched record or in-place map generation, pe_coop.hpp) where
// coop_reset_ok; otherwise lane 0 runs the serial reset (reset_env).
// Per-wave LDS: the window words (max(min(G,2R+3)*WPR + 2, G*WPR) u64: also the
// cooperative reset's scratch), 7 visit rows of NW u32, the D-float obs row.
__host__ __device__ constexpr int wave_win_words(int G, int R, int WPR) {
  return ((((G < 2 * R + 3 ? G : 2 * R + 3) * WPR + 2) > G * WPR ? ((G < 2 * R + 3 ? G : 2 * R + 3) * WPR + 2)
                                                                  : G * WPR) + 1) & ~1;
}
__host__ __device__ constexpr int wave_lds_floats(int G, int R, int WPR, int NW, int D) {
  return 2 * wave_win_words(G, R, WPR) + ((7 * NW + 3) & ~3) + ((D + 3) & ~3);
}
// The workgroup's shared header: the obs tables (Tables' first 344 floats: dist,
// pos, vis) and the LIDAR offsets as int16 (dx & 0xFF | dy << 8) [C][RP], RP = R
// rounded up to 8 (one 16-B LDS read per 8 probes of a ray).
// (the rover-aligned kernels' entries are 3 B: a u16 LDS byte offset [C][RP], then a u8
// bit shift [C][RP]; rounded up to 16 B)
__host__ __device__ constexpr int wave_hdr_floats(int C, int R, bool aln) {
  return 344 + (aln ? ((C * ((R + 7) & ~7) * 3 + 15) & ~15) / 4 : C * ((R + 7) & ~7) / 2);
}
constexpr int kWaveEnvs = 8;  // envs (waves) per workgroup
// Rover-aligned window (ALN): after the transition the post-move rows xp-R .. xp+R
// are re-staged over the raw window, each shifted so that cell yp+dy+R of the
// padded row sits at bit 2(dy+R) of NWA = ceil((4R+2)/32) words, rows off the map
// filled with OBST.  A probe (dx, dy) is then word (dx+R)*NWA + (2(dy+R))>>5,
// shift (2(dy+R))&31 -- constants per (ray, probe) held in the LDS offset table
// (11-bit word | 5-bit shift << 11), no bounds check and no position arithmetic per
// probe.  Used when the aligned rows fit the raw region and kAlnSlots words per lane.
constexpr int kAlnSlots = 8;
__host__ __device__ constexpr int wave_aln_words(int R) { return (2 * R + 1) * ((4 * R + 33) >> 5); }
__host__ __device__ constexpr bool wave_aln_ok(int G, int R, int WPR) {
  return wave_aln_words(R) <= 64 * kAlnSlots && wave_aln_words(R) <= 2 * wave_win_words(G, R, WPR);
}
// one packed (dx & 0xFF | dy << 8) offset -> the aligned window's (word | shift << 11)
__host__ __device__ __forceinline__ uint32_t aln_entry(uint32_t v, int R, int NWA) {
  const int dx = (int)(int8_t)(v & 0xFFu), dy = (int)(int8_t)((v >> 8) & 0xFFu);
  const int cb = 2 * (dy + R);
  return (uint32_t)((dx + R) * NWA + (cb >> 5)) | ((uint32_t)(cb & 31) << 11);
}

// The wave kernel's done path (terminal obs / info, auto-reset), called by the
// wave of a done env with all lanes active.
template <int MAXW>
__device__ __attribute__((noinline)) void wave_done(const StepArgs& a, int64_t e, Scal s, int wfix, float* row,
                                                    uint64_t* win, const float* tdist, const float* tpos,
                                                    const float* tvis, int lane) {
  const Geo& g = a.g;
  const Rules& rl = a.rl;
  const State& st = a.st;
  const Tables* tab = st.tab;
  const int D = g.D;
  if (a.tobs)
    for (int k = lane; k < D; k += 64) a.tobs[e * D + k] = row[k];
  if (!a.autoreset) {
    if (a.tinfo && lane == 0) write_info(st, g, tab, e, s, a.tinfo + e * PE_NINFO);
  } else if (a.coop_max_done > 0) {  // coop_reset_ok geometry (pe_create)
    constexpr int KD = 6;            // D <= 347 (C <= 64): the record's obs row after its check
    PfLoad<MAXW, KD> pl;
    if (a.pf.scal) coop_load_prefetched<MAXW, KD>(a.pf, g, e, pl, lane);  // in flight from here on
    bool keep = false;
    if (st.cur && lane == 0) keep = curriculum_on_reset(st.cur, e, rl);  // A2C_training.py:56-95
    keep = __builtin_amdgcn_readfirstlane((int)keep) != 0;
    // with the curriculum the commit stored this env's rows: they land before the
    // info reads them and the reset rewrites them
    if (st.cur) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.tinfo) coop_write_info<MAXW>(st, g, e, s, a.tinfo + e * PE_NINFO, lane, wfix);
    Row4<MAXW> rw;
    Scal ns;
    asm volatile("" ::: "memory");  // terminal obs read out of the row before the fresh one goes in
    if (a.pf.scal && coop_take_prefetched<MAXW, KD>(a.pf, g, e, s.episode, pl, rw, ns, row, lane)) {
      ns = coop_apply_reset<MAXW>(st, g, e, ns, keep, rw, lane, nullptr, true);
    } else {
      ns = coop_reset_env<MAXW>(st, g, rl, e, s.episode, keep, rw, lane, win);
      coop_fresh_obs<MAXW>(g, rw, ns, row, tdist, tpos, tvis, st.ldx, st.ldy, lane);
    }
    if (lane == 0) {
      if (a.pf.scal) a.pf.flag[e] = 1;  // its next map goes into the next generating batch
      st_wt(st.ep_ret + e, 0.0);
      st_wt(st.scal + e, pack(ns));
    }
  } else if (lane == 0) {  // serial reset (the geometry has no cooperative one)
    if (a.tinfo) write_info(st, g, tab, e, s, a.tinfo + e * PE_NINFO, wfix);
    const Scal ns = reset_env(st, g, rl, tab, e, s.episode);
    st_wt(st.ep_ret + e, 0.0);
    st_wt(st.scal + e, pack(ns));
    build_obs_fresh(a, st.grid + e * g.gstride, ns, row, tab->dist, tab->pos, tab->vis, st.ldx, st.ldy);
  }
  // the LDS row / window are flat accesses here: all of them done before the caller's tile store
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

template <int MAXW, bool ALN>  // the cooperative reset's row words (1 or kCoopWPR); rover-aligned rays
#ifndef PE_WAVE_WPE4  // waves per SIMD of the multi-word variant (A/B builds only): 8 spills
#define PE_WAVE_WPE4 8  // ~130 B/lane yet beats 7 / 6 (64x64/R=32: 110.1 / 117.3 / 112.8 us)
#endif
__global__ __launch_bounds__(64 * kWaveEnvs) __attribute__((amdgpu_waves_per_eu(MAXW == 1 ? 8 : PE_WAVE_WPE4))) void pe_step_wave(StepArgs a) {  // <= 64 VGPRs at 8
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = a.g;
  const Rules& rl = a.rl;
  const State& st = a.st;
  const Tables* tab = st.tab;  // global: the serial reset path's tables
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t e = (int64_t)blockIdx.x * kWaveEnvs + wv;
  const int G = g.G, R = g.R, WPR = g.WPR, NW = g.NW, D = g.D, RP = (R + 7) & ~7;
  // ---- round 1 (uniform): the packed scalars and both action words in one round
  // trip, issued before the shared header's copy (a wave's round 1 waited for the
  // header's loads and the barrier before it started) -- unconditional loads at an
  // index clamped into the batch (the action's load inside a branch on act_bytes
  // was waited for before the return's was issued: three round trips before round 2)
  const int64_t ec = e < a.n ? e : (int64_t)a.n - 1;
  const uint4 sw = st.scal[ec];
  const int ash = a.act_bytes == 8 ? 1 : 0;  // 8-byte actions: two words, low first
  const int32_t* ap = reinterpret_cast<const int32_t*>(a.actions);
  const int32_t alo = ap[ec << ash], ahi = ap[(ec << ash) + ash];
  double ret = st.ep_ret[ec];  // (needed at the commit: in flight through round 2)
  // the shared header (read after the barrier)
  const float* tsrc = reinterpret_cast<const float*>(tab);
  for (int k = threadIdx.x; k < 344; k += blockDim.x) smem[k] = tsrc[k];
  int16_t* lofs = reinterpret_cast<int16_t*>(smem + 344);
  {  // the probe table, 16 B per thread and pass (st.ldxy, built by pe_create -- the
     // aligned-window entries too: converted here they cost 135 VALU per pass)
    const uint4* src = reinterpret_cast<const uint4*>(st.ldxy);
    uint4* dst = reinterpret_cast<uint4*>(lofs);
    const int nq = ALN ? (g.C * RP * 3 + 15) >> 4 : g.C * RP / 8;
    for (int k = threadIdx.x; k < nq; k += blockDim.x) dst[k] = src[k];
  }
  __syncthreads();
  if (e >= a.n) return;  // wave-uniform; no workgroup barrier below
  const float* tdist = smem;
  const float* tpos = smem + 72;
  const float* tvis = smem + 328;
  float* base = smem + wave_hdr_floats(g.C, R, ALN) + wv * wave_lds_floats(G, R, WPR, NW, D);
  uint64_t* win = reinterpret_cast<uint64_t*>(base);
  uint32_t* lvis = reinterpret_cast<uint32_t*>(base + 2 * wave_win_words(G, R, WPR));
  float* row = base + 2 * wave_win_words(G, R, WPR) + ((7 * NW + 3) & ~3);

  Scal s = unpack(sw);
  const int64_t action = ash ? (int64_t)(((uint64_t)(uint32_t)ahi << 32) | (uint32_t)alo) : (int64_t)alo;
  bool mv = false, water = false, bad = false;
  int dxm = 0, dym = 0;
  if (action < 4) {                                        // plantos_env.py:166
    const int64_t ai = action < 0 ? action + 4 : action;   // Python negative index
    if (ai < 0) {
      bad = true;                                          // reference IndexError
    } else {
      mv = true;                                           // :186 N,E,S,W
      dxm = ai == 0 ? -1 : (ai == 2 ? 1 : 0);
      dym = ai == 1 ? 1 : (ai == 3 ? -1 : 0);
    }
  } else {
    water = true;
  }
  const int nx = s.x + dxm, ny = s.y + dym;
  const bool inb = mv && nx >= 0 && nx < G && ny >= 0 && ny < G;  // :193-195

  // ---- round 2: the window span and the visit rows, every load issued before any
  // LDS write (clamped indices: unconditional loads, one memory round trip)
  const int lo = s.x - R - 1 > 0 ? s.x - R - 1 : 0, hi = s.x + R + 1 < G - 1 ? s.x + R + 1 : G - 1;
  const int w0 = (lo * WPR) & ~1;                      // 16-B aligned (env blocks are)
  const int nq = ((hi + 1) * WPR - w0 + 1) >> 1;       // uint4s (a trailing pad word at most)
  const uint4* gsrc = reinterpret_cast<const uint4*>(st.grid + e * g.gstride + w0);
  const int vlo = s.x - 3 > 0 ? s.x - 3 : 0, vhi = s.x + 3 < G - 1 ? s.x + 3 : G - 1;
  const int nv = (vhi - vlo + 1) * NW;
  const uint32_t* vsrc = vis_env(st, g, e, s.episode) + (int64_t)vlo * NW;
  uint32_t eo = 0u, en = 0u;
  const int cell_o = s.x * G + s.y, cell_n = nx * G + (inb ? ny : s.y);
  if (inb && (s.flags & F_EXPL_BITMAP)) {
    eo = st.expl[e * g.estride + (cell_o >> 5)];
    en = st.expl[e * g.estride + (cell_n >> 5)];
  }
  const double cthr = st.cur ? st.cur[e].thr : 0.0;  // CurriculumWrapper threshold
  uint32_t vv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = lane + 64 * j;
    vv[j] = vsrc[k < nv ? k : nv - 1];
  }
  {  // the window's first 256 16-B units (all of it up to 2R+3 rows of 4 words, e.g. 64x64/R32)
    uint4 gv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = lane + 64 * j;
      gv[j] = gsrc[q < nq ? q : nq - 1];
    }
    // every load of round 2 lands here, in one wait (asm operands): as a loop, or with
    // the loads left to the compiler, some were sunk into the conditional LDS writes
    // below and each waited for alone (64x64/R32: the visit rows, then 3 window loads)
    asm volatile("" ::"v"(vv[0]), "v"(vv[1]), "v"(gv[0].x), "v"(gv[1].x), "v"(gv[2].x), "v"(gv[3].x));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = lane + 64 * j;
      if (q < nq) {
        win[2 * q] = (uint64_t)gv[j].x | ((uint64_t)gv[j].y << 32);
        win[2 * q + 1] = (uint64_t)gv[j].z | ((uint64_t)gv[j].w << 32);
      }
    }
  }
  for (int q0 = 4 * 64; q0 < nq; q0 += 4 * 64) {  // (G+2R > 128 cells with many rows)
    uint4 gv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + lane + 64 * j;
      gv[j] = gsrc[q < nq ? q : nq - 1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + lane + 64 * j;
      if (q < nq) {
        win[2 * q] = (uint64_t)gv[j].x | ((uint64_t)gv[j].y << 32);
        win[2 * q + 1] = (uint64_t)gv[j].z | ((uint64_t)gv[j].w << 32);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = lane + 64 * j;
    if (k < nv) lvis[k] = vv[j];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS writes before its reads (in order)

  // cell code / visit nibble from the staged window (rows outside [lo, hi] are off-map)
  auto code_at = [&](int xr, int pcol) -> int {
    if (xr < 0 || xr >= G) return OBST;
    const int bit = 2 * pcol;
    return (int)((win[xr * WPR + (bit >> 6) - w0] >> (bit & 63)) & 3u);
  };
  auto vword = [&](int xr, int col) -> int { return (xr - vlo) * NW + ((4 * (col + 2)) >> 5); };
  const uint32_t* win32 = reinterpret_cast<const uint32_t*>(win);

  // ---- transition (plantos_env.py:160-222), wave-uniform
  s.step = s.step < 65535 ? s.step + 1 : 65535;                 // :162
  bool ok = false, watered = false, wet_hyd = false;
  uint32_t n = 0u;
  double h = 0.0;
  if (mv) {
    ok = inb && code_at(nx, ny + R) != OBST;                     // :193-195 (plants walkable)
    if (ok) {
      n = (lvis[vword(nx, ny)] >> ((4 * (ny + 2)) & 31)) & 15u;
      h = n == 0u ? rl.r_exploration : rl.r_revisit;             // :197, 204-207
    } else {
      s.flags |= F_COLLIDED;                                     // :209
      s.coll = s.coll < 65535 ? s.coll + 1 : 65535;              // :210
      h = rl.r_invalid;                                          // :211
    }
  } else if (water) {
    const int cd = code_at(s.x, s.y + R);
    if (cd == THIRSTY) {                                         // fork plantos_env_new.py:237-240
      watered = true;
      h = rl.r_goal;
    } else if (cd == HYD) {                                      // fork :241-242 (root raises)
      wet_hyd = true;
      h = rl.r_mistake;
    } else {
      h = rl.r_water_empty;                                      // :221-222
    }
  }
  const uint32_t nib = n < 15u ? n + 1u : 15u;                   // :203
  uint32_t wo = eo, wn = en;
  if (ok) {
    if (s.flags & F_EXPL_BITMAP) {                               // explored[old]=1, [new]=2 (:198-200)
      const uint32_t bo = 1u << (cell_o & 31), bn = 1u << (cell_n & 31);
      if ((cell_o >> 5) == (cell_n >> 5)) {
        if (!(wo & bo)) { wo |= bo; s.expl++; }
        if (!(wo & bn)) { wo |= bn; s.expl++; }
      } else {
        if (!(wo & bo)) { wo |= bo; s.expl++; }
        if (!(wn & bn)) { wn |= bn; s.expl++; }
      }
    } else if (n == 0u) {
      s.expl++;  // derived mode: explored[new] was 0 iff never visited
    }
  }
  if (bad) s.flags |= F_POISON_ACT;
  const bool new_hyd_poison = wet_hyd && !(s.flags & F_POISON_HYD);
  if (wet_hyd) s.flags |= F_POISON_HYD;
  const int ox = s.x, oy = s.y;
  if (ok) {
    s.x = nx;                                                    // :199
    s.y = ny;
  }
  double rew = rl.r_step;                                        // :164
  rew += h;
  bool term = s.expl >= s.total;                                 // :176, 244-246, 331
  const bool trunc = s.step >= rl.max_steps;                     // :177
  if (term && !(s.flags & F_BONUS)) {                            // :179-181
    rew += rl.r_complete;
    s.flags |= F_BONUS;
  }
  // the post-step window in LDS (the rays see the watered cell, the slice the visit)
  const int kvn = ok ? vword(nx, ny) : 0;
  const uint32_t wvn = ok ? (lvis[kvn] & ~(0xFu << ((4 * (ny + 2)) & 31))) | (nib << ((4 * (ny + 2)) & 31)) : 0u;
  const int cbit = 2 * (oy + R), kw = ox * WPR + (cbit >> 6) - w0;
  const uint64_t wwr = watered ? win[kw] & ~(1ull << (cbit & 63)) : 0ull;  // code 3 -> 2
  if (lane == 0) {
    if (bad) atomicOr(st.err_bits, F_POISON_ACT);
    if (new_hyd_poison) atomicOr(st.err_bits, F_POISON_HYD);
    if (st.cur) term = curriculum_hit(st.cur, e, cthr, s.expl, s.total, rl.cur_term) || term;  // A2C_training.py:101-103
  }
  term = __builtin_amdgcn_readfirstlane((int)term) != 0;
  const bool done = term || trunc;
  // an env about to be auto-reset gets new rows: its last move / watering is not
  // stored (the terminal info accounts for the watering), unless the curriculum
  // carries its visits over
  const bool reset_now = done && a.autoreset;
  const bool commit_rows = !(reset_now && !st.cur);
  const int wfix = (watered && reset_now && !st.cur) ? 1 : 0;
  if (lane == 0) {
    if (ok) lvis[kvn] = wvn;
    if (watered) win[kw] = wwr;
    if (commit_rows) {
      if (ok) {
        const int b = (ny + 2) >> 1;  // the byte of the target's nibble in row nx
        st_wt(reinterpret_cast<uint8_t*>(vis_env(st, g, e, s.episode) + (int64_t)nx * NW) + b,
              (uint8_t)(wvn >> (8 * (b & 3))));
        // (written here, not deferred through vpend as in the headline kernel: holding the
        // pending word across this kernel spilled 29 more SGPRs, 64x64/R32 85.8 -> 90.2 us,
        // profiles/r4q/ab_g64r32.jsonl)
        visit_bump_exact(st, g, e, cell_n, n);
        if (s.flags & F_EXPL_BITMAP) {
          if (wo != eo) st.expl[e * g.estride + (cell_o >> 5)] = wo;
          if ((cell_o >> 5) != (cell_n >> 5) && wn != en) st.expl[e * g.estride + (cell_n >> 5)] = wn;
        }
      }
      if (watered) {
        const int B = (oy + R) >> 2;  // the byte of the cell's code in row ox
        st_wt(reinterpret_cast<uint8_t*>(st.grid + e * g.gstride + (int64_t)ox * WPR) + B,
              (uint8_t)(wwr >> (8 * (B & 7))));
      }
    }
    ret += rew;
    st_wt(a.reward + e, (float)rew);
    st_wt(a.term + e, (uint8_t)term);
    st_wt(a.trunc + e, (uint8_t)trunc);
    if (done) {  // Monitor's episode return / length of the ended episode
      if (a.ep_ret_out) st_wt(a.ep_ret_out + e, ret);
      if (a.ep_len_out) st_wt(a.ep_len_out + e, (int32_t)s.step);
    }
    if (commit_rows) {  // else the reset below stores the new episode's scalars
      st_wt(st.ep_ret + e, ret);
      st_wt(st.scal + e, pack(s));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- observation (plantos_env.py:251-315) into the LDS row
  const int xp = s.x, yp = s.y;
  if constexpr (ALN) {  // the rover-aligned window over the raw one (every read before any write)
    const int NWA = (4 * R + 33) >> 5, tot = (2 * R + 1) * NWA;
    const uint32_t mg = 0xFFFFFFFFu / (uint32_t)NWA + 1u;  // k / NWA as a high multiply (k < 512; NWA >= 2)
    const int sw = (2 * yp) >> 5, sb = (2 * yp) & 31;
    uint32_t av[kAlnSlots];
#pragma unroll
    for (int t = 0; t < kAlnSlots; ++t) {
      if (64 * t >= tot) break;  // (uniform: slots past the window -- 40x40/R8 uses 1 of 8)
      const int k = lane + 64 * t;
      const int i = NWA == 1 ? k : (int)__umulhi((uint32_t)k, mg), w = k - i * NWA;
      const int xr = xp - R + i;
      av[t] = 0x55555555u;  // OBST (1) in every cell: rows off the map (:271-284)
      if (k < tot && (uint32_t)xr < (uint32_t)G) {
        const int q = 2 * ((int)__umul24((uint32_t)xr, (uint32_t)WPR) - w0) + sw + w;
        av[t] = __builtin_amdgcn_alignbit(win32[q + 1], win32[q], (uint32_t)sb);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t* awin = reinterpret_cast<uint32_t*>(win);
#pragma unroll
    for (int t = 0; t < kAlnSlots; ++t) {
      const int k = lane + 64 * t;
      if (k < tot) awin[k] = av[t];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const char* wbyte = reinterpret_cast<const char*>(win);
  for (int i = lane; i < g.C; i += 64) {
    const uint4* orow = reinterpret_cast<const uint4*>(lofs + i * RP);
    const uint2* srow = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(lofs) + g.C * RP * 2 + i * RP);
    int dist = R, ent = EMPTY;
    for (int r0 = 0; r0 < R; r0 += 8) {  // 8 probes per 16-B offset read, their codes in flight together
      const uint4 o = orow[r0 >> 3];
      const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
      uint2 os = make_uint2(0u, 0u);
      if constexpr (ALN) os = srow[r0 >> 3];
      const uint32_t sw[2] = {os.x, os.y};
      // the 8 probe codes packed 2 bits each (probe j at bits 2j), first hit by one
      // find-first-set (as the sector kernel's quad_rays); 32-bit window reads (a
      // 2-bit code never straddles a word: its bit offset is even; the row offset as a
      // full-rate 24-bit multiply, not the quarter-rate 32-bit one)
      uint32_t pk = 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t v = ow[j >> 1] >> (16 * (j & 1));
        uint32_t c;
        if constexpr (ALN) {  // the probe's LDS byte offset and bit shift; off-map rows hold OBST
          // (ubfe reads the low 5 bits of its offset operand: the shift byte needs no mask)
          c = __builtin_amdgcn_ubfe(*reinterpret_cast<const uint32_t*>(wbyte + (v & 0xFFFFu)),
                                    sw[j >> 2] >> (8 * (j & 3)), 2u);
        } else {
          const int cx = xp + (int)(int8_t)(v & 0xFFu);
          const int bit = 2 * (yp + (int)(int8_t)((v >> 8) & 0xFFu) + R);
          c = (uint32_t)cx < (uint32_t)G  // :271-284 (off-map rows: obstacle)
                  ? (win32[2 * ((int)__umul24((uint32_t)cx, (uint32_t)WPR) - w0) + (bit >> 5)] >> (bit & 31)) & 3u
                  : (uint32_t)OBST;
        }
        pk |= c << (2 * j);
      }
      if (R - r0 < 8) pk &= (1u << (2 * (R - r0))) - 1u;  // the zero-padded offsets past R
      const uint32_t nz = (pk | (pk >> 1)) & 0x5555u;
      if (nz) {
        const int f = __builtin_ctz(nz);  // 2j of the first hit
        dist = r0 + (f >> 1) + 1;
        ent = (int)((pk >> f) & 3u);
        break;
      }
    }
    row[5 * i] = tdist[dist];                                    // :288
    row[5 * i + 1] = ent == 0 ? 1.0f : 0.0f;
    row[5 * i + 2] = ent == 1 ? 1.0f : 0.0f;
    row[5 * i + 3] = ent == 2 ? 1.0f : 0.0f;
    row[5 * i + 4] = ent == 3 ? 1.0f : 0.0f;
  }
  if (lane < 25) {                                               // :298-313
    const int gx = xp + lane / 5 - 2, gy = yp + lane % 5 - 2;
    const bool in = gx >= 0 && gx < G && gy >= 0 && gy < G;
    const uint32_t v = in ? (lvis[vword(gx, gy)] >> ((4 * (gy + 2)) & 31)) & 15u : 10u;
    row[5 * g.C + 2 + lane] = tvis[v];
  } else if (lane < 27) {
    row[5 * g.C + lane - 25] = tpos[lane == 25 ? xp : yp];       // :294-296
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- DummyVecEnv auto-reset (rare) and terminal outputs: out of line, so that the
  // reset path's pointers and state do not shape the hot path's register allocation
  if (done) {  // the kernel's argument read in place (StepArgs is its only argument): taking
              // &a would copy the whole struct to scratch on every launch
    const StepArgs* ap = (const StepArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    wave_done<MAXW>(*ap, e, s, wfix, row, win, tdist, tpos, tvis, lane);
  }
  // the obs row: long rows as 16-B stores from the first 16-B boundary of the row on,
  // the 0-3 floats before it and the tail as single floats
  float* dst = a.obs + e * D;
  const int hd = (int)((16u - ((uint32_t)reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u) >> 2;
  const int n4 = (D - hd) >> 2;
  // (rover-aligned kernels only: in the other one its registers made the SGPRs spill, and
  // none of its geometries benched has rows that long)
  if (ALN && D >= PE_WAVE_ROWSTORE_MIN && (reinterpret_cast<uintptr_t>(dst) & 3u) == 0) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    for (int k = lane; k < n4; k += 64) {
      const float* sr = row + hd + 4 * k;
      const v4f v = {sr[0], sr[1], sr[2], sr[3]};
      *reinterpret_cast<v4f*>(dst + hd + 4 * k) = v;
    }
    if (lane < hd) dst[lane] = row[lane];
    if (lane < D - hd - 4 * n4) dst[hd + 4 * n4 + lane] = row[hd + 4 * n4 + lane];
  } else {
    for (int k = lane; k < D; k += 64) dst[k] = row[k];
  }
}

// reset() with one wave per env (pe_coop.hpp): the map, grid/visit rows and the
// fresh obs of env e by the 64 lanes of wave e % 4 of block e / 4 -- 65536 envs
// are 65536 waves, so the whole chip generates maps at once (the lane-per-env
// kernel below gives one env per lane: 29 ms at 64x64, where it scans its grid
// image in HBM).  Unmasked envs rebuild their obs from the current state.
template <int MAXW>
__global__ __launch_bounds__(256) void pe_reset_coop_kernel(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = a.g;
  load_tables(smem, a.st.tab);
  __syncthreads();
  const float* tdist = smem;
  const float* tpos = smem + 72;
  const float* tvis = smem + 328;
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= a.n) return;  // wave-uniform
  const Scal s = unpack(a.st.scal[e]);
  const bool resetting = !a.mask || a.mask[e];
  if (resetting) {
    bool keep = false;
    if (a.st.cur && lane == 0) keep = curriculum_on_reset(a.st.cur, e, a.rl);  // A2C_training.py:56-95
    keep = __builtin_amdgcn_readfirstlane((int)keep) != 0;
    Row4<MAXW> rw;
    uint64_t* scr = reinterpret_cast<uint64_t*>(smem + kTabFloats) + (threadIdx.x >> 6) * coop_scratch_words(g.G, g.WPR);
    const Scal ns = coop_reset_env<MAXW>(a.st, g, a.rl, e, s.episode, keep, rw, lane, scr);
    if (lane == 0) {
      a.st.ep_ret[e] = 0.0;
      a.st.scal[e] = pack(ns);
    }
    if (a.obs) coop_fresh_obs<MAXW>(g, rw, ns, a.obs + e * g.D, tdist, tpos, tvis, a.st.ldx, a.st.ldy, lane);
  } else if (a.obs && lane == 0) {
    build_obs_generic(a, e, s.episode, s.x, s.y, a.obs + e * g.D, tdist, tpos, tvis, a.st.ldx, a.st.ldy);
  }
}

// The envs flagged by step kernels since the last prefetch launch, compacted into
// pf.queue (256 envs per workgroup, one atomic per workgroup with a flagged env: one per
// wave was 1024 atomics on one counter), flags cleared.  Runs right before the
// queue-mode prefetch launch, on the same stream.
__global__ __launch_bounds__(256) void pe_pf_compact_kernel(Prefetch pf, int n) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool f = e < n && pf.flag[e] != 0;
  const uint64_t m = __ballot(f);
  __shared__ uint32_t wc[4], bb;
  const int w = threadIdx.x >> 6;
  if (lane == 0) wc[w] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wc[0] + wc[1] + wc[2] + wc[3];
    bb = tot ? atomicAdd(pf.qn, tot) : 0u;
  }
  __syncthreads();
  uint32_t base = bb;
  for (int k = 0; k < w; ++k) base += wc[k];
  if (f) {
    pf.queue[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)e;
    pf.flag[e] = 0;
  }
}

// Prefetched resets (pe_coop.hpp Prefetch): generate the next reset's map, grid
// rows and fresh obs of the envs queued by the step kernel (all == 0; grid-stride
// over the queue, then the last workgroup clears the queue), or of every env
// (all != 0: one wave per env; after create / reset()), skipping envs whose
// record already holds the reset of their current episode counter.
template <int MAXW, bool BT = false>  // BT: the records' obs rows as byte codes (a byte-coded step tile)
__global__ __launch_bounds__(256) void pe_prefetch_kernel(StepArgs a, int all) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = a.g;
  const Prefetch& pf = a.pf;
  const uint32_t queued = all ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane((int)pf.qn[0]);
  if (!all && queued == 0u) return;  // nothing queued (the usual launch between synchronized resets)
  load_tables(smem, a.st.tab);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (int64_t)gridDim.x * 4;
  uint64_t* scr = reinterpret_cast<uint64_t*>(smem + kTabFloats) + (threadIdx.x >> 6) * coop_scratch_words(g.G, g.WPR);
  const int64_t cnt = all ? (int64_t)a.n : (int64_t)(queued < (uint32_t)a.n ? queued : (uint32_t)a.n);
  for (int64_t i = wid; i < cnt; i += nwaves) {
    const int64_t e = all ? i : (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)pf.queue[i]);
    const uint32_t ep = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.st.scal[e].w);
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)pf.scal[e].w) == ep + 1u) continue;  // already there
    Row4<MAXW> rw;
    const Scal s = coop_gen_map<MAXW>(g, a.rl, a.st.tab, rw, a.rl.env_off + (uint32_t)e, ep, lane, scr);
    if (lane < g.G) {
      uint64_t* dst = pf.grid + e * g.gstride + (int64_t)lane * g.WPR;
#pragma unroll
      for (int w = 0; w < MAXW; ++w)
        if (MAXW == 1 || w < g.WPR) dst[w] = rw.get(w);
    }
    // the new episode's fresh visit rows into its slot -- the env's idle one (episode
    // ep + 1 vs the running ep): the step that takes this record stores no visit row
    coop_fresh_visits<true>(a.st, g, e, s, lane, reinterpret_cast<const Tables*>(smem));
    if constexpr (BT)
      coop_fresh_obs<MAXW>(g, rw, s, reinterpret_cast<uint8_t*>(pf_obs_row(pf, e)), smem, smem + 72, smem + 328,
                           a.st.ldx, a.st.ldy, lane);
    else
      coop_fresh_obs<MAXW>(g, rw, s, pf_obs_row(pf, e), smem, smem + 72, smem + 328, a.st.ldx, a.st.ldy, lane);
    if (lane == 0) pf.scal[e] = pack(s);  // read by a later launch only
  }
  if (!all) {
    __syncthreads();  // every wave of this workgroup has read the count
    if (threadIdx.x == 0 && atomicAdd(pf.qn + 1, 1u) == gridDim.x - 1) {
      pf.qn[0] = 0u;  // the last workgroup: nobody reads the count any more
      pf.qn[1] = 0u;
    }
  }
}

// reset(): masked device-rng reset, then obs of every env (obs may be NULL).
__global__ __launch_bounds__(kBlock) void pe_reset_kernel(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tdist = smem;
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  float* rows = smem + kTabFloats;
  const Geo& g = a.g;
  // LIDAR offsets after the tile (read by the obs builders in dependent chains)
  signed char* lldx = reinterpret_cast<signed char*>(rows + kBlock * g.DS);
  signed char* lldy = lldx + g.C * g.R;
  load_tables(smem, a.st.tab);
  for (int k = threadIdx.x; k < g.C * g.R; k += blockDim.x) {
    lldx[k] = a.st.ldx[k];
    lldy[k] = a.st.ldy[k];
  }
  const Tables* ltab = reinterpret_cast<const Tables*>(smem);
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * kBlock;
  const int64_t e = e0 + threadIdx.x;
  float* row = rows + threadIdx.x * g.DS;
  // a resetting env generates its map in its own tile row (LDS), cf. pe_step_quad
  const bool scratch_ok = reset_scratch_bytes(g.G, g.WPR, a.rl.P) <= 4 * g.DS;
  uint64_t* sg = reinterpret_cast<uint64_t*>(row + ((threadIdx.x * g.DS) & 1));
  bool resetting = false;
  Scal s;
  if (e < a.n) {
    s = unpack(a.st.scal[e]);
    resetting = !a.mask || a.mask[e];
    if (resetting) {
      s = scratch_ok ? reset_env_scratch(a.st, g, a.rl, ltab, e, s.episode, sg)
                     : reset_env(a.st, g, a.rl, ltab, e, s.episode);
      a.st.ep_ret[e] = 0.0;
      a.st.scal[e] = pack(s);
    }
    if (a.obs && resetting && !scratch_ok)
      build_obs_fresh(a, a.st.grid + e * g.gstride, s, row, tdist, tpos, tvis, lldx, lldy);
    else if (a.obs && !resetting)
      build_obs_generic(a, e, s.episode, s.x, s.y, row, tdist, tpos, tvis, lldx, lldy);
  }
  if (!a.obs) return;
  __syncthreads();
  const int64_t valid = a.n - e0 < kBlock ? a.n - e0 : kBlock;
  store_tile(rows, a.obs + e0 * g.D, (int)valid, g.D, g.DS);
  if (scratch_ok) {  // overwrite the scratch rows the tile store wrote
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (resetting) build_obs_fresh(a, sg, s, a.obs + e * g.D, tdist, tpos, tvis, lldx, lldy);
  }
}

// pe_load_maps: host-supplied layouts (CPython-stream reset mode).
__global__ __launch_bounds__(kBlock) void pe_load_maps_kernel(StepArgs a, int k, const int32_t* idx,
                                                              const uint8_t* cells, const int32_t* rover) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tdist = smem;
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  float* rows = smem + kTabFloats;
  load_tables(smem, a.st.tab);
  const Tables* ltab = reinterpret_cast<const Tables*>(smem);
  __syncthreads();
  const int j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= k) return;
  const Geo& g = a.g;
  const int64_t e = idx[j];
  const uint8_t* c = cells + (int64_t)j * g.GG;
  const bool keep = a.st.cur ? curriculum_on_reset(a.st.cur, e, a.rl) : false;  // A2C_training.py:56-95
  int n_obst = 0;
  for (int row = 0; row < g.G; ++row) {
    for (int w = 0; w < g.WPR; ++w) a.st.grid[e * g.gstride + (int64_t)row * g.WPR + w] = ltab->grid_pad[w];
    for (int col = 0; col < g.G; ++col) {
      int code = c[row * g.G + col] & 3;
      n_obst += code == OBST;
      if (code) grid_set(a.st, g, e, row, col + g.R, code);
    }
  }
  Scal s = unpack(a.st.scal[e]);
  s.x = rover[2 * j];
  s.y = rover[2 * j + 1];
  s.step = 0;
  s.coll = 0;
  s.flags = 0;
  s.episode += 1u;
  s.total = g.GG - n_obst;
  s.expl = 1;
  new_episode_visits(a.st, g, ltab, e, s, keep);  // plantos_env.py:146-147, 236
  a.st.scal[e] = pack(s);
  a.st.ep_ret[e] = 0.0;
  float* row = rows + threadIdx.x * g.DS;
  // reset() obs of the fresh episode (a carried CurriculumWrapper visit map is
  // installed after env.reset() returned, A2C_training.py:90-91: not in this obs)
  build_obs_fresh(a, a.st.grid + e * g.gstride, s, row, tdist, tpos, tvis, a.st.ldx, a.st.ldy);
  if (a.obs)
    for (int q = 0; q < g.D; ++q) a.obs[(int64_t)j * g.D + q] = row[q];
}

// _get_info (plantos_env.py:317-336), integer columns.
__global__ void pe_info_kernel(StepArgs a, int32_t* info) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  const Geo& g = a.g;
  static_assert(PE_NINFO == 11 && PE_I_POISONED == 10, "write_info column layout");
  write_info(a.st, g, a.st.tab, e, unpack(a.st.scal[e]), info + e * PE_NINFO);
}

// get_state: one thread per (env, cell).
__global__ void pe_get_cells_kernel(StepArgs a, uint8_t* cells, int32_t* visits, int8_t* explored) {
  const Geo& g = a.g;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.n * g.GG) return;
  const int64_t e = t / g.GG;
  const int c = (int)(t - e * g.GG);
  const int row = c / g.G, col = c - row * g.G;
  if (cells) cells[t] = (uint8_t)grid_code(a.st, g, e, row, col + g.R);
  const Scal s = unpack(a.st.scal[e]);
  if (visits) visits[t] = visit_exact(a.st, g, e, s.episode, row, col);
  if (explored) {
    int8_t v;
    if (s.flags & F_EXPL_BITMAP) {
      uint32_t w = a.st.expl[e * g.estride + (c >> 5)];
      v = (w >> (c & 31)) & 1u ? 1 : 0;
    } else {
      v = nibble_get(a.st, g, e, s.episode, row, col) ? 1 : 0;  // explored_map > 0 <=> visit > 0
    }
    if (v && s.x == row && s.y == col) v = 2;  // plantos_env.py:200, 236
    explored[t] = v;
  }
}

__global__ void pe_get_scal_kernel(StepArgs a, int32_t* scal) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  Scal s = unpack(a.st.scal[e]);
  int32_t* o = scal + e * PE_NSCAL;
  o[PE_S_X] = s.x;
  o[PE_S_Y] = s.y;
  o[PE_S_STEP] = s.step;
  o[PE_S_COLL] = s.coll;
  o[PE_S_COLLIDED] = (s.flags & F_COLLIDED) ? 1 : 0;
  o[PE_S_BONUS] = (s.flags & F_BONUS) ? 1 : 0;
  o[PE_S_POISONED] = (int)((s.flags >> 2) & 7u);
  o[PE_S_EPISODE] = (int32_t)s.episode;
}

// set_state: one thread per env, in this order: (1) if explored stays derived but
// visits change, freeze the current explored map into the bitmap; (2) cells,
// (3) visits, (4) explored, (5) scalars; (6) derived counters and the explored
// mode: derived (bitmap not read) iff explored_map > 0 <=> visit > 0 everywhere.
__global__ void pe_set_env_kernel(StepArgs a, const uint8_t* cells, const int32_t* visits, const int8_t* explored,
                                  const int32_t* scal) {
  const Geo& g = a.g;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  Scal s = unpack(a.st.scal[e]);
  // the visit rows live in the slot of the episode counter (pe_device.hpp vis_env): the
  // new counter's, when the scalars are set too
  const uint32_t ep0 = s.episode, ep1 = scal ? (uint32_t)scal[e * PE_NSCAL + PE_S_EPISODE] : ep0;
  uint32_t* eb = a.st.expl + e * g.estride;
  if (!(s.flags & F_EXPL_BITMAP) && visits && !explored) {
    for (int w = 0; w < g.estride; ++w) eb[w] = 0u;
    for (int c = 0; c < g.GG; ++c)
      if (nibble_get(a.st, g, e, ep0, c / g.G, c % g.G)) eb[c >> 5] |= 1u << (c & 31);
    s.flags |= F_EXPL_BITMAP;
  }
  if (cells) {
    for (int row = 0; row < g.G; ++row) {
      for (int w = 0; w < g.WPR; ++w) a.st.grid[e * g.gstride + (int64_t)row * g.WPR + w] = a.st.tab->grid_pad[w];
      for (int col = 0; col < g.G; ++col) {
        int code = cells[e * g.GG + row * g.G + col] & 3;
        if (code) grid_set(a.st, g, e, row, col + g.R, code);
      }
    }
  }
  if (visits) {
    uint32_t* vb = vis_env(a.st, g, e, ep1);
    for (int row = 0; row < g.G; ++row) {
      for (int w = 0; w < g.NW; ++w) vb[(int64_t)row * g.NW + w] = a.st.tab->vis_pad[w];
      for (int col = 0; col < g.G; ++col) {
        int32_t v = visits[e * g.GG + row * g.G + col];
        uint32_t vc = v <= 0 ? 0u : (uint32_t)v;
        a.st.vx[e * g.hstride + row * g.G + col] = vc;
        vis_set(a.st, g, e, ep1, row, col, vc < 15u ? vc : 15u);
      }
    }
  } else if ((ep0 ^ ep1) & 1u) {
    carry_visits(a.st, g, e, ep1);  // the counts move with the counter's parity
  }
  if (explored) {
    for (int w = 0; w < g.estride; ++w) {
      uint32_t bits = 0;
      for (int b = 0; b < 32; ++b) {
        int c = w * 32 + b;
        if (c < g.GG && explored[e * g.GG + c] > 0) bits |= 1u << b;
      }
      eb[w] = bits;
    }
    s.flags |= F_EXPL_BITMAP;
  }
  // the prefetched record stays valid only if the counter stays (its key, ep0 + 1, is
  // still the next episode's, and its fresh rows in slot (ep0 + 1) & 1 untouched): a
  // counter moved back would turn an old key into a future one over rows since reused
  if (a.pf.scal && ep1 != ep0) a.pf.scal[e].w = 0u;
  if (scal) {
    const int32_t* i = scal + e * PE_NSCAL;
    s.x = i[PE_S_X];
    s.y = i[PE_S_Y];
    s.step = i[PE_S_STEP] < 0 ? 0 : (i[PE_S_STEP] > 65535 ? 65535 : i[PE_S_STEP]);
    s.coll = i[PE_S_COLL] < 0 ? 0 : (i[PE_S_COLL] > 65535 ? 65535 : i[PE_S_COLL]);
    s.flags = (s.flags & F_EXPL_BITMAP) | (i[PE_S_COLLIDED] ? F_COLLIDED : 0u) | (i[PE_S_BONUS] ? F_BONUS : 0u) |
              ((uint32_t)(i[PE_S_POISONED] & 7) << 2);
    s.episode = (uint32_t)i[PE_S_EPISODE];
  }
  int ex = 0, ob = 0;
  if (s.flags & F_EXPL_BITMAP) {
    bool same = true;
    for (int c = 0; c < g.GG; ++c) {
      const bool bit = (eb[c >> 5] >> (c & 31)) & 1u;
      ex += bit;
      same = same && (bit == (nibble_get(a.st, g, e, ep1, c / g.G, c % g.G) != 0u));
    }
    if (same) s.flags &= ~F_EXPL_BITMAP;
  } else {
    for (int c = 0; c < g.GG; ++c) ex += nibble_get(a.st, g, e, ep1, c / g.G, c % g.G) != 0u;
  }
  for (int row = 0; row < g.G; ++row)
    for (int w = 0; w < g.WPR; ++w) {
      uint64_t v = a.st.grid[e * g.gstride + (int64_t)row * g.WPR + w];
      ob += __popcll(v & ~(v >> 1) & a.st.tab->grid_real[w] & kEven64);
    }
  s.expl = ex;
  s.total = g.GG - ob;
  a.st.scal[e] = pack(s);
}

// pe_seed(reset_episode_counters): episode := 0, an odd episode's visit rows copied
// to slot 0.  A prefetched record keyed k promises fresh rows of episode k in slot
// k & 1; with the counter moved back, an old key becomes a future one (an env at
// episode 1 holds the record of episode 2, whose slot-0 rows the copy just
// overwrote, and the counter reaches 1 again), so every record is dropped except
// episode 1's of an env still at episode 0 (slot 1 untouched since the prefetch).
__global__ void pe_zero_episodes_kernel(StepArgs a) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  uint4 w = a.st.scal[e];
  if (w.w & 1u) {
    const uint32_t* src = vis_env(a.st, a.g, e, 1u);
    uint32_t* dst = vis_env(a.st, a.g, e, 0u);
    for (int64_t k = 0; k < a.g.vslot; ++k) dst[k] = src[k];
  }
  if (a.pf.scal && w.w != 0u) a.pf.scal[e].w = 0u;
  w.w = 0u;
  a.st.scal[e] = w;
}

// The deferred overflow writes (pe_device.hpp vx_pending) of every env applied and
// cleared: before any API call that reads the exact visit counts or replaces them.
__global__ void pe_vx_flush_kernel(StepArgs a) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  const uint32_t p = a.st.vpend[e];
  if (p) {
    vx_apply(a.st, a.g, e, p);
    a.st.vpend[e] = 0u;
  }
}

// CurriculumWrapper.__init__ state of every env (A2C_training.py:41-54).
__global__ void pe_cur_init_kernel(CurRec* cur, int n, double thr) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  CurRec c;
  c.thr = thr;
  c.episodes = c.successes = c.on_maze = c.flags = 0u;
  c.pad[0] = c.pad[1] = 0u;
  cur[e] = c;
}

__global__ void pe_synth_kernel(int n, uint64_t seed, uint32_t env_off, uint32_t t, int32_t* actions) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint4 o = philox(make_uint4(t, env_off + (uint32_t)e, 0u, kDomainAction), (uint32_t)seed, (uint32_t)(seed >> 32));
  actions[e] = (int32_t)(o.x % 5u);
}

}  // namespace

// pe_expand_obs_codes: blocks x rows packed code buffers (codes u8 [rows, D] | reward
// f32 | terminated | truncated, block b at src + b * stride) -> contiguous f32 obs
// (+ the other outputs).  Grid: (x: 16-B output chunks, y: block); one u32 of 4 codes
// per thread through the LDS code table, one 16-B store.
#ifndef PE_EXPAND_PER
#define PE_EXPAND_PER 4
#endif
#ifndef PE_EXPAND_SC1
#define PE_EXPAND_SC1 1  // write-through expanded obs (expansion 7.85 -> 5.93 us, gather leg 20.45 -> 19.4; A/B: 0)
#endif
constexpr int kExpandPer = PE_EXPAND_PER;  // 4-code groups per thread (the table build amortized over them)
__global__ __launch_bounds__(256) void pe_expand_codes_kernel(const Tables* tab, int R, int G, int D, int rows,
                                                              const uint8_t* src, int64_t stride, float* obs,
                                                              float* rew, uint8_t* te, uint8_t* tr) {
  __shared__ float ctab[256];
  const CodeLd cld = obs_code_loads(tab, R, G, (int)threadIdx.x);  // (with the code loads: one round trip)
  const int b = blockIdx.y;
  const uint8_t* sb = src + (int64_t)b * stride;
  const int64_t nc = (int64_t)rows * D;  // codes per block
  float* ob = obs + (int64_t)b * nc;
  // a workgroup expands 256 * kExpandPer consecutive 4-code groups; thread t the groups
  // g0 + t + 256 j (each load and each 16-B store instruction contiguous over the wave),
  // every code word loaded before the table barrier
  const int64_t g0 = (int64_t)blockIdx.x * 256 * kExpandPer + threadIdx.x;
  if ((nc & 3) == 0) {
    uint32_t c[kExpandPer];
#pragma unroll
    for (int j = 0; j < kExpandPer; ++j) {
      const int64_t k = g0 + 256 * j;
      c[j] = 4 * k < nc ? *reinterpret_cast<const uint32_t*>(sb + 4 * k) : 0u;
    }
    ctab[threadIdx.x] = obs_code_pick(cld, R, G, (int)threadIdx.x);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kExpandPer; ++j) {
      const int64_t k = g0 + 256 * j;
      if (4 * k < nc) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        v4f v;
        v.x = ctab[c[j] & 255u];
        v.y = ctab[(c[j] >> 8) & 255u];
        v.z = ctab[(c[j] >> 16) & 255u];
        v.w = ctab[c[j] >> 24];
#if PE_EXPAND_SC1  // the expanded obs stream write-through, as the step kernels' tile stores
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(ob + 4 * k), "v"(v) : "memory");
#else
        *reinterpret_cast<v4f*>(ob + 4 * k) = v;
#endif
      }
    }
  } else {
    ctab[threadIdx.x] = obs_code_pick(cld, R, G, (int)threadIdx.x);
    __syncthreads();
    for (int j = 0; j < kExpandPer; ++j) {
      const int64_t k = g0 + 256 * j;
      for (int64_t i = 4 * k; i < 4 * k + 4 && i < nc; ++i) ob[i] = ctab[sb[i]];
    }
  }
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;  // the per-env outputs below
  // the per-env outputs: one env per thread of the first ceil(rows / 256) workgroups
  if (k < rows) {
    const int64_t ro = (nc + 15) & ~(int64_t)15;
    const int64_t o = (int64_t)b * rows + k;
    if (rew) rew[o] = reinterpret_cast<const float*>(sb + ro)[k];
    if (te) te[o] = sb[ro + 4 * (int64_t)rows + k];
    if (tr) tr[o] = sb[ro + 5 * (int64_t)rows + k];
  }
}

// ====================================================================== host side
#include "pe_handle.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(PE_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define PE_HIP(call)                                   \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return hip_fail(_e, #call);  \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Binds the handle's device for one API call and restores the caller's device
// afterwards (the library never leaves the calling thread on another device).
struct DeviceGuard {
  int prev = -1;
  int rc = PE_OK;
  explicit DeviceGuard(const pe_handle* h) {
    // hipGetLastError() reports the last failed runtime call of this thread,
    // whoever made it (torch probes, the caller's own calls): drop such a stale
    // error so the launch checks below see only this call's launches.
    (void)hipGetLastError();
    hipError_t e = hipGetDevice(&prev);
    if (e != hipSuccess) {
      rc = hip_fail(e, "hipGetDevice");
      prev = -1;
      return;
    }
    if (prev != h->device) {
      e = hipSetDevice(h->device);
      if (e != hipSuccess) rc = hip_fail(e, "hipSetDevice");
    } else {
      prev = -1;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

StepArgs base_args(const pe_handle* h) {
  StepArgs a;
  std::memset(&a, 0, sizeof(a));
  a.st = h->st;
  a.g = h->g;
  a.rl = h->rl;
  a.n = h->n;
  a.autoreset = h->cfg.autoreset;
  a.stagger = h->stagger;
  a.coop_max_done = h->coop_max_done;
  a.pf = h->pf;
  return a;
}

size_t lds_bytes(const Geo& g) {
  return sizeof(float) * (size_t)(kTabFloats + kBlock * g.DS) + align_up(2 * (size_t)g.C * g.R, 16);
}

// Step kernel variants.  The quadrant kernels (4 waves x 64 envs per workgroup)
// are the default for the specialized geometries (compile-time C, R: the LIDAR
// offsets of lidar_tables.inc); the one-lane-per-env kernels stay selectable
// (PE_STEP_KERNEL=lane, debug builds) for A/B measurement at C16R6 / C64R6.
// batch sizes up to which the headline kernel runs 16- / 32-env workgroups (quad_epb)
// (same-box A/B, profiles/r3b_ab_epb*.jsonl: 4096 envs 5.06 -> 4.55 us with 16-env
// workgroups, 8192: 16 ~ 32, 16384: 32 best, 32768: 32 ~ 64)
constexpr int kSmallBatch16 = 8192, kSmallBatch32 = 32768, kSmallBatch8W = 4096;
// The persistent pipelined kernel (pe_pipe.hpp) is compiled into debug builds only
// (PE_PIPE=P workgroups per CU): measured slower than pe_step_quad at every residency
// (same box, 65536 envs, profiles/r4b/ab_pipe.jsonl: quad 9.63 us, pipe P2 12.14, P3
// 11.71, P4 11.54; desynchronized 13.0 vs 23.5-25.4): at 2-3 workgroups per CU the
// compute phase runs at 2-3 waves per SIMD, and P4 spills (128 VGPRs + 47 spilled).

enum Variant {
  V_GENERIC = 0, V_C16R6_1W = 1, V_C16R6 = 2, V_C64R6 = 3,
  V_QUAD_C16R6_1W = 4, V_QUAD_C16R6 = 5, V_QUAD_C64R6 = 6,
  V_QUAD_C10R2_1W = 7, V_QUAD_C10R2 = 8,  // plantos_env.py:25-26 constructor default (G=21: multi-word)
  V_QUAD_C16R4_1W = 9, V_QUAD_C16R4 = 10,  // test_environment.py:24 (G=15, C=16, R=4)
  V_QUAD_RT_1W = 11, V_QUAD_RT = 12,       // runtime (C, R): every other geometry with C <= 64, 2 <= R <= 14
  V_FAR_C64R32 = 13                         // pe_step_far<64, 32>: SURVEY §8(d)'s R = 32 stress variant
};

// the prefetched records' obs row stride (bytes; pe_device.hpp Prefetch)
size_t pf_ostride(const Geo& g, bool codes) { return align_up((size_t)(codes ? g.D : 4 * g.D), 16); }

size_t quad_lds_bytes(const Geo& g, bool codes, bool rt) {
  const size_t off = (size_t)((kTabFloats + (2 * g.R + 3) * kQuadEnvs * 2 + 7 * kQuadEnvs + 3) & ~3) +
                     (rt ? (size_t)quad_rtab_floats(g.C, g.R) : 0);  // (+ the runtime kernel's probe table)
  // + the single-done record's LDS-DMA staging region (pe_coop.hpp pf_stage_issue)
  size_t stage = (size_t)pf_stage_bytes(g.G, g.WPR, (int)pf_ostride(g, codes));
  // (f32 kernels: the register-staged record and, beside it, the info wave's rows --
  // pe_step_quad kRegStage stages whenever the record fits one unit per lane)
  const int ng = pf_grid_units(g.G, g.WPR), no = (int)pf_ostride(g, codes) / 16;
  if (!codes && 1 + ng + no <= 64) stage = std::max(stage, (size_t)((1 + 2 * ng + no + 63) / 64) * 1024);
  // (byte-coded kernels that stage by LDS-DMA: the record, then the info wave's rows)
  if (codes && (rt || g.C >= PE_BT_STAGE_MIN_C) && ng <= 128)
    stage = std::max(stage, (size_t)((1 + 2 * ng + no + 63) / 64) * 1024);
  if (codes)  // byte tile + code table (quad_ctab_off)
    return sizeof(float) * (off + (size_t)((kQuadEnvs * g.D + 15) / 16) * 4 + 256) + stage;
  return sizeof(float) * (off + (size_t)kQuadEnvs * g.D) + stage;
}

bool is_quad(int v) { return v >= V_QUAD_C16R6_1W; }
bool is_far(int v) { return v == V_FAR_C64R32; }

// the step kernel's dynamic LDS (sector kernels)
size_t step_lds_bytes(const Geo& g, int variant, bool codes) {
  if (is_far(variant)) return sizeof(float) * (size_t)far_lds_floats(g.G, g.WPR, g.C, g.R);
  return quad_lds_bytes(g, codes, variant >= V_QUAD_RT_1W);
}

#ifdef PE_DEBUG_KNOBS
// the persistent pipelined kernel's grid and LDS: min(blocks, WPC per CU); the LDS
// request caps residency at WPC workgroups per CU (the grid assumes it)
int launch_pipe(const pe_handle* h, const StepArgs& a, hipStream_t s) {
  const int wpc = h->pipe_wpc;
  const int64_t nblk = ((int64_t)h->n + kQuadEnvs - 1) / kQuadEnvs;
  dim3 grid((unsigned)std::min<int64_t>(nblk, (int64_t)wpc * h->num_cus)), block(256);
  size_t lds = quad_lds_bytes(h->g, false, false);
  if (wpc < 4) lds = std::max(lds, (size_t)160 * 1024 / (wpc + 1) + 16);
  switch (wpc) {
    case 2: hipLaunchKernelGGL((pe_step_pipe<16, 6, 2>), grid, block, lds, s, a); break;
    case 3: hipLaunchKernelGGL((pe_step_pipe<16, 6, 3>), grid, block, lds, s, a); break;
    default: hipLaunchKernelGGL((pe_step_pipe<16, 6, 4>), grid, block, lds, s, a); break;
  }
  PE_HIP(hipGetLastError());
  return PE_OK;
}
#endif

int launch_step(const pe_handle* h, const StepArgs& a, hipStream_t s) {
#ifdef PE_DEBUG_KNOBS
  if (h->pipe_wpc > 0) return launch_pipe(h, a, s);
#endif
  if (is_far(h->variant)) {
    dim3 grid((unsigned)((h->n + kQuadEnvs - 1) / kQuadEnvs)), block(64 * kFarWaves);
    size_t lds = step_lds_bytes(h->g, h->variant, true);
    if (h->lds_floor > lds) lds = h->lds_floor;  // diagnostics: caps workgroups per CU
    hipLaunchKernelGGL((pe_step_far<64, 32>), grid, block, lds, s, a);
  } else if (is_quad(h->variant)) {
    const int nw = h->quad_waves, epb = h->quad_epb;
    dim3 grid((unsigned)((h->n + epb - 1) / epb)), block(nw * 64);
    size_t lds = step_lds_bytes(h->g, h->variant, h->tile_codes);
    if (h->lds_floor > lds) lds = h->lds_floor;  // diagnostics: caps workgroups per CU
#ifdef PE_DEBUG_KNOBS  // 8 waves of 64 envs: the PE_QUAD_WAVES=8 A/B only (they spill: never in the product)
#define PE_QUAD(CC, RR, OW)                                                                 \
  if (h->tile_codes)                                                                        \
    hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 4, true>), grid, block, lds, s, a);        \
  else if (nw == 8)                                                                         \
    hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 8>), grid, block, lds, s, a);              \
  else                                                                                      \
    hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 4>), grid, block, lds, s, a);
#else
#define PE_QUAD(CC, RR, OW)                                                                 \
  if (h->tile_codes)                                                                        \
    hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 4, true>), grid, block, lds, s, a);        \
  else                                                                                      \
    hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 4>), grid, block, lds, s, a);
#endif
#define PE_QUAD4(CC, RR, OW) hipLaunchKernelGGL((pe_step_quad<CC, RR, OW, 4>), grid, block, lds, s, a);
    switch (h->variant) {
      case V_QUAD_C16R6_1W:
        if (epb == 16 && !h->tile_codes && nw == 8)
          hipLaunchKernelGGL((pe_step_quad<16, 6, true, 8, false, 16>), grid, block, lds, s, a);
        else if (epb == 16 && !h->tile_codes)
          hipLaunchKernelGGL((pe_step_quad<16, 6, true, 4, false, 16>), grid, block, lds, s, a);
        else if (epb == 32 && !h->tile_codes)
          hipLaunchKernelGGL((pe_step_quad<16, 6, true, 4, false, 32>), grid, block, lds, s, a);
        else
          PE_QUAD(16, 6, true);
        break;
      case V_QUAD_C16R6:
#if PE_GR2
        if (h->gr2)
          hipLaunchKernelGGL((pe_step_quad<16, 6, false, 4, false, kQuadEnvs, true>), grid, block, lds, s, a);
        else
#endif
          PE_QUAD4(16, 6, false);
        break;
#ifdef PE_DEBUG_KNOBS
      case V_QUAD_C64R6: PE_QUAD(64, 6, false); break;  // (PE_TILE_CODES=0: the f32-tile A/B)
#else
      case V_QUAD_C64R6: hipLaunchKernelGGL((pe_step_quad<64, 6, false, 4, true>), grid, block, lds, s, a); break;
#endif
      case V_QUAD_C10R2_1W: PE_QUAD4(10, 2, true); break;
      case V_QUAD_C10R2: PE_QUAD4(10, 2, false); break;
      case V_QUAD_C16R4_1W: PE_QUAD4(16, 4, true); break;
      case V_QUAD_RT_1W:
        if (h->tile_codes)
          hipLaunchKernelGGL((pe_step_quad<0, 0, true, 4, true>), grid, block, lds, s, a);
        else
          PE_QUAD4(0, 0, true);
        break;
      case V_QUAD_RT:
        if (h->tile_codes)
          hipLaunchKernelGGL((pe_step_quad<0, 0, false, 4, true>), grid, block, lds, s, a);
        else
          PE_QUAD4(0, 0, false);
        break;
      default: PE_QUAD4(16, 4, false); break;
    }
#undef PE_QUAD
#undef PE_QUAD4
  } else {
    dim3 grid((unsigned)((h->n + kBlock - 1) / kBlock)), block(kBlock);
    size_t lds = lds_bytes(h->g);
    switch (h->variant) {
      case V_C16R6_1W: hipLaunchKernelGGL((pe_step_fast<16, 6, true>), grid, block, lds, s, a); break;
      case V_C16R6: hipLaunchKernelGGL((pe_step_fast<16, 6, false>), grid, block, lds, s, a); break;
      case V_C64R6: hipLaunchKernelGGL((pe_step_fast<64, 6, false>), grid, block, lds, s, a); break;
      default: {  // pe_step_wave: one wave per env
        const Geo& g = h->g;
        const size_t wlds = sizeof(float) * ((size_t)wave_hdr_floats(g.C, g.R, wave_aln_ok(g.G, g.R, g.WPR)) +
                                             kWaveEnvs * (size_t)wave_lds_floats(g.G, g.R, g.WPR, g.NW, g.D));
        dim3 wgrid((unsigned)((h->n + kWaveEnvs - 1) / kWaveEnvs)), wblock(64 * kWaveEnvs);
        const bool aln = wave_aln_ok(g.G, g.R, g.WPR);
        if (g.WPR == 1) {
          if (aln)
            hipLaunchKernelGGL((pe_step_wave<1, true>), wgrid, wblock, wlds, s, a);
          else
            hipLaunchKernelGGL((pe_step_wave<1, false>), wgrid, wblock, wlds, s, a);
        } else {
          if (aln)
            hipLaunchKernelGGL((pe_step_wave<kCoopWPR, true>), wgrid, wblock, wlds, s, a);
          else
            hipLaunchKernelGGL((pe_step_wave<kCoopWPR, false>), wgrid, wblock, wlds, s, a);
        }
        break;
      }
    }
  }
  PE_HIP(hipGetLastError());
  return PE_OK;
}

// The prefetch launches (pe_prefetch_kernel): queue mode on one resident grid
// (h->pf_blocks: every workgroup the chip holds at once; a steady-state batch of K
// steps' resets, ~65 K envs at 65536 envs, is about one map per wave), all mode
// with one wave per env.
int launch_prefetch(const pe_handle* h, hipStream_t s, int all) {
  StepArgs a = base_args(h);
  const unsigned nb = (unsigned)((h->n + 3) / 4);
  dim3 grid(all ? nb : std::min(nb, (unsigned)h->pf_blocks)), block(256);
  if (!all) {
    hipLaunchKernelGGL(pe_pf_compact_kernel, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, s, h->pf, h->n);
    PE_HIP(hipGetLastError());
  }
  const size_t lds = sizeof(float) * (size_t)kTabFloats + 4 * 8 * (size_t)coop_scratch_words(h->g.G, h->g.WPR);
  if (h->g.WPR == 1) {
    if (h->tile_codes)
      hipLaunchKernelGGL((pe_prefetch_kernel<1, true>), grid, block, lds, s, a, all);
    else
      hipLaunchKernelGGL((pe_prefetch_kernel<1, false>), grid, block, lds, s, a, all);
  } else {
    if (h->tile_codes)
      hipLaunchKernelGGL((pe_prefetch_kernel<kCoopWPR, true>), grid, block, lds, s, a, all);
    else
      hipLaunchKernelGGL((pe_prefetch_kernel<kCoopWPR, false>), grid, block, lds, s, a, all);
  }
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int launch_reset(const pe_handle* h, const StepArgs& a, hipStream_t s) {
  if (h->coop_max_done > 0) {  // the cooperative reset applies (pe_coop.hpp coop_reset_ok)
    dim3 cgrid((unsigned)((h->n + 3) / 4)), cblock(256);
    const size_t clds = sizeof(float) * (size_t)kTabFloats + 4 * 8 * (size_t)coop_scratch_words(h->g.G, h->g.WPR);
    if (h->g.WPR == 1)
      hipLaunchKernelGGL(pe_reset_coop_kernel<1>, cgrid, cblock, clds, s, a);
    else
      hipLaunchKernelGGL(pe_reset_coop_kernel<kCoopWPR>, cgrid, cblock, clds, s, a);
    PE_HIP(hipGetLastError());
    return PE_OK;
  }
  dim3 grid((unsigned)((h->n + kBlock - 1) / kBlock)), block(kBlock);
  size_t lds = lds_bytes(h->g);
  hipLaunchKernelGGL(pe_reset_kernel, grid, block, lds, s, a);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

template <int C, int R>
bool table_matches(const int8_t* dx, const int8_t* dy) {
  for (int i = 0; i < C; ++i)
    for (int r = 0; r < R; ++r)
      if (LidarTab<C, R>::dx[i][r] != dx[i * R + r] || LidarTab<C, R>::dy[i][r] != dy[i * R + r]) return false;
  return true;
}

const char* variant_name(int v) {
  switch (v) {
    case V_C16R6_1W: return "pe_step_fast<C16,R6,1word>";
    case V_C16R6: return "pe_step_fast<C16,R6>";
    case V_C64R6: return "pe_step_fast<C64,R6>";
    case V_QUAD_C16R6_1W: return "pe_step_quad<C16,R6,1word>";
    case V_QUAD_C16R6: return "pe_step_quad<C16,R6>";
    case V_QUAD_C64R6: return "pe_step_quad<C64,R6>";
    case V_QUAD_C10R2_1W: return "pe_step_quad<C10,R2,1word>";
    case V_QUAD_C10R2: return "pe_step_quad<C10,R2>";
    case V_QUAD_C16R4_1W: return "pe_step_quad<C16,R4,1word>";
    case V_QUAD_C16R4: return "pe_step_quad<C16,R4>";
    case V_QUAD_RT_1W: return "pe_step_quad<runtime C,R,1word>";
    case V_QUAD_RT: return "pe_step_quad<runtime C,R>";
    case V_FAR_C64R32: return "pe_step_far<C64,R32>";
    default: return "pe_step_wave";
  }
}

}  // namespace

extern "C" {

void pe_default_config(pe_config* c, int32_t G, int32_t P, int32_t O, int32_t R, int32_t C) {
  std::memset(c, 0, sizeof(*c));
  c->abi_version = PE_ABI_VERSION;
  c->grid_size = G;
  c->num_plants = P;
  c->num_obstacles = O;
  c->lidar_range = R;
  c->lidar_channels = C;
  c->max_steps = 1000;             // plantos_env.py:120
  c->autoreset = 1;                // DummyVecEnv semantics
  c->thirsty_plant_prob = 0.7;     // plantos_env.py:26
  c->r_goal = 20;                  // plantos_env.py:76-83
  c->r_mistake = -10;
  c->r_invalid = -5;
  c->r_water_empty = -5;
  c->r_step = -0.1;
  c->r_exploration = 10;
  c->r_revisit = -1;
  c->r_complete = 50;
  c->seed = 0;
  c->env_id_offset = 0;
  c->coop_max_done = -1;           // the library's choice per geometry
  c->prefetch_every = -1;
}

int32_t pe_obs_dim(const pe_config* c) { return c->lidar_channels * 5 + 2 + 25; }

const char* pe_last_error(void) { return g_err.c_str(); }

int pe_internal_set_error(int code, const char* msg) { return fail(code, msg); }

int pe_create(const pe_config* c, int32_t device, int32_t n_envs, pe_handle** out) {
  if (!c || !out) return fail(PE_ERR_ARG, "null argument");
  *out = nullptr;
  if (c->abi_version != PE_ABI_VERSION) return fail(PE_ERR_ARG, "ABI version mismatch");
  const int G = c->grid_size, R = c->lidar_range, C = c->lidar_channels, P = c->num_plants, O = c->num_obstacles;
  if (G < 1 || G > 128) return fail(PE_ERR_ARG, "grid_size must be in [1, 128]");
  if (R < 1 || R > 64) return fail(PE_ERR_ARG, "lidar_range must be in [1, 64]");
  if (C < 1 || C > 256) return fail(PE_ERR_ARG, "lidar_channels must be in [1, 256]");
  if (P < 0 || P >= G * G) return fail(PE_ERR_ARG, "num_plants must be in [0, G*G)");
  if (O < 0) return fail(PE_ERR_ARG, "num_obstacles must be >= 0");
  if (O / 3 > 0 && G < 5) return fail(PE_ERR_ARG, "randint(2, G-3) needs grid_size >= 5 (plantos_env.py:344)");
  if (c->max_steps < 1 || c->max_steps > 65535) return fail(PE_ERR_ARG, "max_steps must be in [1, 65535]");
  if (c->map_generation_algo != PE_MAP_ORIGINAL && c->map_generation_algo != PE_MAP_MAZE)
    return fail(PE_ERR_ARG, "map_generation_algo must be PE_MAP_ORIGINAL or PE_MAP_MAZE");
  if (c->map_generation_algo == PE_MAP_MAZE && G < 7)
    return fail(PE_ERR_ARG, "the maze needs grid_size >= 7 (randint(0, (G-1)//6 - 1), plantos_env_new.py:427)");
  if (n_envs < 1) return fail(PE_ERR_ARG, "n_envs must be >= 1");
  if (2 * (G + 2 * R) > 64 * kMaxWPR) return fail(PE_ERR_ARG, "G + 2R too large");

  int ndev = 0;
  hipError_t he = hipGetDeviceCount(&ndev);
  if (he != hipSuccess || ndev == 0) return fail(PE_ERR_DEVICE, "no HIP device available (no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(PE_ERR_ARG, "bad device index");
  (void)hipGetLastError();  // stale error of an earlier call (see DeviceGuard)
  struct Restore {
    int prev = -1;
    ~Restore() {
      if (prev >= 0) (void)hipSetDevice(prev);
    }
  } restore;
  PE_HIP(hipGetDevice(&restore.prev));
  PE_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  PE_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(PE_ERR_DEVICE, std::string("built for gfx950, device is ") + prop.gcnArchName);

  pe_handle* h = new (std::nothrow) pe_handle();
  if (!h) return fail(PE_ERR_NOMEM, "host allocation failed");
  h->device = device;
  h->n = n_envs;
  h->cfg = *c;
  Geo& g = h->g;
  g.G = G;
  g.C = C;
  g.R = R;
  g.D = 5 * C + 27;
  g.DS = g.D | 1;
  g.GG = G * G;
  g.WPR = (2 * (G + 2 * R) + 63) / 64;
  // visit row words: the padded row's G+4 nibbles + a spare word, so that the 8-nibble
  // window starting at any padded column y-1 (words vw, vw+1) stays inside the row.
  // (Tried: 4 words up to G = 25 -- 16-B rows, one load per window row in the
  // multi-word kernel: 25x25 10.38 -> 10.97 us, 21x21/C10/R2 one-word 8.05 -> 8.14;
  // profiles/r3j_ab_*.jsonl.)
  g.NW = (4 * (G + 4) + 31) / 32 + 1;
  if (g.NW < 4) g.NW = 4;  // 16-B visit rows: one dwordx4 per row in the sector kernel
  g.EW = (g.GG + 31) / 32;
  g.gstride = (int64_t)align_up((size_t)G * g.WPR, 2);  // 16-B aligned env blocks (row-pair loads)
  // two visit slots per env, 16-B aligned (episode k's visits in slot k & 1: pe_device.hpp vis_env)
  g.vslot = (int64_t)align_up((size_t)G * g.NW, 4);
  g.vstride = 2 * g.vslot;
  g.hstride = (int64_t)align_up((size_t)g.GG, 8);
  // explored words; also the picks scratch of a curriculum reset that keeps visits
  g.estride = (int64_t)align_up((size_t)std::max(g.EW, (P + 1) / 2), 4);
  // LDS limits: the lane-per-env kernels that every geometry keeps (pe_load_maps_kernel,
  // and pe_reset_kernel where the cooperative reset does not apply) hold a [64 x D]
  // obs tile -- this caps C at 120 whatever the step kernel; the one-wave-per-env step
  // kernel (the step kernel of every geometry without a sector kernel) its header +
  // 8 per-wave regions.
  if (lds_bytes(g) > 160 * 1024) {
    delete h;
    return fail(PE_ERR_ARG, "observation tile does not fit LDS (lidar_channels <= 120)");
  }
  if (sizeof(float) * ((size_t)wave_hdr_floats(C, R, wave_aln_ok(G, R, g.WPR)) + kWaveEnvs * (size_t)wave_lds_floats(G, R, g.WPR, g.NW, g.D)) >
      160 * 1024) {
    delete h;
    return fail(PE_ERR_ARG, "the one-wave-per-env step kernel's window does not fit LDS");
  }

  Rules& rl = h->rl;
  rl.r_goal = c->r_goal;
  rl.r_mistake = c->r_mistake;
  rl.r_invalid = c->r_invalid;
  rl.r_water_empty = c->r_water_empty;
  rl.r_step = c->r_step;
  rl.r_exploration = c->r_exploration;
  rl.r_revisit = c->r_revisit;
  rl.r_complete = c->r_complete;
  rl.p_thirsty = c->thirsty_plant_prob;
  rl.seed = c->seed;
  rl.env_off = c->env_id_offset;
  rl.P = P;
  rl.O = O;
  rl.map_algo = c->map_generation_algo;
  // Auto-resets in the step kernel: wave-cooperative (pe_coop.hpp: one env at a
  // time per wave, ~10 us each at 20x20) when a block has few done envs; one lane
  // per env (all of a wave's envs at once, ~0.26 ms for a whole batch at 20x20)
  // when many are done together -- unless the lane path would have to scan its
  // grid image in HBM (no room for it in the obs-tile row), where it is ~30x
  // slower (29 ms for a whole 64x64 batch) and the cooperative path always wins.
  if (!coop_reset_ok(G, R, g.WPR, g.NW, P, C, c->map_generation_algo))
    h->coop_max_done = 0;
  else if (reset_scratch_bytes(G, g.WPR, P) <= 4 * g.D)
    h->coop_max_done = kCoopMaxDone;
  else
    h->coop_max_done = kQuadEnvs;
  rl.max_steps = c->max_steps;

  // host tables
  Tables tab;
  std::memset(&tab, 0, sizeof(tab));
  for (int r = 0; r <= R; ++r) tab.dist[r] = (float)((double)r / (double)R);
  for (int x = 0; x < G; ++x) tab.pos[x] = (float)((double)x / (double)G);
  for (int v = 0; v < 16; ++v) tab.vis[v] = (float)((double)(v < 10 ? v : 10) / 10.0);
  for (int p = 0; p < G + 2 * R; ++p) {
    int w = (2 * p) / 64, b = (2 * p) % 64;
    if (p < R || p >= G + R)
      tab.grid_pad[w] |= 1ull << b;
    else
      tab.grid_real[w] |= 1ull << b;
  }
  for (int p = 0; p < G + 4; ++p)
    if (p < 2 || p >= G + 2) tab.vis_pad[(4 * p) / 32] |= 10u << ((4 * p) % 32);
  const size_t nl = (size_t)C * R;
  int8_t* ldx = new int8_t[nl];
  int8_t* ldy = new int8_t[nl];
  const double pi = 3.141592653589793;  // math.pi; plantos_env.py:261-267
  for (int i = 0; i < C; ++i) {
    double angle = ((2.0 * pi) * (double)i) / (double)C;
    for (int r = 1; r <= R; ++r) {
      ldx[i * R + r - 1] = (int8_t)(int)((double)r * std::cos(angle));
      ldy[i * R + r - 1] = (int8_t)(int)((double)r * std::sin(angle));
    }
  }
  h->variant = V_GENERIC;
  if (C == 16 && R == 6 && table_matches<16, 6>(ldx, ldy)) h->variant = g.WPR == 1 ? V_C16R6_1W : V_C16R6;
  if (C == 64 && R == 6 && table_matches<64, 6>(ldx, ldy)) h->variant = V_C64R6;
  // A/B knobs of the measurement tools (tools/ab_build.sh builds a SEPARATE library
  // with -DPE_DEBUG_KNOBS); the product library reads no environment variable.
  bool lane_kernels = false;
  h->quad_waves = 4;  // measured best at C=16 and C=64 (profiles/r1c-r1e)
  h->stagger = 0;
  h->lds_floor = 0;
#ifdef PE_DEBUG_KNOBS
  if (const char* kenv = std::getenv("PE_STEP_KERNEL")) lane_kernels = std::strcmp(kenv, "lane") == 0;
  if (const char* qw = std::getenv("PE_QUAD_WAVES")) h->quad_waves = std::atoi(qw) == 8 ? 8 : 4;
  if (const char* sg = std::getenv("PE_STAGGER")) h->stagger = std::atoi(sg);
  if (const char* lf = std::getenv("PE_LDS_FLOOR")) h->lds_floor = std::min<size_t>(std::strtoul(lf, nullptr, 10), 160 * 1024);
#endif
  if (!lane_kernels && h->variant != V_GENERIC) h->variant += V_QUAD_C16R6_1W - V_C16R6_1W;
  // sector kernels of the other specialized geometries (4 waves; no lane-kernel twin)
  if (!lane_kernels && C == 10 && R == 2 && table_matches<10, 2>(ldx, ldy)) h->variant = V_QUAD_C10R2_1W;
  if (!lane_kernels && C == 16 && R == 4 && table_matches<16, 4>(ldx, ldy)) h->variant = V_QUAD_C16R4_1W;
  // R > 14 with a compile-time table: the far sector kernel (its rows and the auto-reset
  // path's are kCoopWPR words: 96 < G + 2R <= 128)
  if (!lane_kernels && C == 64 && R == 32 && g.WPR == kCoopWPR && table_matches<64, 32>(ldx, ldy))
    h->variant = V_FAR_C64R32;
  // the one-word form (whole padded row in one u64) needs WPR == 1 and 16-B visit
  // rows (NW == 4: G <= 20); otherwise the multi-word (funnel-shifted) form
  const bool oneword = g.WPR == 1 && g.NW == 4;
  if ((h->variant == V_QUAD_C10R2_1W || h->variant == V_QUAD_C16R4_1W) && !oneword) h->variant += 1;
  // every other geometry with 4 <= C <= 32 and 2 <= R <= 14: the sector kernel with
  // table-driven rays (quad_rays_rt) instead of one wave per env -- 64 envs per
  // workgroup share the per-env work the wave kernel repeats per wave
  // (33 <= C <= 64: with the byte-coded tile, below)
  if (!lane_kernels && h->variant == V_GENERIC && C >= 4 && C <= kRtCMaxBT && R >= 2 && R <= kRtRMax)
    h->variant = oneword ? V_QUAD_RT_1W : V_QUAD_RT;
  // the sector kernels of these geometries (and the runtime-(C, R) one) exist with 4 waves only
  if (h->variant >= V_QUAD_C10R2_1W) h->quad_waves = 4;
  if (h->variant == V_QUAD_C16R6_1W && g.NW != 4) h->variant = V_C16R6_1W;  // needs 16-B visit rows
  // byte-coded obs tile where the f32 tile limits the sector kernel's occupancy
  // (C = 64: 89 KB -> 22 KB of LDS per workgroup)
  h->tile_codes = h->variant == V_QUAD_C64R6 || is_far(h->variant) ||
                          (is_quad(h->variant) && h->variant >= V_QUAD_RT_1W && C > kRtCMax)
                      ? 1 : 0;
  // the runtime kernel with C <= 32 too, where its f32 tile holds fewer workgroups per CU than
  // the byte tile and the batch needs more than one round of them (32x32 / C24 / R9: 54 KB, two
  // per CU -- 65536 envs ran as two waves of workgroups, the second starting ~13 us in,
  // profiles/r5s/stamps_g32.json); small batches keep the f32 tile (no expansion at the store)
  if (!h->tile_codes && is_quad(h->variant) && h->variant >= V_QUAD_RT_1W) {
    auto per_cu = [](size_t l) { return std::min<size_t>(4, (size_t)160 * 1024 / l); };
    const size_t lf = quad_lds_bytes(g, false, true), lb = quad_lds_bytes(g, true, true);
    const int64_t blocks = ((int64_t)n_envs + kQuadEnvs - 1) / kQuadEnvs;
    if (per_cu(lb) > per_cu(lf) && blocks > (int64_t)prop.multiProcessorCount * (int64_t)per_cu(lf)) h->tile_codes = 1;
  }
#ifdef PE_DEBUG_KNOBS
  if (const char* tc = std::getenv("PE_TILE_CODES"))
    if (h->variant == V_QUAD_C16R6_1W || h->variant == V_QUAD_C64R6) h->tile_codes = std::atoi(tc) != 0;
#endif
  // obs as byte codes at the boundary (pe_step_codes): the byte-coded tile kernels
  h->obs_codes = c->obs_codes ? 1 : 0;
  if (h->obs_codes) {
    if (!(h->variant == V_QUAD_C16R6_1W || h->variant == V_QUAD_C64R6 || h->variant == V_QUAD_RT_1W ||
          h->variant == V_QUAD_RT || is_far(h->variant))) {
      delete[] ldx;
      delete[] ldy;
      delete h;
      return fail(PE_ERR_ARG, "obs_codes needs a byte-coded sector kernel (C=16/R=6 with G<=20, C=64/R=6, or "
                              "4<=C<=64 with 2<=R<=14 and no compile-time kernel)");
    }
    h->tile_codes = 1;
  }
  if (h->tile_codes) {
    h->quad_waves = 4;
    // (not the byte-coded C16 kernel -- config 5's codes step: its quarters started apart
    // cost it ~0.9 us desynchronized, 11.68 -> 10.75 us without, profiles/r6c/ab_codesstag;
    // the runtime byte-tile kernel keeps it: 32x32/C24/R9 17.0 -> 18.1 us without)
    // all 1024 workgroups of a 65536-env batch are resident at once (4 per CU) and
    // would run their load, compute and 89-KB store phases in lockstep: starting the
    // grid's quarters ~0.85 us apart overlaps one quarter's stores with the next
    // one's loads (64x64 / 64 rays, same-box: 28.7 -> 26.3 us; 2x that: 27.0)
    // (the far kernel: 8 -- 52.8 -> 52.1 us, desynchronized unchanged, profiles/r6d/ab_farstag)
    h->stagger = h->variant == V_QUAD_C16R6_1W ? 0 : (is_far(h->variant) ? 8 : 4);
  }
#ifdef PE_DEBUG_KNOBS
  if (const char* sg = std::getenv("PE_STAGGER")) h->stagger = std::atoi(sg);
#endif
  if (is_quad(h->variant) && step_lds_bytes(g, h->variant, h->tile_codes) > 160 * 1024)
    h->variant = h->variant <= V_QUAD_C64R6 ? h->variant - (V_QUAD_C16R6_1W - V_C16R6_1W) : V_GENERIC;
#ifdef PE_DEBUG_KNOBS
  if (const char* kenv = std::getenv("PE_STEP_KERNEL"))
    if (std::strcmp(kenv, "wave") == 0) h->variant = V_GENERIC;  // A/B: the one-wave-per-env kernel
#endif
  if (!is_quad(h->variant)) h->tile_codes = 0;
  if (h->obs_codes && !h->tile_codes) {
    delete[] ldx;
    delete[] ldy;
    delete h;
    return fail(PE_ERR_ARG, "obs_codes: the byte-coded tile does not fit this geometry");
  }
  // envs per workgroup: a batch too small to give every CU four 64-env workgroups
  // (1024 at 65536 envs) is cut into 16- or 32-env workgroups instead, so that it
  // still spreads over all 256 CUs (headline geometry's kernel only; 4 waves, f32 tile)
  // (up to 4096 envs: 8 waves x 16 envs -- two waves per SIMD on every CU, sectors of 2
  // rays: 2048 envs 4.56 -> 4.41 us, 4096 4.56 -> 4.49; 8192 4.82 -> 4.98 us, kept at 4)
  h->quad_epb = kQuadEnvs;
  if (h->variant == V_QUAD_C16R6_1W && !h->tile_codes && h->quad_waves == 4) {
    h->quad_epb = n_envs <= kSmallBatch16 ? 16 : (n_envs <= kSmallBatch32 ? 32 : kQuadEnvs);
    if (n_envs <= kSmallBatch8W) h->quad_waves = 8;
  }
#ifdef PE_DEBUG_KNOBS
  if (const char* ep = std::getenv("PE_QUAD_EPB"))
    if (h->variant == V_QUAD_C16R6_1W && !h->tile_codes) {
      const int v = std::atoi(ep);
      h->quad_epb = v == 16 || (v == 32 && h->quad_waves == 4) ? v : kQuadEnvs;  // 8 waves: 16 or 64
    }
#endif
  h->num_cus = prop.multiProcessorCount;
  h->pipe_wpc = 0;
#ifdef PE_DEBUG_KNOBS
  // the persistent pipelined kernel (pe_pipe.hpp, A/B): the headline geometry's 64-env,
  // 4-wave, f32-tile kernel at batches that fill the chip
  if (const char* pp = std::getenv("PE_PIPE"))
    h->pipe_wpc = n_envs > kSmallBatch32 ? std::min(std::max(std::atoi(pp), 0), 4) : 0;
#endif
  if (h->pipe_wpc == 1) h->pipe_wpc = 2;
  if (!(h->variant == V_QUAD_C16R6_1W && h->quad_epb == kQuadEnvs && h->quad_waves == 4 && !h->tile_codes))
    h->pipe_wpc = 0;
  h->kname = variant_name(h->variant);
  if (h->pipe_wpc > 0) {
    std::snprintf(h->kname_buf, sizeof(h->kname_buf), "pe_step_pipe<C16,R6,1word,P%d>", h->pipe_wpc);
    h->kname = h->kname_buf;
  }
  if (h->quad_epb != kQuadEnvs) {
    std::snprintf(h->kname_buf, sizeof(h->kname_buf), "%.*s%s,E%d>", (int)std::strlen(h->kname) - 1, h->kname,
                  h->quad_waves == 8 ? ",W8" : "", h->quad_epb);
    h->kname = h->kname_buf;
  } else if (h->tile_codes) {  // the byte-coded tile instantiation (pe_step_quad<..., BT = true>)
    std::snprintf(h->kname_buf, sizeof(h->kname_buf), "%.*s,bytetile>", (int)std::strlen(h->kname) - 1, h->kname);
    h->kname = h->kname_buf;
  }
  // the two-word kernel with the loader env's whole grid block in round 1 (pe_step_quad GR2)
  h->gr2 = PE_GR2 && h->variant == V_QUAD_C16R6 && g.WPR == 2 && G <= kGr2MaxG && !h->tile_codes &&
           h->quad_waves == 4 && h->quad_epb == kQuadEnvs;
  if (h->gr2) h->kname = "pe_step_quad<C16,R6,gridr1>";
  // explicit reset-path tuning (pe_config.coop_max_done; -1: the choice above) --
  // applied before the prefetch decision, which depends on it
  if (c->coop_max_done >= 0 && coop_reset_ok(G, R, g.WPR, g.NW, P, C, c->map_generation_algo))
    h->coop_max_done = std::min(c->coop_max_done, kQuadEnvs);
  // Prefetched resets (pe_coop.hpp Prefetch) where the sector kernel takes the
  // cooperative path.  The done-count threshold above stays: a whole block done at
  // once (a synchronized batch truncating) is cheaper through the lane-per-env path,
  // which consumes no record and so queues no regeneration (20x20: 0.26 ms per
  // batch reset, against 0.09 ms for the copies + ~0.3 ms to regenerate 65536 maps).
  h->pf_every = c->prefetch_every >= 0 ? c->prefetch_every : kPrefetchEvery;
  if (!(is_quad(h->variant) || h->variant == V_GENERIC) || h->coop_max_done <= 0 || !c->autoreset) h->pf_every = 0;

  // one device allocation carved into 256-B aligned arrays
  const size_t n = (size_t)n_envs;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t o_tab = carve(sizeof(Tables));
  const size_t o_ldx = carve(nl), o_ldy = carve(nl);
  const int RP = (R + 7) & ~7;
  const bool wave_aln = h->variant == V_GENERIC && wave_aln_ok(G, R, g.WPR);  // pe_step_wave<., true>
  const bool rt_tab = h->variant == V_QUAD_RT_1W || h->variant == V_QUAD_RT;  // u32 probe entries (quad_rays_rt)
  // (rt_tab: the LDS-form entries, then the register-window header [4][4] and entries, pe_quad.hpp)
  const size_t o_ldxy = carve(wave_aln ? ((size_t)C * RP * 3 + 15) & ~(size_t)15
                                       : (rt_tab ? (2 * (size_t)C * RP + 16) * 4 : (size_t)C * RP * 2));
  const size_t o_err = carve(sizeof(uint32_t));
  const size_t o_scal = carve(n * sizeof(uint4));
  const size_t o_ret = carve(n * sizeof(double));
  const size_t o_grid = carve(n * (size_t)g.gstride * 8);
  const size_t o_vis = carve(n * (size_t)g.vstride * 4);
  const size_t o_vx = carve(n * (size_t)g.hstride * 4);
  const size_t o_vpend = carve(n * sizeof(uint32_t));
  const size_t o_expl = carve(n * (size_t)g.estride * 4);
  h->bytes = off;
  if (is_far(h->variant)) {
    // pe_step_far loads a quadrant's off-map rows UNCLAMPED (pe_far.hpp far_sector: up to
    // R rows before the env's grid block and R rows + one raw word after it, selected away
    // afterwards): the first env's must land in the arrays carved before the grid, the last
    // env's in those after it -- inside this one allocation
    const size_t row_b = (size_t)kFarRow32 * 4, grid_end = o_grid + n * (size_t)g.gstride * 8;
    if (g.WPR != kCoopWPR || o_grid < (size_t)R * row_b || h->bytes - grid_end < (size_t)(R + 1) * row_b) {
      delete[] ldx;
      delete[] ldy;
      delete h;
      return fail(PE_ERR_ARG, "pe_step_far: the allocation leaves less than R padded grid rows of slack around the "
                              "grid array (its off-map row loads would leave the allocation)");
    }
  }
  hipError_t me = hipMalloc(&h->mem, h->bytes);
  if (me != hipSuccess) {
    delete[] ldx;
    delete[] ldy;
    delete h;
    return fail(PE_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(me));
  }
  char* base = static_cast<char*>(h->mem);
  h->st.tab = reinterpret_cast<const Tables*>(base + o_tab);
  h->st.ldx = reinterpret_cast<const signed char*>(base + o_ldx);
  h->st.ldy = reinterpret_cast<const signed char*>(base + o_ldy);
  h->st.ldxy = reinterpret_cast<const int16_t*>(base + o_ldxy);
  h->st.err_bits = reinterpret_cast<uint32_t*>(base + o_err);
  h->st.scal = reinterpret_cast<uint4*>(base + o_scal);
  h->st.ep_ret = reinterpret_cast<double*>(base + o_ret);
  h->st.grid = reinterpret_cast<uint64_t*>(base + o_grid);
  h->st.vis = reinterpret_cast<uint32_t*>(base + o_vis);
  h->st.vx = reinterpret_cast<uint32_t*>(base + o_vx);
  h->st.vpend = reinterpret_cast<uint32_t*>(base + o_vpend);
  h->st.expl = reinterpret_cast<uint32_t*>(base + o_expl);
  int rc = PE_OK;
  if (h->pf_every > 0) {
    size_t po = 0;
    auto pcarve = [&](size_t bytes) {
      size_t o = po;
      po = align_up(po + bytes, 256);
      return o;
    };
    const size_t p_scal = pcarve(n * sizeof(uint4)), p_grid = pcarve(n * (size_t)g.gstride * 8);
    const uint32_t ostride = (uint32_t)pf_ostride(g, h->tile_codes);
    const size_t p_obs = pcarve(n * (size_t)ostride), p_q = pcarve(n * 4), p_qn = pcarve(2 * 4);
    const size_t p_flag = pcarve(n);
    if (hipMalloc(&h->pf_mem, po) != hipSuccess || hipMemset(h->pf_mem, 0, po) != hipSuccess) {
      if (h->pf_mem) (void)hipFree(h->pf_mem);
      (void)hipFree(h->mem);
      delete[] ldx;
      delete[] ldy;
      delete h;
      return fail(PE_ERR_NOMEM, "prefetch buffers: hipMalloc failed");
    }
    char* pb = static_cast<char*>(h->pf_mem);
    h->pf.scal = reinterpret_cast<uint4*>(pb + p_scal);
    h->pf.grid = reinterpret_cast<uint64_t*>(pb + p_grid);
    h->pf.obs = reinterpret_cast<float*>(pb + p_obs);
    h->pf.ostride = ostride;
    h->pf.queue = reinterpret_cast<uint32_t*>(pb + p_q);
    h->pf.qn = reinterpret_cast<uint32_t*>(pb + p_qn);
    h->pf.flag = reinterpret_cast<uint8_t*>(pb + p_flag);
    const size_t plds = sizeof(float) * (size_t)kTabFloats + 4 * 8 * (size_t)coop_scratch_words(G, g.WPR);
    int per_cu = 0;
    hipError_t oe = g.WPR == 1
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pe_prefetch_kernel<1, false>, 256, plds)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pe_prefetch_kernel<kCoopWPR, false>, 256, plds);
    if (oe != hipSuccess || per_cu < 1) per_cu = 1;
    h->pf_blocks = per_cu * prop.multiProcessorCount;
  }
  hipError_t e1 = hipMemset(h->mem, 0, h->bytes);
  hipError_t e2 = hipMemcpy(base + o_tab, &tab, sizeof(Tables), hipMemcpyHostToDevice);
  hipError_t e3 = hipMemcpy(base + o_ldx, ldx, nl, hipMemcpyHostToDevice);
  hipError_t e4 = hipMemcpy(base + o_ldy, ldy, nl, hipMemcpyHostToDevice);
  std::vector<int16_t> ldxy((size_t)C * RP, 0);
  for (int i = 0; i < C; ++i)
    for (int r = 0; r < R; ++r)
      ldxy[(size_t)i * RP + r] = (int16_t)((uint8_t)ldx[i * R + r] | ((int)ldy[i * R + r] << 8));
  hipError_t e5;
  if (wave_aln) {  // pe_step_wave<., true>'s LDS header entries: [C][RP] u16 byte offsets into
                   // the aligned window, then [C][RP] u8 bit shifts
    std::vector<uint8_t> aln(((ldxy.size() * 3 + 15) & ~(size_t)15), 0);
    for (size_t k = 0; k < ldxy.size(); ++k) {
      const uint32_t en = aln_entry((uint16_t)ldxy[k], R, (4 * R + 33) >> 5);
      const uint16_t off = (uint16_t)(4u * (en & 0x7FFu));
      std::memcpy(aln.data() + 2 * k, &off, 2);
      aln[2 * ldxy.size() + k] = (uint8_t)((en >> 11) & 31u);
    }
    e5 = hipMemcpy(base + o_ldxy, aln.data(), aln.size(), hipMemcpyHostToDevice);
  } else if (rt_tab) {  // the runtime sector kernel's entries (pe_quad.hpp quad_rays_rt): the probe's LDS
                        // byte offset from the rover row (dx rows of 64 envs x 8 B) | its bit shift 2(dy+R) << 16
    std::vector<uint32_t> rt(2 * (size_t)C * RP + 16, 0u);
    for (int i = 0; i < C; ++i)
      for (int r = 0; r < R; ++r)
        rt[(size_t)i * RP + r] = (uint32_t)(uint16_t)(int16_t)(ldx[i * R + r] * kQuadEnvs * 8) |
                                 ((uint32_t)(2 * (ldy[i * R + r] + R)) << 16);
    // the register-window form (pe_quad.hpp quad_rays_rt_reg): per wave w (rays [wC/4, (w+1)C/4))
    // the header {LO, DLO, NROWS, ok}, per probe (dx - LO) | 2(dy - DLO) << 8
    uint32_t* hdr = rt.data() + (size_t)C * RP;
    uint32_t* ent = hdr + 16;
    for (int w = 0; w < 4; ++w) {
      const int i0 = w * C / 4, i1 = (w + 1) * C / 4;
      int lo = 1 << 20, hi = -(1 << 20), dlo = 1 << 20, dhi = -(1 << 20);
      for (int i = i0; i < i1; ++i)
        for (int r = 0; r < R; ++r) {
          lo = std::min(lo, (int)ldx[i * R + r]);
          hi = std::max(hi, (int)ldx[i * R + r]);
          dlo = std::min(dlo, (int)ldy[i * R + r]);
          dhi = std::max(dhi, (int)ldy[i * R + r]);
        }
      const bool ok = i1 > i0 && hi - lo + 1 <= kRtRegRows && dhi - dlo + 1 <= 16;
      hdr[4 * w] = (uint32_t)lo;
      hdr[4 * w + 1] = (uint32_t)dlo;
      hdr[4 * w + 2] = (uint32_t)(hi - lo + 1);
      hdr[4 * w + 3] = ok ? 1u : 0u;
      if (ok)
        for (int i = i0; i < i1; ++i)
          for (int r = 0; r < R; ++r)
            ent[(size_t)i * RP + r] = (uint32_t)(ldx[i * R + r] - lo) | ((uint32_t)(2 * (ldy[i * R + r] - dlo)) << 8);
    }
    e5 = hipMemcpy(base + o_ldxy, rt.data(), rt.size() * 4, hipMemcpyHostToDevice);
  } else {
    e5 = hipMemcpy(base + o_ldxy, ldxy.data(), ldxy.size() * 2, hipMemcpyHostToDevice);
  }
  delete[] ldx;
  delete[] ldy;
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess || e5 != hipSuccess) {
    if (h->pf_mem) (void)hipFree(h->pf_mem);
    (void)hipFree(h->mem);
    delete h;
    return fail(PE_ERR_DEVICE, "initial upload failed");
  }
  // every env starts reset (episode 0), like DummyVecEnv.reset() before the first step
  StepArgs a = base_args(h);
  rc = launch_reset(h, a, nullptr);
  if (rc == PE_OK && h->pf_every > 0) rc = launch_prefetch(h, nullptr, 1);
  if (rc == PE_OK) {
    hipError_t se = hipDeviceSynchronize();
    if (se != hipSuccess) rc = hip_fail(se, "initial reset");
  }
  if (rc != PE_OK) {
    if (h->pf_mem) (void)hipFree(h->pf_mem);
    (void)hipFree(h->mem);
    delete h;
    return rc;
  }
  *out = h;
  return PE_OK;
}

int pe_destroy(pe_handle* h) {
  if (!h) return PE_OK;
  DeviceGuard dg(h);
  int rc = dg.rc;
  if (rc == PE_OK && h->mem) {
    hipError_t e = hipFree(h->mem);
    if (e != hipSuccess) rc = hip_fail(e, "hipFree");
  }
  if (h->cur_mem) (void)hipFree(h->cur_mem);
  if (h->pf_mem) (void)hipFree(h->pf_mem);
  delete h;
  return rc;
}

int pe_curriculum_enable(pe_handle* h, double initial_threshold, double max_threshold, double threshold_increment,
                         int32_t max_episodes_per_maze, int32_t terminate_on_threshold, void* stream) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  if (max_episodes_per_maze < 1) return fail(PE_ERR_ARG, "max_episodes_per_maze must be >= 1");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  if (!h->cur_mem) {
    hipError_t me = hipMalloc(&h->cur_mem, sizeof(CurRec) * (size_t)h->n);
    if (me != hipSuccess) {
      h->cur_mem = nullptr;
      return fail(PE_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(me));
    }
  }
  // A2C_training.py:41-54 / trainingCode.py:29-42: counters 0, maze_completed False,
  // persistent None -- written on the caller's stream, after its queued steps
  hipLaunchKernelGGL(pe_cur_init_kernel, dim3((h->n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<CurRec*>(h->cur_mem), h->n, initial_threshold);
  PE_HIP(hipGetLastError());
  h->st.cur = static_cast<CurRec*>(h->cur_mem);
  h->rl.cur_max = max_threshold;
  h->rl.cur_inc = threshold_increment;
  h->rl.cur_max_eps = max_episodes_per_maze;
  h->rl.cur_term = terminate_on_threshold ? 1 : 0;
  return PE_OK;
}

int pe_curriculum_disable(pe_handle* h) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  h->st.cur = nullptr;
  return PE_OK;
}

int pe_curriculum_get(pe_handle* h, double* threshold, int32_t* counters, void* stream) {
  if (!h || !h->st.cur) return fail(PE_ERR_ARG, "curriculum not enabled");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t pitch = sizeof(CurRec);
  if (threshold)
    PE_HIP(hipMemcpy2DAsync(threshold, sizeof(double), h->st.cur, pitch, sizeof(double), (size_t)h->n,
                            hipMemcpyDeviceToDevice, s));
  if (counters)
    PE_HIP(hipMemcpy2DAsync(counters, 4 * sizeof(int32_t), reinterpret_cast<char*>(h->st.cur) + 8, pitch,
                            4 * sizeof(int32_t), (size_t)h->n, hipMemcpyDeviceToDevice, s));
  return PE_OK;
}

int pe_seed(pe_handle* h, uint64_t seed, int32_t reset_episode_counters, void* stream) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  // on the caller's stream: a step or prefetch kernel queued before this call must
  // finish before the records and counters are cleared (a prefetch still running
  // could otherwise publish an old-seed record after the clear)
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (h->pf.scal && seed != h->rl.seed)  // every prefetched map belongs to the old seed
    PE_HIP(hipMemsetAsync(h->pf.scal, 0, sizeof(uint4) * (size_t)h->n, s));
  h->rl.seed = seed;
  h->cfg.seed = seed;
  if (reset_episode_counters) {
    // the episode counters to 0, the visit rows of envs at an odd episode moved along
    // (they live in the counter's slot, pe_device.hpp vis_env)
    StepArgs a = base_args(h);
    hipLaunchKernelGGL(pe_zero_episodes_kernel, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, s, a);
    PE_HIP(hipGetLastError());
  }
  return PE_OK;
}

// The steps' deferred overflow writes applied (pe_vx_flush_kernel), before a call that
// reads the exact visit counts (state export, the MCTS clone) or replaces them (set
// state, resets: reset_env's map scratch is the overflow array).
int flush_vx(const pe_handle* h, hipStream_t s) {
  hipLaunchKernelGGL(pe_vx_flush_kernel, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, s, base_args(h));
  PE_HIP(hipGetLastError());
  return PE_OK;
}

extern "C" int pe_internal_flush_vx(const pe_handle* h, void* stream) {
  return flush_vx(h, static_cast<hipStream_t>(stream));
}

int pe_reset(pe_handle* h, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  a.mask = mask;
  a.obs = obs;
  if (const int fr = flush_vx(h, static_cast<hipStream_t>(stream))) return fr;
  const int rc = launch_reset(h, a, static_cast<hipStream_t>(stream));
  if (rc != PE_OK || h->pf_every <= 0) return rc;
  return launch_prefetch(h, static_cast<hipStream_t>(stream), 1);  // the new episodes' next maps
}

int pe_step(pe_handle* h, const void* actions, int32_t action_bytes, float* obs, float* reward, uint8_t* terminated,
            uint8_t* truncated, float* terminal_obs, double* ep_ret, int32_t* ep_len, int32_t* terminal_info,
            void* stream) {
  if (!h || !actions || !obs || !reward || !terminated || !truncated) return fail(PE_ERR_ARG, "null argument");
  if (action_bytes != 4 && action_bytes != 8) return fail(PE_ERR_ARG, "action_bytes must be 4 or 8");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  a.act_bytes = action_bytes;
  a.actions = actions;
  a.obs = obs;
  a.reward = reward;
  a.term = terminated;
  a.trunc = truncated;
  a.tobs = terminal_obs;
  a.ep_ret_out = ep_ret;
  a.ep_len_out = ep_len;
  a.tinfo = terminal_info;
  const int rc = launch_step(h, a, static_cast<hipStream_t>(stream));
  if (rc != PE_OK || h->pf_every <= 0 || ++h->pf_count < h->pf_every) return rc;
  h->pf_count = 0;
  return launch_prefetch(h, static_cast<hipStream_t>(stream), 0);  // maps for the envs reset since the last one
}

int pe_step_codes(pe_handle* h, const void* actions, int32_t action_bytes, uint8_t* obs_codes, float* reward,
                  uint8_t* terminated, uint8_t* truncated, float* terminal_obs, double* ep_ret, int32_t* ep_len,
                  int32_t* terminal_info, void* stream) {
  if (!h || !actions || !obs_codes || !reward || !terminated || !truncated) return fail(PE_ERR_ARG, "null argument");
  if (!h->obs_codes) return fail(PE_ERR_ARG, "pe_step_codes needs a handle created with obs_codes = 1");
  if (action_bytes != 4 && action_bytes != 8) return fail(PE_ERR_ARG, "action_bytes must be 4 or 8");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  a.act_bytes = action_bytes;
  a.actions = actions;
  a.obs_codes = obs_codes;
  a.reward = reward;
  a.term = terminated;
  a.trunc = truncated;
  a.tobs = terminal_obs;
  a.ep_ret_out = ep_ret;
  a.ep_len_out = ep_len;
  a.tinfo = terminal_info;
  const int rc = launch_step(h, a, static_cast<hipStream_t>(stream));
  if (rc != PE_OK || h->pf_every <= 0 || ++h->pf_count < h->pf_every) return rc;
  h->pf_count = 0;
  return launch_prefetch(h, static_cast<hipStream_t>(stream), 0);
}

int pe_obs_code_table(const pe_handle* h, float* table) {
  if (!h || !table) return fail(PE_ERR_ARG, "null argument");
  // obs_code_pick's table on the host tables: the same f32 quotients pe_create uploads
  const int R = h->g.R, G = h->g.G;
  for (int c = 0; c < 256; ++c) {
    float v = 0.0f;
    if (c <= R) v = (float)((double)c / (double)R);
    else if (c == R + 1) v = 1.0f;
    else if (c >= kCodeVis && c < kCodeVis + 16) v = (float)((double)(c - kCodeVis < 10 ? c - kCodeVis : 10) / 10.0);
    else if (c >= kCodePos && c < kCodePos + G) v = (float)((double)(c - kCodePos) / (double)G);
    table[c] = v;
  }
  return PE_OK;
}

int pe_expand_obs_codes(const pe_handle* h, int32_t blocks, int32_t rows, const uint8_t* src, int64_t src_stride,
                        float* obs, float* reward, uint8_t* terminated, uint8_t* truncated, void* stream) {
  if (!h || !src || !obs) return fail(PE_ERR_ARG, "null argument");
  if (blocks < 1 || blocks > 65535 || rows < 1) return fail(PE_ERR_ARG, "blocks must be 1..65535, rows >= 1");
  const int64_t need = (((int64_t)rows * h->g.D + 15) & ~(int64_t)15) + 6 * (int64_t)rows;
  if (blocks > 1 && (src_stride < need || (src_stride & 15))) return fail(PE_ERR_ARG, "src_stride too small or not a multiple of 16");
  if ((reinterpret_cast<uintptr_t>(src) & 15u) || (reinterpret_cast<uintptr_t>(obs) & 15u))
    return fail(PE_ERR_ARG, "src and obs must be 16-B aligned");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  const int64_t groups = ((int64_t)rows * h->g.D + 3) / 4;
  // kExpandPer groups per thread; the per-env outputs need a thread per env
  const int64_t gx = std::max((groups + 256 * kExpandPer - 1) / (256 * kExpandPer), ((int64_t)rows + 255) / 256);
  dim3 grid((unsigned)gx, (unsigned)blocks), block(256);
  hipLaunchKernelGGL(pe_expand_codes_kernel, grid, block, 0, static_cast<hipStream_t>(stream), h->st.tab, h->g.R,
                     h->g.G, h->g.D, rows, src, src_stride, obs, reward, terminated, truncated);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int pe_get_info(pe_handle* h, int32_t* info, void* stream) {
  if (!h || !info) return fail(PE_ERR_ARG, "null argument");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  hipLaunchKernelGGL(pe_info_kernel, dim3((h->n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), a, info);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int pe_get_state(pe_handle* h, uint8_t* cells, int32_t* visits, int8_t* explored, int32_t* scalars, void* stream) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (visits)
    if (const int fr = flush_vx(h, s)) return fr;
  if (cells || visits || explored) {
    int64_t total = (int64_t)h->n * h->g.GG;
    hipLaunchKernelGGL(pe_get_cells_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a, cells, visits,
                       explored);
    PE_HIP(hipGetLastError());
  }
  if (scalars) {
    hipLaunchKernelGGL(pe_get_scal_kernel, dim3((h->n + 255) / 256), dim3(256), 0, s, a, scalars);
    PE_HIP(hipGetLastError());
  }
  return PE_OK;
}

int pe_set_state(pe_handle* h, const uint8_t* cells, const int32_t* visits, const int8_t* explored,
                 const int32_t* scalars, void* stream) {
  if (!h) return fail(PE_ERR_ARG, "null handle");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (const int fr = flush_vx(h, s)) return fr;
  hipLaunchKernelGGL(pe_set_env_kernel, dim3((h->n + 127) / 128), dim3(128), 0, s, a, cells, visits, explored, scalars);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int pe_load_maps(pe_handle* h, int32_t k, const int32_t* env_index, const uint8_t* cells, const int32_t* rover,
                 float* obs_k, void* stream) {
  if (!h || (k > 0 && (!env_index || !cells || !rover))) return fail(PE_ERR_ARG, "null argument");
  if (k <= 0) return PE_OK;
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  StepArgs a = base_args(h);
  a.obs = obs_k;
  if (const int fr = flush_vx(h, static_cast<hipStream_t>(stream))) return fr;
  hipLaunchKernelGGL(pe_load_maps_kernel, dim3((k + kBlock - 1) / kBlock), dim3(kBlock), lds_bytes(h->g),
                     static_cast<hipStream_t>(stream), a, k, env_index, cells, rover);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int pe_synth_actions(pe_handle* h, uint64_t seed, uint32_t t, int32_t* actions, void* stream) {
  if (!h || !actions) return fail(PE_ERR_ARG, "null argument");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  hipLaunchKernelGGL(pe_synth_kernel, dim3((h->n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), h->n,
                     seed, h->rl.env_off, t, actions);
  PE_HIP(hipGetLastError());
  return PE_OK;
}

int pe_poll_errors(pe_handle* h, int32_t* bits, void* stream) {
  if (!h || !bits) return fail(PE_ERR_ARG, "null argument");
  DeviceGuard dg(h);
  if (dg.rc) return dg.rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t v = 0;
  PE_HIP(hipMemcpyAsync(&v, h->st.err_bits, sizeof(v), hipMemcpyDeviceToHost, s));
  PE_HIP(hipMemsetAsync(h->st.err_bits, 0, sizeof(uint32_t), s));
  PE_HIP(hipStreamSynchronize(s));
  *bits = (int32_t)((v >> 2) & 7u);
  return PE_OK;
}

#ifdef PE_STAMPS
int pe_debug_dstamps(uint64_t* host, int64_t count) {
  if (count > 16384 * 8) count = 16384 * 8;
  PE_HIP(hipDeviceSynchronize());
  PE_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dstamps), (size_t)count * 8, 0, hipMemcpyDeviceToHost));
  return PE_OK;
}
#endif
#if defined(PE_STAMPS) || defined(PE_STAMPS_RESET)
int pe_debug_stamps(uint64_t* host, int64_t count) {
  if (count > 16384 * 8) count = 16384 * 8;
  PE_HIP(hipDeviceSynchronize());
  PE_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)count * 8, 0, hipMemcpyDeviceToHost));
  return PE_OK;
}
#endif

int32_t pe_num_envs(const pe_handle* h) { return h ? h->n : 0; }
int32_t pe_kernel_variant(const pe_handle* h) { return h ? h->variant : -1; }
const char* pe_kernel_name(const pe_handle* h) { return h ? h->kname : ""; }
int32_t pe_prefetch_every(const pe_handle* h) { return h ? h->pf_every : 0; }
uint64_t pe_state_bytes(const pe_handle* h) { return h ? (uint64_t)h->bytes : 0; }

}  // extern "C"
