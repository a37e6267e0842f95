// pe_device.hpp -- device-side state layout and per-env primitives of the
// batched PlantOSEnv (MI355X / gfx950).
//
// HBM layout (struct-of-arrays, env-major records):
//   scal   uint4  [N]              packed scalars (below), one 16-B load per lane
//   ep_ret f64    [N]              running episode return (Monitor semantics)
//   grid   u64    [N][G][WPR]      2-bit cell codes, each row padded by R obstacle
//                                  cells on both sides: a LIDAR probe never needs a
//                                  column bounds test (off-map == obstacle,
//                                  plantos_env.py:271-274)
//   vis    u32    [N][2][G][NW]    4-bit saturating visit counts min(v,15), padded by
//                                  2 cells of value 10 on both sides (off-map reads
//                                  1.0 = min(10,10)/10, plantos_env.py:307-311).
//                                  The nibble IS the visit count while it is < 15.
//                                  Two slots per env: episode k's visits live in slot
//                                  k & 1 (vis_env), so the next episode's fresh rows
//                                  can be written ahead of time into the idle slot (the
//                                  prefetch kernel) and an auto-reset that takes a
//                                  prefetched record stores no visit row at all.
//   vx     u32    [N][G*G]         exact visit count, valid only where the nibble is 15
//                                  (plantos_env.py:203): written once at the 15th
//                                  visit, then bumped by no-return atomics (never read
//                                  by the step kernels); never cleared.  A step defers
//                                  its write (vpend): scattered writes to cold lines
//                                  issued at the commit held the end of the launch
//   vpend  u32    [N]              the overflow write of an env's last step (vx_pending:
//                                  cell | SET15 / INC, 0 = none; the headline kernel
//                                  only), applied by the commit lane of the next step at
//                                  the start of its compute phase, or by
//                                  pe_vx_flush_kernel before any API call that reads or
//                                  replaces the counts
//   expl   u32    [N][EW]          explored bitmap (explored_map > 0), authoritative
//                                  only in F_EXPL_BITMAP mode; otherwise explored is
//                                  derived: explored_map > 0  <=>  visit > 0 (true for
//                                  every state the reference dynamics reach)
//
// Packed scalars (scal):
//   w0 = x | y<<8 | step<<16        w1 = explored_count | total_cells<<16
//   w2 = collisions | flags<<16     w3 = episode (resets so far)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pe {

enum : int { EMPTY = 0, OBST = 1, HYD = 2, THIRSTY = 3 };

// flags (high half of w2)
enum : uint32_t {
  F_COLLIDED = 1u,      // collided_with_wall (sticky)
  F_BONUS = 2u,         // completion_bonus_given
  F_POISON_HYD = 4u,    // root env would raise TypeError (plantos_env.py:217-220)
  F_POISON_ACT = 8u,    // action < -4 (reference IndexError)
  F_NOROOM = 16u,       // last reset had no room (plantos_env.py:360-364)
  F_EXPL_BITMAP = 32u,  // explored map decoupled from visits (injected state, e.g.
                        // CurriculumWrapper visit_counts, A2C_training.py:88-93)
};

constexpr uint64_t kEven64 = 0x5555555555555555ull;  // low bit of every 2-bit code
constexpr uint32_t kDomainReset = 0x50455352u;        // Philox counter domain words
constexpr uint32_t kDomainAction = 0x4E544341u;       // (must match oracle/plantos_oracle.c)
constexpr int kMaxWPR = 8;                            // G + 2R <= 256
constexpr int kMaxNW = 20;                            // (G + 4) * 4 bits + 1 word

struct Geo {
  int G, C, R, D, DS;   // D = 5C+27 obs floats, DS = LDS row stride (odd)
  int WPR, NW, EW, GG;
  int64_t gstride, vstride, hstride, estride;  // per-env strides in elements
  int64_t vslot;                               // one visit slot (G * NW words); vstride = 2 vslot
};

// Host-built constant tables (one copy per handle, global memory, read-only).
struct Tables {
  float dist[72];              // dist[r] = float(r / R)             plantos_env.py:288
  float pos[256];              // pos[x]  = float(x / G)             plantos_env.py:295-296
  float vis[16];               // vis[n]  = float(min(n,10) / 10.0)  plantos_env.py:308
  uint64_t grid_pad[kMaxWPR];  // empty row: obstacle codes in the 2R pad columns
  uint64_t grid_real[kMaxWPR]; // low-bit mask of the G real columns
  uint32_t vis_pad[kMaxNW];    // empty visit row: nibble 10 in the 4 pad columns
};

// Batched CurriculumWrapper state per env (A2C_training.py:41-54), when enabled.
struct CurRec {
  double thr;          // exploration_threshold
  uint32_t episodes;   // episode_count
  uint32_t successes;  // successful_explorations
  uint32_t on_maze;    // episodes_on_current_maze
  uint32_t flags;      // CUR_* below
  uint32_t pad[2];
};
enum : uint32_t {
  CUR_COMPLETED = 1u,  // maze_completed
  CUR_CARRY = 2u,      // persistent_visit_counts is not None
};

struct State {
  uint4* scal;
  double* ep_ret;
  uint64_t* grid;
  uint32_t* vis;
  uint32_t* vx;    // visit-count overflow slots (see layout above)
  uint32_t* vpend; // each env's deferred overflow write (see layout above)
  uint32_t* expl;
  const Tables* tab;
  const signed char* ldx;  // [C][R] LIDAR offsets (generic kernel)
  const signed char* ldy;
  // [C][(R+7)&~7] (dx & 0xFF) | dy << 8, zero-padded (pe_step_wave's LDS header, the
  // runtime sector kernel's probes); for pe_step_wave<., true> the same probes as
  // [C][RP] u16 aligned-window byte offsets, then [C][RP] u8 bit shifts (pe_create)
  const int16_t* ldxy;
  uint32_t* err_bits;      // OR of error flags raised since the last poll
  CurRec* cur;             // batched CurriculumWrapper records, NULL when disabled
};

// Prefetched resets, see pe_coop.hpp coop_take_prefetched.
struct Prefetch {
  uint4* scal;      // [N] packed scalars the reset produces (before coop_apply_reset)
  uint64_t* grid;   // [N][gstride] grid rows of the new map
  float* obs;       // [N] rows of ostride bytes: the fresh observation of the new episode (D floats,
                    // or D byte codes for a byte-coded tile), rows 16-B aligned (LDS-DMA staging)
  uint8_t* flag;    // [N] 1: the env consumed its record (a plain byte store by the step
                    // kernel -- no returning atomic on its critical path)
  uint32_t* queue;  // [N] flagged envs, compacted by pe_pf_compact_kernel (the next batch to generate)
  uint32_t* qn;     // [0] queued count, [1] ticket of the generating launch
  uint32_t ostride; // bytes per obs row (multiple of 16)
};

// The record's obs row of env e (floats or codes).
__device__ __forceinline__ float* pf_obs_row(const Prefetch& pf, int64_t e) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(pf.obs) + e * (int64_t)pf.ostride);
}

struct Rules {
  double r_goal, r_mistake, r_invalid, r_water_empty, r_step, r_exploration, r_revisit, r_complete;
  double p_thirsty;
  uint64_t seed;
  uint32_t env_off;
  int P, O, max_steps;
  double cur_max, cur_inc;  // CurriculumWrapper max_threshold, threshold_increment
  int cur_max_eps;          // max_episodes_per_maze (A2C_training.py:54, trainingCode.py:42)
  int cur_term;             // 1: the threshold also terminates (A2C_training.py:101-103);
                            // 0: it only marks the maze completed (trainingCode.py:87-89)
  int map_algo;             // PE_MAP_ORIGINAL / PE_MAP_MAZE (the fork, plantos_env_new.py:355-358)
};

// CurriculumWrapper.step (A2C_training.py:97-109, trainingCode.py:84-96):
// exploration_percentage >= the env's threshold marks the maze completed and, in the
// A2C variant (term_on_hit), reports terminated; the env's own termination and
// completion bonus are untouched.  pct as the reference computes it.
__device__ __forceinline__ bool curriculum_hit(CurRec* cur, int64_t e, double thr, int expl, int total,
                                               int term_on_hit) {
  const double pct = ((double)expl / (double)total) * 100.0;  // plantos_env.py:331
  if (pct >= thr) {
    cur[e].flags |= CUR_COMPLETED;
    return term_on_hit != 0;
  }
  return false;
}

// CurriculumWrapper.reset (A2C_training.py:56-95) of env e, run before its
// env.reset(); returns true when the new episode keeps the previous episode's
// visit counts (self.env.visit_counts = persistent_visit_counts).
__device__ inline bool curriculum_on_reset(CurRec* cur, int64_t e, const Rules& rl) {
  CurRec c = cur[e];
  c.episodes += 1;
  c.on_maze += 1;
  const bool timeout = (int)c.on_maze >= rl.cur_max_eps;
  bool keep = false;
  if ((c.flags & CUR_COMPLETED) || timeout) {
    if (c.flags & CUR_COMPLETED) {
      c.thr = fmin(c.thr + rl.cur_inc, rl.cur_max);
      c.successes += 1;
    }
    c.flags = 0;  // maze_completed = False, persistent_visit_counts = None
    c.on_maze = 0;
  } else {
    keep = (c.flags & CUR_CARRY) != 0;
    c.flags |= CUR_CARRY;  // persistent = visit_counts.copy() (tracks the live counts)
  }
  cur[e] = c;
  return keep;
}

// ------------------------------------------------------------------ scalars
struct Scal {
  int x, y, step, expl, total, coll;
  uint32_t flags, episode;
};

// Write-through (sc1) stores for the per-step state commit: a relaxed agent-scope
// atomic store is a plain store with sc1 (MI355X: the line goes on to the
// Infinity Cache / HBM at once instead of staying dirty in the XCD's L2), so the
// kernel-end L2 writeback has nothing of it left to flush at the launch boundary.
#ifndef PE_SCAL_STORE16
#define PE_SCAL_STORE16 1  // 16-B packed-scalar stores (headline 9.54 -> 9.28 us, desync 10.57 -> 10.40; A/B: 0)
#endif
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(uint4* p, uint4 v) {
#if PE_SCAL_STORE16
  // one 16-B write-through store (the packed scalars of consecutive lanes are contiguous:
  // whole lines per wave-instruction) -- two 8-B atomic stores left every line half
  // written per instruction
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
#else
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
  st_wt(q, (uint64_t)v.x | ((uint64_t)v.y << 32));
  st_wt(q + 1, (uint64_t)v.z | ((uint64_t)v.w << 32));
#endif
}

__device__ __forceinline__ Scal unpack(uint4 w) {
  Scal s;
  s.x = w.x & 0xFF;
  s.y = (w.x >> 8) & 0xFF;
  s.step = w.x >> 16;
  s.expl = w.y & 0xFFFF;
  s.total = w.y >> 16;
  s.coll = w.z & 0xFFFF;
  s.flags = w.z >> 16;
  s.episode = w.w;
  return s;
}

__device__ __forceinline__ uint4 pack(const Scal& s) {
  uint4 w;
  w.x = (uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.step << 16);
  w.y = (uint32_t)s.expl | ((uint32_t)s.total << 16);
  w.z = (uint32_t)s.coll | (s.flags << 16);
  w.w = s.episode;
  return w;
}

// ------------------------------------------------------------------ Philox4x32-10
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Sequential u32 stream over Philox blocks: identical draw order to the oracle's
// u32src (oracle/plantos_oracle.c) for (seed, env_id, episode).
struct Stream {
  uint32_t k0, k1, env, episode, blk;
  uint32_t buf[4];
  int pos;
  __device__ void init(uint64_t seed, uint32_t env_id, uint32_t ep) {
    k0 = (uint32_t)seed;
    k1 = (uint32_t)(seed >> 32);
    env = env_id;
    episode = ep;
    blk = 0;
    pos = 4;
  }
  __device__ uint32_t next() {
    if (pos == 4) {
      uint4 o = philox(make_uint4(blk, env, episode, kDomainReset), k0, k1);
      buf[0] = o.x; buf[1] = o.y; buf[2] = o.z; buf[3] = o.w;
      ++blk;
      pos = 0;
    }
    // mask select: a ternary chain over buf[] is folded into a dynamically
    // indexed load, which would put the stream state in scratch memory
    const uint32_t m0 = 0u - (uint32_t)(pos == 0), m1 = 0u - (uint32_t)(pos == 1);
    const uint32_t m2 = 0u - (uint32_t)(pos == 2), m3 = 0u - (uint32_t)(pos == 3);
    const uint32_t v = (buf[0] & m0) | (buf[1] & m1) | (buf[2] & m2) | (buf[3] & m3);
    ++pos;
    return v;
  }
  // random.py:239-248 _randbelow_with_getrandbits (getrandbits(k) = u32 >> (32-k))
  __device__ uint32_t below(uint32_t n) {
    if (!n) return 0;
    int k = 32 - __clz(n);
    uint32_t r = next() >> (32 - k);
    while (r >= n) r = next() >> (32 - k);
    return r;
  }
  // random.random()
  __device__ double random53() {
    uint32_t a = next() >> 5, b = next() >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }
};

// ------------------------------------------------------------------ cell access
__device__ __forceinline__ int grid_code(const State& st, const Geo& g, int64_t e, int row, int pcol) {
  int bit = 2 * pcol;
  uint64_t w = st.grid[e * g.gstride + (int64_t)row * g.WPR + (bit >> 6)];
  return (int)((w >> (bit & 63)) & 3u);
}

__device__ __forceinline__ void grid_set(const State& st, const Geo& g, int64_t e, int row, int pcol, int code) {
  int bit = 2 * pcol;
  uint64_t* p = st.grid + e * g.gstride + (int64_t)row * g.WPR + (bit >> 6);
  uint64_t w = *p;
  w &= ~(3ull << (bit & 63));
  w |= (uint64_t)code << (bit & 63);
  *p = w;
}

// The visit rows of env e in episode `ep` (its packed scalars' episode counter): slot ep & 1.
__device__ __forceinline__ uint32_t* vis_env(const State& st, const Geo& g, int64_t e, uint32_t ep) {
  return st.vis + e * g.vstride + (int64_t)(ep & 1u) * g.vslot;
}

// 5 nibbles (padded columns y..y+4 == real columns y-2..y+2) of one visit row.
__device__ __forceinline__ uint32_t vis_window(const State& st, const Geo& g, int64_t e, uint32_t ep, int row, int y) {
  int bit = 4 * y;
  const uint32_t* p = vis_env(st, g, e, ep) + (int64_t)row * g.NW + (bit >> 5);
  uint64_t two = (uint64_t)p[0] | ((uint64_t)p[1] << 32);
  return (uint32_t)(two >> (bit & 31)) & 0xFFFFFu;
}

__device__ __forceinline__ void vis_set(const State& st, const Geo& g, int64_t e, uint32_t ep, int row, int col,
                                        uint32_t v) {
  int bit = 4 * (col + 2);
  uint32_t* p = vis_env(st, g, e, ep) + (int64_t)row * g.NW + (bit >> 5);
  uint32_t w = *p;
  w &= ~(0xFu << (bit & 31));
  w |= v << (bit & 31);
  *p = w;
}

__device__ __forceinline__ uint32_t nibble_get(const State& st, const Geo& g, int64_t e, uint32_t ep, int row,
                                               int col) {
  int bit = 4 * (col + 2);
  return (vis_env(st, g, e, ep)[(int64_t)row * g.NW + (bit >> 5)] >> (bit & 31)) & 15u;
}

// exact visit count of a real cell (nibble below 15, else the u16 overflow slot)
__device__ __forceinline__ int visit_exact(const State& st, const Geo& g, int64_t e, uint32_t ep, int row, int col) {
  const uint32_t n = nibble_get(st, g, e, ep, row, col);
  return n < 15u ? (int)n : (int)st.vx[e * g.hstride + row * g.G + col];
}

// visit_counts[cell] += 1 (plantos_env.py:203) given the cell's current nibble n: the
// overflow slot is set at the 15th visit and bumped in memory after that.  The
// headline sector kernel (pe_step_quad<C16,R6,1word>, 64 envs) defers that write as a
// vpend entry (vx_pending), stores it, and applies the previous step's early in the next
// launch (vx_apply; the same lane, program order): a write to vx issued at the commit --
// one per ~100 env-steps, each to a cold line of a 105 MB array at 65536 envs -- held
// the launch's end (profiles/r4p/, r4q/).  Every other step kernel writes at once
// (visit_bump_exact): their handles never hold a pending word.
enum : uint32_t { VP_SET15 = 1u << 31, VP_INC = 1u << 30, VP_CELL = VP_INC - 1u };
__device__ __forceinline__ uint32_t vx_pending(int cell, uint32_t n) {
  return n == 14u ? (VP_SET15 | (uint32_t)cell) : (n == 15u ? (VP_INC | (uint32_t)cell) : 0u);
}
__device__ __forceinline__ void visit_bump_exact(const State& st, const Geo& g, int64_t e, int cell, uint32_t n) {
  uint32_t* vp = st.vx + e * g.hstride + cell;
  if (n == 14u)
    *vp = 15u;
  else if (n == 15u)
    atomicAdd(vp, 1u);  // no-return atomic: the count is never read by a step
}
__device__ __forceinline__ void vx_apply(const State& st, const Geo& g, int64_t e, uint32_t p) {
  uint32_t* vp = st.vx + e * g.hstride + (p & VP_CELL);
  if (p & VP_SET15)
    *vp = 15u;
  else
    atomicAdd(vp, 1u);  // no-return atomic: the count is never read by a step
}

__device__ __forceinline__ bool expl_test_set(const State& st, const Geo& g, int64_t e, int cell) {
  uint32_t* p = st.expl + e * g.estride + (cell >> 5);
  uint32_t m = 1u << (cell & 31);
  uint32_t w = *p;
  if (w & m) return false;
  *p = w | m;
  return true;
}

// _get_info (plantos_env.py:317-336), integer columns (pe_info layout of
// include/plantos_batch.h) for env e with scalars s.
// wfix: the env's last watering (THIRSTY -> HYD) was not stored (an auto-reset
// overwrites the grid rows, quad kernel commit).
__device__ inline void write_info(const State& st, const Geo& g, const Tables* tab, int64_t e, const Scal& s,
                                  int32_t* o, int wfix = 0) {
  int th = 0, hy = 0;
  for (int row = 0; row < g.G; ++row)
    for (int w = 0; w < g.WPR; ++w) {
      const uint64_t v = st.grid[e * g.gstride + (int64_t)row * g.WPR + w];
      const uint64_t lo = v & kEven64, hi = (v >> 1) & kEven64, real = tab->grid_real[w];
      th += __popcll(lo & hi & real);   // sum(plants.values())           :318
      hy += __popcll(~lo & hi & real);  // len(plants) - thirsty          :319
    }
  th -= wfix;
  hy += wfix;
  o[0] = s.x;                                 // rover_position           :324
  o[1] = s.y;
  o[2] = th;
  o[3] = hy;
  o[4] = th + hy;                             // total_plants             :327
  o[5] = s.step;                              // step_count               :328
  o[6] = s.expl;                              // explored_cells           :320
  o[7] = s.total;                             // total_cells              :321
  o[8] = (s.flags & F_COLLIDED) ? 1 : 0;      // collided_with_wall       :333
  o[9] = s.coll;                              // total_collisions         :334
  o[10] = (int)((s.flags >> 2) & 7u);         // error flags (PE_S_POISONED layout)
}

// ------------------------------------------------------------------ map generation
// A "grid image" is one env's grid rows [G][WPR] (padded 2-bit codes) anywhere:
// the env's block in HBM, or a scratch copy in LDS during an in-kernel reset.
__device__ __forceinline__ int img_code(const uint64_t* sg, const Geo& g, int row, int pcol) {
  const int bit = 2 * pcol;
  return (int)((sg[row * g.WPR + (bit >> 6)] >> (bit & 63)) & 3u);
}

__device__ __forceinline__ void img_set(uint64_t* sg, const Geo& g, int row, int pcol, int code) {
  const int bit = 2 * pcol;
  uint64_t& w = sg[row * g.WPR + (bit >> 6)];
  w = (w & ~(3ull << (bit & 63))) | ((uint64_t)code << (bit & 63));
}

// Index of the j-th real cell (row-major) whose code matches `kind`
// (kind 0: not an obstacle, kind 1: empty).  Returns the cell id x*G+y.
__device__ inline int img_nth_cell(const uint64_t* sg, const Geo& g, const Tables* tab, int j, int kind) {
  for (int row = 0; row < g.G; ++row) {
    for (int w = 0; w < g.WPR; ++w) {
      const uint64_t v = sg[row * g.WPR + w];
      const uint64_t lo = v & kEven64, hi = (v >> 1) & kEven64;
      const uint64_t real = tab->grid_real[w];
      uint64_t m = kind == 0 ? (real & ~(lo & ~hi)) : (real & ~(lo | hi));
      const int c = __popcll(m);
      if (j < c) {
        for (int k = 0; k < j; ++k) m &= m - 1;
        const int pcol = w * 32 + (__ffsll((unsigned long long)m) - 1) / 2;
        return row * g.G + (pcol - g.R);
      }
      j -= c;
    }
  }
  return 0;  // unreachable when j < count
}

// Obstacle clusters of _generate_map (plantos_env.py:341-354) on an empty image.
__device__ inline void clusters_original(const Geo& g, const Rules& rl, const Tables* tab, uint64_t* sg, Stream& rng) {
  const int G = g.G;
  for (int row = 0; row < G; ++row)
    for (int w = 0; w < g.WPR; ++w) sg[row * g.WPR + w] = tab->grid_pad[w];
  const int clusters = rl.O / 3;
  for (int q = 0; q < clusters; ++q) {
    const int cx = 2 + (int)rng.below((uint32_t)(G - 4));
    const int cy = 2 + (int)rng.below((uint32_t)(G - 4));
    const int size = 2 + (int)rng.below(2u);
    for (int dx = 0; dx < size; ++dx)
      for (int dy = 0; dy < size; ++dy) {
        const int ox = cx + dx - size / 2, oy = cy + dy - size / 2;
        if (0 <= ox && ox < G && 0 <= oy && oy < G) img_set(sg, g, ox, oy + g.R, OBST);
      }
  }
}

// ---- the fork's maze (gradio-app/plantos_env_new.py:408-604) on a grid image.
__device__ __forceinline__ void img_carve(uint64_t* sg, const Geo& g, int x, int y) {
  if (0 <= x && x < g.G && 0 <= y && y < g.G) img_set(sg, g, x, y + g.R, EMPTY);  // obstacles.discard
}

// _carve_irregular_room (:479-516)
__device__ inline void maze_room(const Geo& g, uint64_t* sg, Stream& rng, int mx, int my) {
  const int bx = mx * 6 + 1, by = my * 6 + 1;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) img_carve(sg, g, bx + i, by + j);
  if (rng.random53() < 0.3)  // extend right
    for (int i = 0; i < 2; ++i)
      for (int j = 2; j < 4; ++j) img_carve(sg, g, bx + 5 + i, by + j);
  if (rng.random53() < 0.3)  // extend down
    for (int i = 2; i < 4; ++i)
      for (int j = 0; j < 2; ++j) img_carve(sg, g, bx + i, by + 5 + j);
  if (rng.random53() < 0.4) {  // corner cut: random.choice([(0,0), (4,0), (0,4), (4,4)])
    const int k = (int)rng.below(4u);
    const int x = bx + ((k & 1) ? 4 : 0), y = by + ((k & 2) ? 4 : 0);
    if (x < g.G && y < g.G) img_set(sg, g, x, y + g.R, OBST);  // obstacles.add
  }
}

// _carve_irregular_path (:518-536, cardinal moves) = _carve_straight_path (:538-557,
// width 5) + a 20 % path bulge (_add_path_bulge :559-582)
__device__ inline void maze_path(const Geo& g, uint64_t* sg, Stream& rng, int cx, int cy, int nx, int ny) {
  if (cx == nx) {
    const int lo = cy < ny ? cy : ny, hi = cy < ny ? ny : cy;
    for (int m = lo; m <= hi; ++m)
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 6; ++j) img_carve(sg, g, cx * 6 + 1 + i, m * 6 + 1 + j);
  } else {
    const int lo = cx < nx ? cx : nx, hi = cx < nx ? nx : cx;
    for (int m = lo; m <= hi; ++m)
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 5; ++j) img_carve(sg, g, m * 6 + 1 + i, cy * 6 + 1 + j);
  }
  if (rng.random53() < 0.2) {
    const int mx = (cx + nx) / 2, my = (cy + ny) / 2;
    const int dir = rng.below(2u) ? 1 : -1;  // random.choice([-1, 1])
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) {
        if (cx == nx)  // dx == 0: vertical path, horizontal bulge
          img_carve(sg, g, mx * 6 + 2 + dir * 2 + i, my * 6 + 2 + j);
        else
          img_carve(sg, g, mx * 6 + 2 + i, my * 6 + 2 + dir * 2 + j);
      }
  }
}

// Maze obstacles (:408-456): all cells obstacles, randomized DFS over the
// (G-1)/6 meta grid carving rooms and paths.  G >= 7 (pe_create checks).  A meta
// cell is visited iff its centre (6a+3, 6b+3) is carved: rooms always carve it and
// nothing else ever touches a centre (paths carve only between visited cells,
// bulges/extensions/corners sit at other residues mod 6), so no visited map is
// kept; the DFS stack is the chain of parent directions (2 bits per meta cell in
// `par`, maze_scratch_bytes).
__device__ inline void maze_obstacles(const Geo& g, const Tables* tab, uint64_t* sg, uint8_t* par, Stream& rng) {
  const int G = g.G, mw = (G - 1) / 6;
  for (int row = 0; row < G; ++row)
    for (int w = 0; w < g.WPR; ++w) sg[row * g.WPR + w] = tab->grid_pad[w] | tab->grid_real[w];
  const int sx = (int)rng.below((uint32_t)mw), sy = (int)rng.below((uint32_t)mw);  // randint(0, meta_w-1)
  maze_room(g, sg, rng, sx, sy);
  int cx = sx, cy = sy;
  for (;;) {
    int cand[4], nc = 0;
    // (0,1), (0,-1), (1,0), (-1,0) (:440)
    if (cy + 1 < mw && img_code(sg, g, cx * 6 + 3, (cy + 1) * 6 + 3 + g.R) == OBST) cand[nc++] = 0;
    if (cy > 0 && img_code(sg, g, cx * 6 + 3, (cy - 1) * 6 + 3 + g.R) == OBST) cand[nc++] = 1;
    if (cx + 1 < mw && img_code(sg, g, (cx + 1) * 6 + 3, cy * 6 + 3 + g.R) == OBST) cand[nc++] = 2;
    if (cx > 0 && img_code(sg, g, (cx - 1) * 6 + 3, cy * 6 + 3 + g.R) == OBST) cand[nc++] = 3;
    if (nc) {
      const uint32_t r = rng.below((uint32_t)nc);
      const int d = r == 0 ? cand[0] : (r == 1 ? cand[1] : (r == 2 ? cand[2] : cand[3]));
      const int nx = cx + (d == 2 ? 1 : (d == 3 ? -1 : 0)), ny = cy + (d == 0 ? 1 : (d == 1 ? -1 : 0));
      maze_path(g, sg, rng, cx, cy, nx, ny);
      maze_room(g, sg, rng, nx, ny);
      const int m = nx * mw + ny;
      par[m >> 2] = (uint8_t)((par[m >> 2] & ~(3u << (2 * (m & 3)))) | ((uint32_t)d << (2 * (m & 3))));
      cx = nx;
      cy = ny;
    } else {
      if (cx == sx && cy == sy) break;  // stack empty
      const int m = cx * mw + cy;
      const int d = (par[m >> 2] >> (2 * (m & 3))) & 3;  // pop: back to the parent
      cx -= d == 2 ? 1 : (d == 3 ? -1 : 0);
      cy -= d == 0 ? 1 : (d == 1 ? -1 : 0);
    }
  }
}

// _generate_map (plantos_env.py:338-372; the fork's 'maze' :355-358, 408-477) in the
// device-rng mode defined by oracle po_reset_philox: Philox stream keyed by (seed,
// global env id, episode), candidate lists in row-major order.  Writes the grid
// image sg (all rows) and returns the new scalars of the episode (flags F_NOROOM
// if there is no room, plantos_env.py:360-364).  picks: max(2P,
// maze_scratch_bytes(G)) bytes of scratch.
__device__ __forceinline__ Scal gen_map(const Geo& g, const Rules& rl, const Tables* tab, uint64_t* sg, uint16_t* picks,
                               uint32_t env_id, uint32_t episode) {
  const int G = g.G;
  Stream rng;
  rng.init(rl.seed, env_id, episode);
  if (rl.map_algo == 1) {
    maze_obstacles(g, tab, sg, reinterpret_cast<uint8_t*>(picks), rng);
    int nfree = 0;
    for (int row = 0; row < G; ++row)
      for (int w = 0; w < g.WPR; ++w) {
        const uint64_t v = sg[row * g.WPR + w];
        nfree += __popcll(~v & tab->grid_real[w]);  // real cells whose code has the low bit clear
      }
    if (nfree < rl.P + 1) clusters_original(g, rl, tab, sg, rng);  // fallback, same stream (:461-466)
  } else {
    clusters_original(g, rl, tab, sg, rng);
  }
  int n_obst = 0;
  for (int row = 0; row < G; ++row)
    for (int w = 0; w < g.WPR; ++w) {
      const uint64_t v = sg[row * g.WPR + w];
      n_obst += __popcll(v & ~(v >> 1) & tab->grid_real[w] & kEven64);
    }
  const int nfree = g.GG - n_obst;
  Scal s;
  s.step = 0;
  s.coll = 0;
  s.flags = 0;
  s.episode = episode + 1u;
  s.total = nfree;
  s.expl = 1;
  if (nfree < rl.P + 1) {  // ValueError, plantos_env.py:360-364
    s.flags = F_NOROOM;
    s.x = 0;
    s.y = 0;
    s.expl = 0;
    return s;
  }
  // random.sample(list(available), P): set-based selection, row-major list
  for (int i = 0; i < rl.P; ++i) {
    int c;
    for (;;) {
      c = img_nth_cell(sg, g, tab, (int)rng.below((uint32_t)nfree), 0);
      if (img_code(sg, g, c / G, c % G + g.R) == EMPTY) break;  // else already selected
    }
    img_set(sg, g, c / G, c % G + g.R, HYD);
    picks[i] = (uint16_t)c;
  }
  // thirsty draws in sample order, plantos_env.py:367-369
  for (int i = 0; i < rl.P; ++i) {
    const int c = picks[i];
    if (rng.random53() < rl.p_thirsty) img_set(sg, g, c / G, c % G + g.R, THIRSTY);
  }
  // rover: choice(list(available - plants)), plantos_env.py:370-372
  const int rc = img_nth_cell(sg, g, tab, (int)rng.below((uint32_t)(nfree - rl.P)), 1);
  s.x = rc / G;
  s.y = rc % G;
  return s;
}

// Fresh visit rows of env e (all zero, pads 10) with visit[rover] = 1
// (plantos_env.py:146-147; explored[rover] = 2 follows from it, :236).  The
// overflow slots and the explored bitmap are not cleared: every nibble is now 0
// (vx is read only behind a nibble of 15) and a fresh episode is in derived mode.
// (s: the NEW episode's scalars: the rows go to its slot)
__device__ inline void reset_visits(const State& st, const Geo& g, const Tables* tab, int64_t e, const Scal& s) {
  uint32_t* vb = vis_env(st, g, e, s.episode);
  for (int row = 0; row < g.G; ++row)
    for (int w = 0; w < g.NW; ++w) vb[(int64_t)row * g.NW + w] = tab->vis_pad[w];
  if (!(s.flags & F_NOROOM)) vis_set(st, g, e, s.episode, s.x, s.y, 1u);
}

// The previous episode's visit rows (slot of episode - 1) into the new episode's slot.
__device__ inline void carry_visits(const State& st, const Geo& g, int64_t e, uint32_t new_ep) {
  const uint32_t* src = vis_env(st, g, e, new_ep - 1u);
  uint32_t* dst = vis_env(st, g, e, new_ep);
  for (int64_t k = 0; k < g.vslot; ++k) dst[k] = src[k];
}

// Visits of a new episode: fresh (reset_visits), or -- CurriculumWrapper carrying
// the previous episode's counts -- carried into the new slot with only the explored
// map restarted at the rover ({rover}, bitmap mode: explored no longer follows visits).
__device__ inline void new_episode_visits(const State& st, const Geo& g, const Tables* tab, int64_t e, Scal& s,
                                          bool keep) {
  if (!keep) {
    reset_visits(st, g, tab, e, s);
    return;
  }
  carry_visits(st, g, e, s.episode);
  uint32_t* eb = st.expl + e * g.estride;
  for (int w = 0; w < g.estride; ++w) eb[w] = 0u;
  if (!(s.flags & F_NOROOM)) {
    const int rc = s.x * g.G + s.y;
    eb[rc >> 5] = 1u << (rc & 31);  // explored_map[rover] = 2 (plantos_env.py:236)
  }
  s.flags |= F_EXPL_BITMAP;
}

// reset() for one env (plantos_env.py:125-158), generated in place in HBM.
// tab: the handle's tables, ideally a copy in LDS (read in every scan step).
__device__ __forceinline__ Scal reset_env(const State& st, const Geo& g, const Rules& rl, const Tables* tab, int64_t e,
                                 uint32_t episode) {
  const bool keep = st.cur ? curriculum_on_reset(st.cur, e, rl) : false;
  uint16_t* picks = reinterpret_cast<uint16_t*>(st.vx + e * g.hstride);  // scratch (all nibbles 0 after)
  if (keep) picks = reinterpret_cast<uint16_t*>(st.expl + e * g.estride);  // vx holds carried counts
  Scal s = gen_map(g, rl, tab, st.grid + e * g.gstride, picks, rl.env_off + (uint32_t)e, episode);
  if (s.flags & F_NOROOM) atomicOr(st.err_bits, F_NOROOM);
  new_episode_visits(st, g, tab, e, s, keep);
  return s;
}

// Scratch of the maze DFS: 2 bits per meta cell.
__host__ __device__ constexpr int maze_scratch_bytes(int G) { return (((G - 1) / 6) * ((G - 1) / 6) + 3) / 4; }

// Bytes of LDS scratch reset_env_scratch needs (grid image + picks/maze DFS, 8-B aligned).
__host__ __device__ constexpr int reset_scratch_bytes(int G, int WPR, int P) {
  return 8 + G * WPR * 8 + (2 * P > maze_scratch_bytes(G) ? 2 * P : maze_scratch_bytes(G));
}

// reset() generated in a scratch image (LDS) and written to HBM row by row:
// the rejection-sampling scans run at LDS latency instead of HBM latency.
__device__ __forceinline__ Scal reset_env_scratch(const State& st, const Geo& g, const Rules& rl, const Tables* tab, int64_t e,
                                         uint32_t episode, uint64_t* sg) {
  const bool keep = st.cur ? curriculum_on_reset(st.cur, e, rl) : false;
  uint16_t* picks = reinterpret_cast<uint16_t*>(sg + g.G * g.WPR);
  Scal s = gen_map(g, rl, tab, sg, picks, rl.env_off + (uint32_t)e, episode);
  if (s.flags & F_NOROOM) atomicOr(st.err_bits, F_NOROOM);
  uint64_t* gb = st.grid + e * g.gstride;
  for (int k = 0; k < g.G * g.WPR; ++k) gb[k] = sg[k];
  new_episode_visits(st, g, tab, e, s, keep);
  return s;
}

}  // namespace pe
