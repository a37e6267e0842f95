// pe_mcts.hip -- batched MCTS search on MI355X (gfx950): one MCTS.search of the
// reference (mcts_custom_trainer.py:72-243) per env, all envs at once.
//
// One lane owns one env's search.  The search is sequential inside an env (every
// simulation reads the statistics the previous ones wrote), so the parallelism is
// across envs; everything a lane touches is its own:
//   cellw  u32 [N][G*G]        the sim env (_copy_env_state, :221-243): exact visit
//                              count (bits 0-28) | cell code << 29 | explored << 31
//   ulog   uint2 [N][D+4]      undo log of the current simulation: (cell, old word);
//                              replayed backwards instead of re-copying the state
//                              per simulation (a simulation touches <= D+2 cells)
//   nodes  MNode [N][S+1]      the tree: MCTSNode (:20-33) records, 32 B
//   rng    u32 [N][628]        the env's np.random stream (persistent across searches)
// The clone kernel rebuilds cellw from the live batch state (one thread per cell,
// coalesced) before every search; the search kernel reads nothing else of it.
//
// np.random stream (numpy legacy RandomState = MT19937).  Device form of a stream at
// position p: words [0,p) already hold the NEXT round's words, [p,624) this round's;
// the next output is temper(mt[p]).  A draw regenerates its own word (the twist done
// one word at a time, which is order-equivalent to numpy's block twist), so no lane
// ever stops for a 624-word twist.  Draws are generated ahead into a per-lane LDS ring
// (wave-uniform top-ups, all loads of a top-up in flight together); the unconsumed
// tail is rewound at the end, so the stream stops exactly at its first unconsumed draw.
// mt[625] keeps this round's mt[0] (overwritten at position 0) so the host can give
// the state back in numpy's own terms (pe_mcts_get_rng).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/plantos_batch.h"
#include "pe_device.hpp"
#include "pe_handle.hpp"

using namespace pe;

namespace {

constexpr int kMtN = 624, kMtM = 397;
constexpr int kRngStride = 628;  // mt[624], pos, saved mt[0], 2 pad (16-B rows)
constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMag = 0x9908b0dfu;

constexpr uint32_t kVisMask = 0x1FFFFFFFu;
constexpr int kCodeShift = 29;
constexpr uint32_t kCodeMask = 3u << kCodeShift;
constexpr uint32_t kExpl = 1u << 31;
constexpr uint32_t kOffMap = (uint32_t)OBST << kCodeShift;  // off-map neighbour == obstacle (:193-195)

struct MNode {          // MCTSNode, mcts_custom_trainer.py:20-33
  double value;         // sum of rollout rewards (:133)
  int32_t visits;
  uint32_t untried;     // bits 0-2: len(untried_actions); action j at bits 3+3j (list order, :32)
  uint16_t kid[5];      // children in dict insertion order (:31, :124)
  uint16_t parent;      // 0xFFFF at the root
  uint8_t nkid, action, pad[2];
};
static_assert(sizeof(MNode) == 32, "32-B tree records");

constexpr uint32_t kAllUntried = 5u | (0u << 3) | (1u << 6) | (2u << 9) | (3u << 12) | (4u << 15);

struct MctsArgs {
  State st;
  Geo g;
  Rules rl;
  int n;
  uint32_t* cellw;
  uint8_t* cellb;   // [N][ggp] clone bytes (LDS path)
  uint32_t* csim;   // [N][G*G] (LDS path)
  uint32_t* csg;    // [N][G*G] (LDS path)
  int ggp, ldsp;    // global / LDS per-env byte strides of the clone bytes
  uint2* ulog;
  MNode* nodes;
  uint32_t* rng;
  int n_sims, max_depth;
  double c;
  const double* logt;  // logt[k] = log(k) from the host's libm (CPython's math.log)
  const uint8_t* mask;
  int32_t* actions;
  int32_t* rorder;
  int32_t* rvisits;
  double* rvalue;
};

__device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t twist(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & kUpper) | (nxt & kLower);
  return far ^ (y >> 1) ^ ((y & 1u) ? kMag : 0u);
}

// One env's np.random stream, device form (see the file comment).
__device__ __forceinline__ uint32_t untemper(uint32_t y) {
  y ^= y >> 18;
  y ^= (y << 15) & 0xefc60000u;
  uint32_t t = y;
#pragma unroll
  for (int i = 0; i < 4; ++i) t = y ^ ((t << 7) & 0x9d2c5680u);
  y = t;
  return y ^ (y >> 11) ^ (y >> 22);
}

constexpr int kRing = 32;  // buffered draws per lane (LDS ring)
constexpr int kTop = 16;   // draws per top-up: one 16-aligned block of stream positions
constexpr int kLow = 8;    // the wave tops up when any lane has fewer left (> draws of one step, typically)
static_assert(kMtN % kTop == 0 && kRngStride % 4 == 0, "16-aligned blocks never straddle the wrap");

// One env's np.random stream, device form (see the file comment).  Draws are
// generated ahead into an LDS ring, one 16-aligned block of stream positions per
// top-up: the block's words, its successors and its "far" words (+397) come in as
// 16-B loads and the next-round words go out as 16-B stores.  Top-ups are
// wave-uniform (top_up_if_low), so a wave pays one memory round trip for all its
// lanes.  Until the position is 16-aligned (a stream left mid-block by a previous
// search) draws come one at a time (gen_direct).  close() rewinds the
// generated-but-unconsumed tail (raw word = untemper(output)), so the stored stream
// stops exactly at the first unconsumed draw.  The ring is [slot][lane] interleaved
// (a top-up's 64 lanes write one slot row: no bank conflicts).
struct NpStream {
  uint32_t* mt;
  uint32_t* ring;      // &ring_base[lane]; slot k at ring[k * 64]
  int p;               // position of the next draw to generate
  uint32_t cur;        // mt[p] (the current-round word at p)
  int head, cnt;       // ring read slot, draws buffered
  uint32_t saved_prev; // mt[625] before the last generation of position 0
#ifdef PE_MCTS_PROF
  uint64_t topups = 0;
#endif

  __device__ void open(uint32_t* m, uint32_t* r) {
    mt = m;
    ring = r;
    p = (int)m[kMtN];
    cur = m[p];
    head = 0;
    cnt = 0;
    saved_prev = m[kMtN + 1];
  }
  __device__ void top_up() {  // positions p .. p+15 (p % 16 == 0, cnt <= kRing - kTop)
    const uint4* m4 = reinterpret_cast<const uint4*>(mt);
    uint32_t nx[kTop], far[kTop];
    // successors p+1 .. p+16: the block itself shifted by one, plus the next block's first word
    const uint4 b0 = m4[p / 4], b1 = m4[p / 4 + 1], b2 = m4[p / 4 + 2], b3 = m4[p / 4 + 3];
    int pn = p + kTop;
    pn -= pn >= kMtN ? kMtN : 0;
    const uint32_t w16 = mt[pn];
    // far words p+397 .. p+412 lie in the 4-word chunks starting at p+396, +400, ..., +412
    uint4 f[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      int q = p + 396 + 4 * k;
      q -= q >= kMtN ? kMtN : 0;
      q -= q >= kMtN ? kMtN : 0;
      f[k] = m4[q / 4];
    }
    const uint32_t blk[16] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w,
                              b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w};
    const uint32_t fw[20] = {f[0].x, f[0].y, f[0].z, f[0].w, f[1].x, f[1].y, f[1].z, f[1].w,
                             f[2].x, f[2].y, f[2].z, f[2].w, f[3].x, f[3].y, f[3].z, f[3].w,
                             f[4].x, f[4].y, f[4].z, f[4].w};
#pragma unroll
    for (int k = 0; k < kTop; ++k) {
      nx[k] = k + 1 < kTop ? blk[k + 1] : w16;
      far[k] = fw[k + 1];
    }
    if (p == 0) {  // this round's mt[0], kept for pe_mcts_get_rng
      saved_prev = mt[kMtN + 1];
      mt[kMtN + 1] = cur;
    }
    uint32_t nw[kTop];
    const int slot0 = (head + cnt) & (kRing - 1);
#pragma unroll
    for (int k = 0; k < kTop; ++k) {
      nw[k] = twist(cur, nx[k], far[k]);
      ring[((slot0 + k) & (kRing - 1)) * 64] = temper(cur);
      cur = nx[k];
    }
    uint4* o4 = reinterpret_cast<uint4*>(mt) + p / 4;
    o4[0] = make_uint4(nw[0], nw[1], nw[2], nw[3]);
    o4[1] = make_uint4(nw[4], nw[5], nw[6], nw[7]);
    o4[2] = make_uint4(nw[8], nw[9], nw[10], nw[11]);
    o4[3] = make_uint4(nw[12], nw[13], nw[14], nw[15]);
    p = pn;
    cnt += kTop;
  }
  __device__ void top_up_if_low() {
    if (__any(cnt < kLow) && cnt <= kRing - kTop && (p & (kTop - 1)) == 0) {
#ifdef PE_MCTS_PROF
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      top_up();
      topups += __builtin_amdgcn_s_memtime() - t0;
#else
      top_up();
#endif
    }
  }
  // one draw straight from the stream (ring empty: before the first aligned block,
  // or a long rejection streak)
  __device__ uint32_t gen_direct() {
    int i1 = p + 1, i2 = p + kMtM;
    i1 -= i1 >= kMtN ? kMtN : 0;
    i2 -= i2 >= kMtN ? kMtN : 0;
    const uint32_t nxt = mt[i1], far = mt[i2];
    if (p == 0) {
      saved_prev = mt[kMtN + 1];
      mt[kMtN + 1] = cur;
    }
    mt[p] = twist(cur, nxt, far);
    const uint32_t v = temper(cur);
    cur = nxt;
    p = i1;
    return v;
  }
  __device__ uint32_t next() {
    if (cnt == 0) return gen_direct();
    const uint32_t v = ring[head * 64];
    head = (head + 1) & (kRing - 1);
    --cnt;
    return v;
  }
  __device__ void close() {
    int q = p - cnt;
    q += q < 0 ? kMtN : 0;
    for (int j = 0; j < cnt; ++j) {  // rewind the unconsumed tail
      int pos = q + j;
      pos -= pos >= kMtN ? kMtN : 0;
      mt[pos] = untemper(ring[((head + j) & (kRing - 1)) * 64]);
      if (pos == 0) mt[kMtN + 1] = saved_prev;
    }
    mt[kMtN] = (uint32_t)q;
  }
  // np.random.random(): 53 bits from two draws
  __device__ double random() {
    // both ring reads issued before any branch (the ring is rarely short)
    const uint32_t r0 = ring[head * 64], r1 = ring[((head + 1) & (kRing - 1)) * 64];
    uint32_t a, b;
    if (cnt >= 2) {
      a = r0;
      b = r1;
      head = (head + 2) & (kRing - 1);
      cnt -= 2;
    } else {
      a = next();
      b = next();
    }
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
  }
  // np.random.random() < 0.7, decided on the 53-bit integer: random() = N / 2^53 exactly
  // and the double 0.7 is 6305039478318694 / 2^53, so the comparison is N < that.
  __device__ bool random_lt_07() {
    const uint32_t r0 = ring[head * 64], r1 = ring[((head + 1) & (kRing - 1)) * 64];
    uint32_t a, b;
    if (cnt >= 2) {
      a = r0;
      b = r1;
      head = (head + 2) & (kRing - 1);
      cnt -= 2;
    } else {
      a = next();
      b = next();
    }
    const uint64_t nbits = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
    return nbits < 6305039478318694ull;
  }
  // np.random.randint(n): masked rejection on 32-bit draws, no draw for n == 1
  __device__ int randint(int n) {
    const uint32_t rng = (uint32_t)(n - 1);
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next() & mask)) > rng) {
    }
    return (int)v;
  }
};

struct Sim {
  int x, y, step, expl;
  bool cur_expl, bonus;
};

// What one sim step reads: the rover's N, E, S, W neighbours (plantos_env.py:186)
// and its own cell (index 4).  Off-map neighbours read as obstacles (:193-195).
struct Nbr {
  uint32_t code[5], vis[5];  // cell code, exact visit count
  uint32_t expl;             // bit q: explored_map > 0
};

__device__ __forceinline__ uint32_t sel5(const uint32_t w[5], int k) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) v |= w[j] & (0u - (uint32_t)(j == k));
  return v;
}

__device__ __forceinline__ int nbr_cell(int c, int G, int q) {
  return q == 0 ? c - G : (q == 1 ? c + 1 : (q == 2 ? c + G : (q == 3 ? c - 1 : c)));
}

__device__ __forceinline__ bool nbr_on_map(const Sim& s, int G, int q) {
  return q == 0 ? s.x > 0 : (q == 1 ? s.y + 1 < G : (q == 2 ? s.x + 1 < G : (q == 3 ? s.y > 0 : true)));
}

// Sim cells in global memory (any G): u32 words, exact visits; undo log of
// (cell, old word).
struct GCells {
  uint32_t* cw;
  uint2* lg;
  int nlog, G, c;
  uint32_t w[5];
  __device__ void load(const Sim& s, Nbr& nb) {
    c = s.x * G + s.y;
    nb.expl = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {  // all five loads issued together (off-map: read own cell, replace)
      const bool on = nbr_on_map(s, G, q);
      const uint32_t r = cw[on ? nbr_cell(c, G, q) : c];
      w[q] = on ? r : kOffMap;
      nb.code[q] = (w[q] & kCodeMask) >> kCodeShift;
      nb.vis[q] = w[q] & kVisMask;
      nb.expl |= (w[q] & kExpl) ? 1u << q : 0u;
    }
  }
  // visit_counts[new] += 1, explored_map[new] = 2, explored_map[old] = 1 (:198-203)
  __device__ void move(int q, bool set_old) {
    if (set_old) {
      lg[nlog++] = make_uint2((uint32_t)c, w[4]);
      cw[c] = w[4] | kExpl;
    }
    const int nc = nbr_cell(c, G, q);
    const uint32_t nw = sel5(w, q);
    lg[nlog++] = make_uint2((uint32_t)nc, nw);
    cw[nc] = (nw | kExpl) + 1u;
  }
  __device__ void water() {  // thirsty -> hydrated (fork :237-240)
    lg[nlog++] = make_uint2((uint32_t)c, w[4]);
    cw[c] = (w[4] & ~kCodeMask) | ((uint32_t)HYD << kCodeShift);
  }
  __device__ void undo() {
    for (int k = nlog - 1; k >= 0; --k) {
      const uint2 u = lg[k];
      cw[u.x] = u.y;
    }
    nlog = 0;
  }
};

// Sim cells in LDS (G <= 64): one byte per cell = visits min(v,31) (bits 0-4) |
// explored << 5 | code << 6.  A field of 31 means "31 or more": the exact count is
// the clone's word (cellw) or, once this simulation has bumped the cell, csim
// (valid where csg holds the simulation's stamp).  Undo = copy the clone's pristine
// bytes (cellb, global, 16-B loads) back over the lane's LDS cells.  cb is 4-B aligned.
constexpr uint32_t kLSat = 31u, kLExpl = 32u;
constexpr int kLCodeShift = 6;

__device__ __forceinline__ uint32_t sat_byte(uint32_t w) {
  const uint32_t v = w & kVisMask;
  return (v < kLSat ? v : kLSat) | ((w & kExpl) ? kLExpl : 0u) | (((w & kCodeMask) >> kCodeShift) << kLCodeShift);
}

struct LCells {
  uint8_t* cb;            // this lane's cells (LDS)
  const uint4* pristine;  // this lane's clone bytes (global)
  const uint32_t* cw;     // exact clone words (global)
  uint32_t* csim;         // exact sim counts of bumped saturated cells (global)
  uint32_t* csg;          // their stamps
  int G, c, nchunk, ldsw; // nchunk = pristine 16-B chunks, ldsw = LDS dwords per lane
  uint32_t stamp;
  uint32_t b[5];
  __device__ uint32_t exact(int i) const { return csg[i] == stamp ? csim[i] : (cw[i] & kVisMask); }
  __device__ void load(const Sim& s, Nbr& nb) {
    c = s.x * G + s.y;
    nb.expl = 0;
    uint32_t sat = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {  // all five LDS reads issued together (off-map: read own cell, replace)
      const bool on = nbr_on_map(s, G, q);
      const uint32_t r = cb[on ? nbr_cell(c, G, q) : c];
      b[q] = on ? r : ((uint32_t)OBST << kLCodeShift);
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      nb.code[q] = b[q] >> kLCodeShift;
      nb.vis[q] = b[q] & kLSat;
      sat |= nb.vis[q] == kLSat ? 1u << q : 0u;
      nb.expl |= (b[q] & kLExpl) ? 1u << q : 0u;
    }
    if (sat) {  // rare: counts of 31 or more come from global memory
#pragma unroll
      for (int q = 0; q < 5; ++q)
        if (sat & (1u << q)) nb.vis[q] = exact(nbr_cell(c, G, q));
    }
  }
  __device__ void move(int q, bool set_old) {
    if (set_old) cb[c] = (uint8_t)(b[4] | kLExpl);
    const int nc = nbr_cell(c, G, q);
    const uint32_t nb_ = sel5(b, q);
    const uint32_t f = nb_ & kLSat;
    uint32_t nv = nb_ | kLExpl;
    if (f + 1u < kLSat) {
      nv += 1u;
    } else {
      const uint32_t x = f < kLSat ? kLSat : exact(nc) + 1u;
      nv |= kLSat;
      csim[nc] = x;
      csg[nc] = stamp;
    }
    cb[nc] = (uint8_t)nv;
  }
  __device__ void water() {
    cb[c] = (uint8_t)((b[4] & ~(3u << kLCodeShift)) | ((uint32_t)HYD << kLCodeShift));
  }
  __device__ void undo() {
    uint32_t* d = reinterpret_cast<uint32_t*>(cb);
#pragma unroll 8
    for (int k = 0; k < nchunk; ++k) {  // LDS stores never alias the loads
      const uint4 v = pristine[k];
      if (4 * k + 0 < ldsw) d[4 * k + 0] = v.x;
      if (4 * k + 1 < ldsw) d[4 * k + 1] = v.y;
      if (4 * k + 2 < ldsw) d[4 * k + 2] = v.z;
      if (4 * k + 3 < ldsw) d[4 * k + 3] = v.w;
    }
    ++stamp;
  }
};

// PlantOSEnv.step on the sim env (plantos_env.py:160-183; watering of the fork,
// plantos_env_new.py:236-245).  Only what MCTS reads is produced: reward,
// terminated, truncated (the observation and info dict are never used by the search).
template <class CS>
__device__ double sim_step(const Rules& rl, CS& cs, Sim& s, int total, int act, const Nbr& nb, bool& te, bool& tr) {
  s.step += 1;                                                   // :162
  double r = rl.r_step;                                          // :164
  if (act < 4) {
    if (sel5(nb.code, act) != (uint32_t)OBST) {                 // in bounds, not an obstacle (:193-195)
      const bool never = sel5(nb.vis, act) == 0u;                // :197
      const bool new_unexpl = ((nb.expl >> act) & 1u) == 0u;
      cs.move(act, !s.cur_expl);                                 // :198-203
      s.expl += (s.cur_expl ? 0 : 1) + (new_unexpl ? 1 : 0);
      s.x += act == 0 ? -1 : (act == 2 ? 1 : 0);
      s.y += act == 1 ? 1 : (act == 3 ? -1 : 0);
      s.cur_expl = true;
      r += never ? rl.r_exploration : rl.r_revisit;              // :204-207
    } else {
      r += rl.r_invalid;                                         // :208-211
    }
  } else {
    const uint32_t code = nb.code[4];
    if (code == (uint32_t)THIRSTY) {                             // fork :237-240
      cs.water();
      r += rl.r_goal;
    } else if (code == (uint32_t)HYD) {
      r += rl.r_mistake;                                         // fork :241-242
    } else {
      r += rl.r_water_empty;                                     // :221-222
    }
  }
  // exploration_percentage = explored / total * 100 >= 100 (:320-331, 176, 244-246)
  // holds exactly when explored >= total: for e < t the f64 quotient is at most
  // 1 - 2^-53 and its product with 100 rounds below 100
  const bool full = s.expl >= total;
  te = full;
  tr = s.step >= rl.max_steps;                                   // :177
  if (full && !s.bonus) {                                        // :179-181
    r += rl.r_complete;
    s.bonus = true;
  }
  return r;
}

// _copy_env_state (:221-243): the live env -> the lane's sim cells, one thread per cell.
__global__ void pe_mcts_clone_kernel(MctsArgs a) {
  const Geo& g = a.g;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.n * g.GG) return;
  const int64_t e = t / g.GG;
  if (a.mask && !a.mask[e]) return;
  const int c = (int)(t - e * g.GG);
  const int row = c / g.G, col = c - row * g.G;
  const Scal s = unpack(a.st.scal[e]);
  const uint32_t code = (uint32_t)grid_code(a.st, g, e, row, col + g.R);
  const uint32_t v = (uint32_t)visit_exact(a.st, g, e, s.episode, row, col);
  bool ex;
  if (s.flags & F_EXPL_BITMAP)
    ex = (a.st.expl[e * g.estride + (c >> 5)] >> (c & 31)) & 1u;
  else
    ex = v > 0u;  // explored_map > 0 <=> visit > 0 (derived mode)
  const uint32_t w = (v & kVisMask) | (code << kCodeShift) | (ex ? kExpl : 0u);
  a.cellw[e * (int64_t)g.GG + c] = w;
  if (a.cellb) {
    a.cellb[e * (int64_t)a.ggp + c] = (uint8_t)sat_byte(w);
    a.csg[e * (int64_t)g.GG + c] = 0u;
  }
}

__device__ __forceinline__ MNode load_node(const MNode* T, int i) {
  MNode nd;
  const uint4* src = reinterpret_cast<const uint4*>(T + i);
  uint4* dst = reinterpret_cast<uint4*>(&nd);
  dst[0] = src[0];
  dst[1] = src[1];
  return nd;
}

__device__ __forceinline__ void store_node(MNode* T, int i, const MNode& nd) {
  const uint4* src = reinterpret_cast<const uint4*>(&nd);
  uint4* dst = reinterpret_cast<uint4*>(T + i);
  dst[0] = src[0];
  dst[1] = src[1];
}

__device__ __forceinline__ MNode fresh_node(int parent, int action) {
  MNode nd;
  nd.value = 0.0;
  nd.visits = 0;
  nd.untried = kAllUntried;  // list(range(5)) (:32)
#pragma unroll
  for (int j = 0; j < 5; ++j) nd.kid[j] = 0;
  nd.parent = (uint16_t)parent;
  nd.nkid = 0;
  nd.action = (uint8_t)action;
  nd.pad[0] = nd.pad[1] = 0;
  return nd;
}

__device__ __forceinline__ int kid_at(const MNode& nd, int j) {
  int v = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) v |= k == j ? nd.kid[k] : 0;
  return v;
}

// MCTS.search (:91-139) for env e with its sim cells in `cs`.  The four phases of a
// simulation are one loop of sim steps: each iteration picks the step's action by
// the lane's current phase (tree descent, expansion, rollout) and all lanes then
// run the same sim step together, whatever phase each is in.
enum : int { PH_SELECT = 0, PH_EXPAND = 1, PH_ROLLOUT = 2, PH_DONE = 3 };

#ifdef PE_MCTS_PROF  // diagnostics build: shader-clock cycles per phase, summed per lane
__device__ unsigned long long g_mcts_prof[1 << 20][4];
#define PE_MP_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PE_MP_ACC(a_, b_, c_, d_) \
  do {                            \
    pa += b_ - a_;                \
    pb += c_ - b_;                \
    pc += d_ - c_;                \
  } while (0)
#define PE_MP_STORE(e_)                                                     \
  do {                                                                      \
    if ((e_) < (1 << 20)) {                                                 \
      g_mcts_prof[e_][0] = pa;                                              \
      g_mcts_prof[e_][1] = pb;                                              \
      g_mcts_prof[e_][2] = pc;                                              \
      g_mcts_prof[e_][3] = rng.topups;                                      \
    }                                                                       \
  } while (0)
#else
#define PE_MP_T(v)
#define PE_MP_ACC(a_, b_, c_, d_)
#define PE_MP_STORE(e_)
#endif

template <class CS>
__device__ void search_env(const MctsArgs& a, int64_t e, CS& cs, uint32_t* ring) {
#pragma clang fp contract(off)
  const Scal s0 = unpack(a.st.scal[e]);
  const int total = s0.total;
  MNode* T = a.nodes + e * (int64_t)(a.n_sims + 1);
  NpStream rng;
  rng.open(a.rng + e * (int64_t)kRngStride, ring);
  Nbr nb;
  Sim s;
  s.x = s0.x;
  s.y = s0.y;
  cs.load(s, nb);
  const bool root_expl = (nb.expl >> 4) & 1u;

  store_node(T, 0, fresh_node(0xFFFF, 0xFF));
  int nn = 1;
#ifdef PE_MCTS_PROF
  uint64_t pa = 0, pb = 0, pc = 0;
#endif
  for (int sim = 0; sim < a.n_sims; ++sim) {
    s.x = s0.x;
    s.y = s0.y;
    s.step = s0.step;
    s.expl = s0.expl;
    s.cur_expl = root_expl;
    s.bonus = false;  // a fresh PlantOSEnv: completion_bonus_given False (:221-243)
    int node = 0, depth = 0, phase = PH_SELECT;
    uint64_t pth0 = 0, pth1 = 0;  // node indices on the path (16 bits each), root first
    int plen = 1;
#define PUSH_PATH(idx)                                                 \
  do {                                                                 \
    if (plen < 4) pth0 |= (uint64_t)(idx) << (16 * plen);              \
    else if (plen < 8) pth1 |= (uint64_t)(idx) << (16 * (plen - 4));   \
    ++plen;                                                            \
  } while (0)
    double tot = 0.0;
    MNode nd = load_node(T, 0);
    PE_MP_T(t0);
    // 1.-2. tree descent and expansion: a few steps, one shared sim step
    while (phase != PH_ROLLOUT) {
      rng.top_up_if_low();
      int act = -1;
      if (phase == PH_SELECT) {
        // 1. selection (:106-114): descend while fully expanded
        if ((nd.untried & 7u) == 0u && nd.nkid > 0 && depth < a.max_depth) {
          // a fully expanded node has all 5 children: their records load together
          const double lv = a.logt[nd.visits];
          MNode ch[5];
#pragma unroll
          for (int j = 0; j < 5; ++j) ch[j] = load_node(T, nd.kid[j]);
          int bj = 0;
          double bw = 0.0;
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            double wgt;
            if (ch[j].visits == 0) {
              wgt = INFINITY;
            } else {
              const double exploitation = ch[j].value / (double)ch[j].visits;       // :55
              const double exploration = a.c * sqrt(lv / (double)ch[j].visits);    // :56
              wgt = exploitation + exploration;                                     // :57
            }
            if (j == 0 || wgt > bw) {  // max(): the first maximal child (:60)
              bj = j;
              bw = wgt;
            }
          }
          int bidx = nd.kid[0];
          MNode bn = ch[0];
#pragma unroll
          for (int j = 1; j < 5; ++j)
            if (bj == j) {
              bidx = nd.kid[j];
              bn = ch[j];
            }
          node = bidx;
          nd = bn;
          PUSH_PATH(node);
          act = nd.action;
        } else {
          phase = PH_EXPAND;
        }
      }
      if (phase == PH_EXPAND) {
        // 2. expansion (:117-125); depth is not advanced
        if ((nd.untried & 7u) > 0u && depth < a.max_depth) {
          const int cnt = (int)(nd.untried & 7u);
          const int k = rng.randint(cnt);
          act = (int)((nd.untried >> (3 + 3 * k)) & 7u);
          const uint32_t below = nd.untried & ((1u << (3 + 3 * k)) - 1u) & ~7u;
          const uint32_t above = (nd.untried >> (3 + 3 * (k + 1))) << (3 + 3 * k);
          nd.untried = below | above | (uint32_t)(cnt - 1);
          const int ci = nn++;
#pragma unroll
          for (int j = 0; j < 5; ++j)
            if (j == nd.nkid) nd.kid[j] = (uint16_t)ci;
          nd.nkid += 1;
          store_node(T, node, nd);
          store_node(T, ci, fresh_node(node, act));
          node = ci;
          PUSH_PATH(node);
        } else {
          phase = PH_ROLLOUT;
        }
      }
      if (phase == PH_ROLLOUT) break;
      bool te, tr;
      cs.load(s, nb);
      sim_step(a.rl, cs, s, total, act, nb, te, tr);
      if (phase == PH_SELECT) {
        depth += 1;
        if (te || tr) phase = PH_EXPAND;
      } else {
        phase = PH_ROLLOUT;
      }
    }
    PE_MP_T(t1);
    // 3. rollout (:141-168), depth counts on from the descent
    for (int d = depth; d < a.max_depth; ++d) {
      rng.top_up_if_low();
      cs.load(s, nb);
      int act;
      if (rng.random_lt_07()) {                                   // np.random.random() < 0.7 (:180)
        // _exploration_heuristic (:187-219): first strictly least-visited valid move
        int best = -1;
        uint32_t minv = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (nb.code[q] != (uint32_t)OBST && (best < 0 || nb.vis[q] < minv)) {
            best = q;
            minv = nb.vis[q];
          }
        }
        act = best >= 0 ? best : rng.randint(5);
      } else {
        act = rng.randint(5);                                     // :183
      }
      bool te, tr;
      const double r = sim_step(a.rl, cs, s, total, act, nb, te, tr);
      tot += r;
      if (te || tr) {
        if (s.expl >= total) tot += 500.0;  // exploration_percentage >= 100 (:160-163)
        break;
      }
    }
    PE_MP_T(t2);
    // 4. backpropagation (:130-134): the path's records load together when it is
    // short (the usual case), else walk the parent links
    if (plen <= 8) {
      MNode pb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < plen) pb[k] = load_node(T, (int)(((k < 4 ? pth0 : pth1) >> (16 * (k & 3))) & 0xFFFFu));
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < plen) {
          pb[k].visits += 1;
          pb[k].value += tot;
          store_node(T, (int)(((k < 4 ? pth0 : pth1) >> (16 * (k & 3))) & 0xFFFFu), pb[k]);
        }
    } else {
      for (int i = node; i != 0xFFFF;) {
        MNode b = load_node(T, i);
        b.visits += 1;
        b.value += tot;
        store_node(T, i, b);
        i = b.parent;
      }
    }
    cs.undo();  // the next simulation starts from a fresh copy (:104)
    PE_MP_T(t3);
    PE_MP_ACC(t0, t1, t2, t3);
  }
  PE_MP_STORE(e);
  // best_action (:62-69)
  const MNode root = load_node(T, 0);
  int act;
  if (root.nkid == 0) {
    act = rng.randint(5);
  } else {
    int best = -1;
    double bq = 0.0;
    for (int j = 0; j < root.nkid; ++j) {
      const MNode ch = load_node(T, kid_at(root, j));
      const double q = ch.value / (double)(ch.visits > 1 ? ch.visits : 1);
      if (best < 0 || q > bq) {
        best = ch.action;
        bq = q;
      }
    }
    act = best;
  }
  rng.close();
  a.actions[e] = act;
  if (a.rorder || a.rvisits || a.rvalue) {
    for (int j = 0; j < 5; ++j) {
      const bool has = j < root.nkid;
      MNode ch;
      if (has) ch = load_node(T, kid_at(root, j));
      if (a.rorder) a.rorder[e * 5 + j] = has ? ch.action : -1;
      if (a.rvisits) a.rvisits[e * 5 + j] = has ? ch.visits : 0;
      if (a.rvalue) a.rvalue[e * 5 + j] = has ? ch.value : 0.0;
    }
  }
}

// Any G: sim cells in global memory.
__global__ __launch_bounds__(64) void pe_mcts_search_kernel(MctsArgs a) {
  __shared__ uint32_t ring[64 * kRing];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  if (a.mask && !a.mask[e]) return;
  GCells cs;
  cs.cw = a.cellw + e * (int64_t)a.g.GG;
  cs.lg = a.ulog + e * (int64_t)(a.max_depth + 4);
  cs.nlog = 0;
  cs.G = a.g.G;
  search_env(a, e, cs, ring + threadIdx.x);
}

// G <= 64: the workgroup's 64 sim envs live in LDS (lane-private regions with an
// odd dword stride, so lanes at the same cell hit different banks): the rollout's
// neighbour reads and updates never leave the CU.
__global__ __launch_bounds__(64) void pe_mcts_search_lds_kernel(MctsArgs a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int lane = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * 64;
  const int ggp = a.ggp, ldsw = a.ldsp / 4, nchunk = ggp / 16;
  // cooperative copy of the 64 clones (coalesced 16-B reads)
  const int64_t nenv = (int64_t)a.n - e0 < 64 ? (int64_t)a.n - e0 : 64;
  const uint4* src = reinterpret_cast<const uint4*>(a.cellb + e0 * ggp);
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lds);
  for (int64_t i = lane; i < nenv * nchunk; i += 64) {
    const int el = (int)(i / nchunk), k = (int)(i - (int64_t)el * nchunk);
    const uint4 v = src[i];
    uint32_t* d = l32 + el * ldsw + 4 * k;
    if (4 * k + 0 < ldsw) d[0] = v.x;
    if (4 * k + 1 < ldsw) d[1] = v.y;
    if (4 * k + 2 < ldsw) d[2] = v.z;
    if (4 * k + 3 < ldsw) d[3] = v.w;
  }
  __syncthreads();
  const int64_t e = e0 + lane;
  if (e >= a.n) return;
  if (a.mask && !a.mask[e]) return;
  LCells cs;
  cs.cb = lds + lane * a.ldsp;
  cs.pristine = reinterpret_cast<const uint4*>(a.cellb + e * ggp);
  cs.cw = a.cellw + e * (int64_t)a.g.GG;
  cs.csim = a.csim + e * (int64_t)a.g.GG;
  cs.csg = a.csg + e * (int64_t)a.g.GG;
  cs.G = a.g.G;
  cs.nchunk = nchunk;
  cs.ldsw = ldsw;
  cs.stamp = 1;
  search_env(a, e, cs, reinterpret_cast<uint32_t*>(lds + 64 * a.ldsp) + lane);
}

// np.random.seed(seed) (init_genrand, pos 624) then the pending block twist, giving
// the device form at position 0.  One thread per env.
__global__ void pe_mcts_seed_kernel(uint32_t* rng, int n, const uint32_t* seeds, uint32_t base) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint32_t* mt = rng + e * (int64_t)kRngStride;
  uint32_t v = seeds ? seeds[e] : base + (uint32_t)e;
  mt[0] = v;
  for (int i = 1; i < kMtN; ++i) {
    v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
    mt[i] = v;
  }
  uint32_t first = mt[0];
  uint32_t cur = first;
  for (int i = 0; i < kMtN; ++i) {
    const uint32_t nxt = i + 1 < kMtN ? mt[i + 1] : mt[0];
    const uint32_t far = mt[i + kMtM < kMtN ? i + kMtM : i + kMtM - kMtN];
    mt[i] = twist(cur, nxt, far);
    cur = nxt;
  }
  mt[kMtN] = 0;
  mt[kMtN + 1] = first;
  mt[kMtN + 2] = 0;
  mt[kMtN + 3] = 0;
}

// ---------------------------------------------------------------- host side
int fail(int code, const std::string& msg) { return pe_internal_set_error(code, msg.c_str()); }

int hip_fail(hipError_t e, const char* what) {
  return fail(PE_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define MC_HIP(call)                                   \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return hip_fail(_e, #call);  \
  } while (0)

struct DevBind {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DevBind(int dev) {
    (void)hipGetLastError();  // drop a stale error of an earlier call (launch checks below)
    int cur = -1;
    err = hipGetDevice(&cur);
    if (err == hipSuccess && cur != dev) {
      err = hipSetDevice(dev);
      if (err == hipSuccess) prev = cur;
    }
  }
  ~DevBind() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// numpy (key, pos) -> device form (host; see the file comment)
void np_to_device(const uint32_t* key, int pos, uint32_t* out) {
  std::memcpy(out, key, kMtN * sizeof(uint32_t));
  out[kMtN + 1] = key[0];
  out[kMtN + 2] = out[kMtN + 3] = 0;
  const int upto = pos >= kMtN ? kMtN : pos;
  for (int i = 0; i < upto; ++i) {
    const uint32_t nxt = i + 1 < kMtN ? out[i + 1] : out[0];
    const uint32_t far = out[i + kMtM < kMtN ? i + kMtM : i + kMtM - kMtN];
    const uint32_t y = (out[i] & kUpper) | (nxt & kLower);
    out[i] = far ^ (y >> 1) ^ ((y & 1u) ? kMag : 0u);
  }
  out[kMtN] = (uint32_t)(pos >= kMtN ? 0 : pos);
}

// device form -> numpy (key, pos): undo the twist of the words below pos.
void device_to_np(const uint32_t* dev, uint32_t* key, int32_t* pos) {
  const int p = (int)dev[kMtN];
  std::memcpy(key, dev, kMtN * sizeof(uint32_t));
  *pos = p;
  if (p == 0) return;  // a fresh round: (twisted words, pos 0) is numpy's own form too
  // y_i from new[i] = far_i ^ (y_i >> 1) ^ (y_i & 1 ? MAG : 0)
  auto far_of = [&](int i) -> uint32_t { return i + kMtM < kMtN ? key[i + kMtM] : dev[i + kMtM - kMtN]; };
  auto y_of = [&](int i) -> uint32_t {
    uint32_t t = dev[i] ^ far_of(i);
    const uint32_t b = t >> 31;
    if (b) t ^= kMag;
    return (t << 1) | b;
  };
  for (int j = p - 1; j >= 1; --j) key[j] = (y_of(j) & kUpper) | (y_of(j - 1) & kLower);
  key[0] = dev[kMtN + 1];
}

}  // namespace

constexpr size_t kMctsLdsMax = 64 * 1024;  // >= 2 workgroups per CU

struct pe_mcts {
  pe_handle* h;
  int force_global;  // PE_MCTS_GLOBAL=1 (PE_DEBUG_KNOBS builds): the global-memory sim cells even when LDS fits
  int n_sims, max_depth;
  double c;
  void* mem;
  uint32_t* cellw;
  uint8_t* cellb;   // [N][ggp] clone bytes (LDS path)
  uint32_t* csim;   // [N][G*G] (LDS path)
  uint32_t* csg;    // [N][G*G] (LDS path)
  int ggp;
  uint2* ulog;
  MNode* nodes;
  uint32_t* rng;
  double* logt;
};

extern "C" {

int pe_mcts_create(pe_handle* h, int32_t n_simulations, double c_param, int32_t max_depth, pe_mcts** out) {
  if (!h || !out) return fail(PE_ERR_ARG, "null argument");
  *out = nullptr;
  if (n_simulations < 0 || n_simulations > 65534) return fail(PE_ERR_ARG, "n_simulations must be in [0, 65534]");
  if (max_depth < 0 || max_depth > (1 << 20)) return fail(PE_ERR_ARG, "max_depth must be in [0, 2^20]");
  DevBind db(h->device);
  if (db.err != hipSuccess) return hip_fail(db.err, "hipSetDevice");
  const size_t n = (size_t)h->n, GG = (size_t)h->g.GG;
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  const size_t ggp = (GG + 15) / 16 * 16;
  const size_t b_cell = al(n * GG * 4), b_log = al(n * (size_t)(max_depth + 4) * 8),
               b_lds = al(n * ggp) + 2 * al(n * GG * 4),
               b_node = al(n * (size_t)(n_simulations + 1) * sizeof(MNode)), b_rng = al(n * kRngStride * 4),
               b_log_t = al((size_t)(n_simulations + 1) * 8);
  pe_mcts* m = new (std::nothrow) pe_mcts();
  if (!m) return fail(PE_ERR_NOMEM, "host allocation failed");
  hipError_t e = hipMalloc(&m->mem, b_cell + b_log + b_node + b_rng + b_log_t + b_lds);
  if (e != hipSuccess) {
    delete m;
    return fail(PE_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  char* p = static_cast<char*>(m->mem);
  m->cellw = reinterpret_cast<uint32_t*>(p);
  m->ulog = reinterpret_cast<uint2*>(p + b_cell);
  m->nodes = reinterpret_cast<MNode*>(p + b_cell + b_log);
  m->rng = reinterpret_cast<uint32_t*>(p + b_cell + b_log + b_node);
  m->logt = reinterpret_cast<double*>(p + b_cell + b_log + b_node + b_rng);
  char* q = p + b_cell + b_log + b_node + b_rng + b_log_t;
  m->cellb = reinterpret_cast<uint8_t*>(q);
  m->csim = reinterpret_cast<uint32_t*>(q + al(n * ggp));
  m->csg = reinterpret_cast<uint32_t*>(q + al(n * ggp) + al(n * GG * 4));
  m->ggp = (int)ggp;
  m->h = h;
  m->force_global = 0;
#ifdef PE_DEBUG_KNOBS  // A/B builds only (tools/ab_build.sh): the product library reads no environment variable
  m->force_global = getenv("PE_MCTS_GLOBAL") && atoi(getenv("PE_MCTS_GLOBAL")) != 0;
#endif
  m->n_sims = n_simulations;
  m->max_depth = max_depth;
  m->c = c_param;
  std::vector<double> lt((size_t)n_simulations + 1);
  lt[0] = -INFINITY;
  for (int k = 1; k <= n_simulations; ++k) lt[k] = std::log((double)k);  // math.log(self.visits) (:56)
  e = hipMemcpy(m->logt, lt.data(), lt.size() * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(pe_mcts_seed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, m->rng, (int)n,
                       nullptr, 0u);  // np.random.seed(e) until pe_mcts_seed
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
  }
  if (e != hipSuccess) {
    (void)hipFree(m->mem);
    delete m;
    return hip_fail(e, "pe_mcts_create");
  }
  *out = m;
  return PE_OK;
}

int pe_mcts_destroy(pe_mcts* m) {
  if (!m) return PE_OK;
  DevBind db(m->h->device);
  hipError_t e = hipFree(m->mem);
  delete m;
  return e == hipSuccess ? PE_OK : hip_fail(e, "hipFree");
}

int pe_mcts_seed(pe_mcts* m, const uint32_t* seeds, uint32_t base_seed, void* stream) {
  if (!m) return fail(PE_ERR_ARG, "null handle");
  DevBind db(m->h->device);
  if (db.err != hipSuccess) return hip_fail(db.err, "hipSetDevice");
  const int n = m->h->n;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t* dseeds = nullptr;
  if (seeds) {
    MC_HIP(hipMalloc(&dseeds, (size_t)n * 4));
    hipError_t e = hipMemcpy(dseeds, seeds, (size_t)n * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(dseeds);
      return hip_fail(e, "hipMemcpy");
    }
  }
  hipLaunchKernelGGL(pe_mcts_seed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m->rng, n, dseeds,
                     base_seed);
  hipError_t e = hipGetLastError();
  if (dseeds) {
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(dseeds);
  }
  return e == hipSuccess ? PE_OK : hip_fail(e, "pe_mcts_seed");
}

int pe_mcts_set_rng(pe_mcts* m, const uint32_t* key, const int32_t* pos) {
  if (!m || !key || !pos) return fail(PE_ERR_ARG, "null argument");
  const int n = m->h->n;
  std::vector<uint32_t> dev((size_t)n * kRngStride);
  for (int e = 0; e < n; ++e) {
    if (pos[e] < 0 || pos[e] > kMtN) return fail(PE_ERR_ARG, "pos must be in [0, 624]");
    np_to_device(key + (size_t)e * kMtN, pos[e], dev.data() + (size_t)e * kRngStride);
  }
  DevBind db(m->h->device);
  if (db.err != hipSuccess) return hip_fail(db.err, "hipSetDevice");
  MC_HIP(hipDeviceSynchronize());
  MC_HIP(hipMemcpy(m->rng, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
  return PE_OK;
}

int pe_mcts_get_rng(pe_mcts* m, uint32_t* key, int32_t* pos) {
  if (!m || !key || !pos) return fail(PE_ERR_ARG, "null argument");
  const int n = m->h->n;
  std::vector<uint32_t> dev((size_t)n * kRngStride);
  DevBind db(m->h->device);
  if (db.err != hipSuccess) return hip_fail(db.err, "hipSetDevice");
  MC_HIP(hipDeviceSynchronize());
  MC_HIP(hipMemcpy(dev.data(), m->rng, dev.size() * 4, hipMemcpyDeviceToHost));
  for (int e = 0; e < n; ++e) device_to_np(dev.data() + (size_t)e * kRngStride, key + (size_t)e * kMtN, pos + e);
  return PE_OK;
}

int pe_mcts_search(pe_mcts* m, const uint8_t* mask, int32_t* actions, int32_t* root_order, int32_t* root_visits,
                   double* root_value, void* stream) {
  if (!m || !actions) return fail(PE_ERR_ARG, "null argument");
  pe_handle* h = m->h;
  DevBind db(h->device);
  if (db.err != hipSuccess) return hip_fail(db.err, "hipSetDevice");
  MctsArgs a;
  std::memset(&a, 0, sizeof(a));
  a.st = h->st;
  a.g = h->g;
  a.rl = h->rl;
  a.n = h->n;
  a.cellw = m->cellw;
  a.ulog = m->ulog;
  a.nodes = m->nodes;
  a.rng = m->rng;
  a.n_sims = m->n_sims;
  a.max_depth = m->max_depth;
  a.c = m->c;
  a.logt = m->logt;
  a.mask = mask;
  a.actions = actions;
  a.rorder = root_order;
  a.rvisits = root_visits;
  a.rvalue = root_value;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t cells = (int64_t)h->n * h->g.GG;
  int ldsp = (h->g.GG + 3) / 4 * 4;
  if ((ldsp / 4) % 2 == 0) ldsp += 4;  // odd dword stride between lanes
  const size_t lds = 64 * ((size_t)ldsp + 4 * (size_t)kRing);
  const bool use_lds = h->g.G <= 64 && lds <= kMctsLdsMax && !m->force_global;
  if (use_lds) {
    a.cellb = m->cellb;
    a.csim = m->csim;
    a.csg = m->csg;
    a.ggp = m->ggp;
    a.ldsp = ldsp;
  }
  if (cells > 0) {
    // the steps' deferred visit-overflow writes first: the clone reads the exact counts
    if (const int fr = pe_internal_flush_vx(h, s)) return fr;
    hipLaunchKernelGGL(pe_mcts_clone_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, a);
    if (use_lds)
      hipLaunchKernelGGL(pe_mcts_search_lds_kernel, dim3((unsigned)((h->n + 63) / 64)), dim3(64), lds, s, a);
    else
      hipLaunchKernelGGL(pe_mcts_search_kernel, dim3((unsigned)((h->n + 63) / 64)), dim3(64), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? PE_OK : hip_fail(e, "pe_mcts_search");
}

#ifdef PE_MCTS_PROF
int pe_mcts_debug_prof(uint64_t* host, int64_t count) {
  if (count > (int64_t)(1 << 20) * 4) count = (int64_t)(1 << 20) * 4;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mcts_prof), (size_t)count * 8);
  return e == hipSuccess ? PE_OK : hip_fail(e, "hipMemcpyFromSymbol");
}
#endif

}  // extern "C"
