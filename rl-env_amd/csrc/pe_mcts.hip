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
// ever stops for a 624-word twist.  Draws are produced 8 at a time with all 16 loads
// in flight together; a drawn word is written back only when it is consumed, so an
// unfinished batch leaves the stream exactly at its first unconsumed position.
// mt[625] keeps this round's mt[0] (overwritten at position 0) so the host can give
// the state back in numpy's own terms (pe_mcts_get_rng).
#include <hip/hip_runtime.h>

#include <cmath>
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
struct NpStream {
  uint32_t* mt;
  int p, base, ib;  // p: position after the buffered batch; base: position of out[0]
  uint32_t cur;     // mt[p] (this round's word at p)
  uint32_t raw0;    // this round's word at position 0, if the batch holds position 0
  uint32_t out[8], nw[8];

  __device__ void open(uint32_t* m) {
    mt = m;
    p = (int)m[kMtN];
    cur = m[p];
    base = p;
    ib = 8;  // empty
  }
  __device__ void refill() {
    uint32_t nx[8], far[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int i1 = p + 1 + k, i2 = p + kMtM + k;
      i1 -= i1 >= kMtN ? kMtN : 0;
      i2 -= i2 >= kMtN ? kMtN : 0;
      nx[k] = mt[i1];
      far[k] = mt[i2];
    }
    base = p;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (p + k == 0 || p + k == kMtN) raw0 = cur;
      nw[k] = twist(cur, nx[k], far[k]);
      out[k] = temper(cur);
      cur = nx[k];
    }
    p += 8;
    p -= p >= kMtN ? kMtN : 0;
    ib = 0;
  }
  __device__ uint32_t next() {
    if (ib == 8) refill();
    uint32_t o = 0, w = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t m = 0u - (uint32_t)(k == ib);
      o |= out[k] & m;
      w |= nw[k] & m;
    }
    int pos = base + ib;
    pos -= pos >= kMtN ? kMtN : 0;
    mt[pos] = w;
    if (pos == 0) mt[kMtN + 1] = raw0;  // this round's mt[0], kept for pe_mcts_get_rng
    ++ib;
    return o;
  }
  __device__ void close() {
    int pos = ib == 8 ? p : base + ib;  // first unconsumed position
    pos -= pos >= kMtN ? kMtN : 0;
    mt[kMtN] = (uint32_t)pos;
  }
  // np.random.random(): 53 bits from two draws
  __device__ double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
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

// N, E, S, W neighbours (plantos_env.py:186) and the rover's own cell.
__device__ __forceinline__ void load_cells(const uint32_t* cw, int G, const Sim& s, uint32_t w[5]) {
  const int c = s.x * G + s.y;
  w[0] = s.x > 0 ? cw[c - G] : kOffMap;
  w[1] = s.y + 1 < G ? cw[c + 1] : kOffMap;
  w[2] = s.x + 1 < G ? cw[c + G] : kOffMap;
  w[3] = s.y > 0 ? cw[c - 1] : kOffMap;
  w[4] = cw[c];
}

__device__ __forceinline__ uint32_t sel5(const uint32_t w[5], int k) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) v |= w[j] & (0u - (uint32_t)(j == k));
  return v;
}

// PlantOSEnv.step on the sim env (plantos_env.py:160-183; watering of the fork,
// plantos_env_new.py:236-245).  Only what MCTS reads is produced: reward,
// terminated, truncated (the observation and info dict are never used by the search).
__device__ double sim_step(const MctsArgs& a, uint32_t* cw, uint2* lg, int& nlog, Sim& s, int total, int act,
                           const uint32_t w[5], bool& te, bool& tr) {
  const Rules& rl = a.rl;
  const int G = a.g.G;
  s.step += 1;                                                   // :162
  double r = rl.r_step;                                          // :164
  if (act < 4) {
    const uint32_t nw = sel5(w, act);
    if (((nw & kCodeMask) >> kCodeShift) != (uint32_t)OBST) {   // in bounds, not an obstacle (:193-195)
      const int dx = act == 0 ? -1 : (act == 2 ? 1 : 0), dy = act == 1 ? 1 : (act == 3 ? -1 : 0);
      const int oc = s.x * G + s.y, nc = oc + dx * G + dy;
      const bool never = (nw & kVisMask) == 0u;                  // :197
      if (!s.cur_expl) {                                         // explored_map[old] = 1 (:198)
        lg[nlog++] = make_uint2((uint32_t)oc, w[4]);
        cw[oc] = w[4] | kExpl;
        s.expl += 1;
      }
      lg[nlog++] = make_uint2((uint32_t)nc, nw);
      s.expl += (nw & kExpl) ? 0 : 1;                            // explored_map[new] = 2 (:200)
      cw[nc] = (nw | kExpl) + 1u;                                // visit_counts[new] += 1 (:203)
      s.x += dx;
      s.y += dy;
      s.cur_expl = true;
      r += never ? rl.r_exploration : rl.r_revisit;              // :204-207
    } else {
      r += rl.r_invalid;                                         // :208-211
    }
  } else {
    const uint32_t code = (w[4] & kCodeMask) >> kCodeShift;
    if (code == (uint32_t)THIRSTY) {                             // fork :237-240
      const int oc = s.x * G + s.y;
      lg[nlog++] = make_uint2((uint32_t)oc, w[4]);
      cw[oc] = (w[4] & ~kCodeMask) | ((uint32_t)HYD << kCodeShift);
      r += rl.r_goal;
    } else if (code == (uint32_t)HYD) {
      r += rl.r_mistake;                                         // fork :241-242
    } else {
      r += rl.r_water_empty;                                     // :221-222
    }
  }
  const double pct = ((double)s.expl / (double)total) * 100.0;  // :320-331
  te = pct >= 100.0;                                             // :176, 244-246
  tr = s.step >= rl.max_steps;                                   // :177
  if (pct >= 100.0 && !s.bonus) {                                // :179-181
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
  const uint32_t v = (uint32_t)visit_exact(a.st, g, e, row, col);
  bool ex;
  if (s.flags & F_EXPL_BITMAP)
    ex = (a.st.expl[e * g.estride + (c >> 5)] >> (c & 31)) & 1u;
  else
    ex = v > 0u;  // explored_map > 0 <=> visit > 0 (derived mode)
  a.cellw[e * (int64_t)g.GG + c] = (v & kVisMask) | (code << kCodeShift) | (ex ? kExpl : 0u);
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

// MCTS.search (:91-139) for the lane's env.
__global__ __launch_bounds__(64) void pe_mcts_search_kernel(MctsArgs a) {
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n) return;
  if (a.mask && !a.mask[e]) return;
  const Geo& g = a.g;
  const int G = g.G;
  const Scal s0 = unpack(a.st.scal[e]);
  const int total = s0.total;
  uint32_t* cw = a.cellw + e * (int64_t)g.GG;
  uint2* lg = a.ulog + e * (int64_t)(a.max_depth + 4);
  MNode* T = a.nodes + e * (int64_t)(a.n_sims + 1);
  NpStream rng;
  rng.open(a.rng + e * (int64_t)kRngStride);
  const bool root_expl = (cw[s0.x * G + s0.y] & kExpl) != 0u;

  store_node(T, 0, fresh_node(0xFFFF, 0xFF));
  int nn = 1;
  for (int sim = 0; sim < a.n_sims; ++sim) {
    Sim s;
    s.x = s0.x;
    s.y = s0.y;
    s.step = s0.step;
    s.expl = s0.expl;
    s.cur_expl = root_expl;
    s.bonus = false;  // a fresh PlantOSEnv: completion_bonus_given False (:221-243)
    int nlog = 0;
    int node = 0, depth = 0;
    bool te = false, tr = false;
    uint32_t w[5];
    MNode nd = load_node(T, 0);
    // 1. selection (:106-114)
    while ((nd.untried & 7u) == 0u && nd.nkid > 0 && depth < a.max_depth) {
      const double lv = a.logt[nd.visits];
      int best = -1;
      double bw = 0.0;
      for (int j = 0; j < nd.nkid; ++j) {
        const int ci = kid_at(nd, j);
        const MNode ch = load_node(T, ci);
        double wgt;
        if (ch.visits == 0) {
          wgt = INFINITY;
        } else {
          const double exploitation = ch.value / (double)ch.visits;                 // :55
          const double exploration = a.c * sqrt(lv / (double)ch.visits);          // :56
          wgt = exploitation + exploration;                                         // :57
        }
        if (best < 0 || wgt > bw) {  // max(): the first maximal child (:60)
          best = ci;
          bw = wgt;
        }
      }
      node = best;
      nd = load_node(T, node);
      load_cells(cw, G, s, w);
      sim_step(a, cw, lg, nlog, s, total, nd.action, w, te, tr);
      depth += 1;
      if (te || tr) break;
    }
    // 2. expansion (:117-125); depth is not advanced
    if ((nd.untried & 7u) > 0u && depth < a.max_depth) {
      const int cnt = (int)(nd.untried & 7u);
      const int k = rng.randint(cnt);
      const int act = (int)((nd.untried >> (3 + 3 * k)) & 7u);
      const uint32_t below = nd.untried & ((1u << (3 + 3 * k)) - 1u) & ~7u;
      const uint32_t above = (nd.untried >> (3 + 3 * (k + 1))) << (3 + 3 * k);
      nd.untried = below | above | (uint32_t)(cnt - 1);
      const int ci = nn++;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (j == nd.nkid) nd.kid[j] = (uint16_t)ci;
      nd.nkid += 1;
      store_node(T, node, nd);
      load_cells(cw, G, s, w);
      sim_step(a, cw, lg, nlog, s, total, act, w, te, tr);
      store_node(T, ci, fresh_node(node, act));
      node = ci;
    }
    // 3. rollout (:141-168)
    double tot = 0.0;
    for (int d = depth; d < a.max_depth; ++d) {
      load_cells(cw, G, s, w);
      int act;
      if (rng.random() < 0.7) {                                  // :180
        // _exploration_heuristic (:187-219): first strictly least-visited valid move
        int best = -1;
        uint32_t minv = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = ((w[q] & kCodeMask) >> kCodeShift) != (uint32_t)OBST;
          const uint32_t v = w[q] & kVisMask;
          if (ok && (best < 0 || v < minv)) {
            best = q;
            minv = v;
          }
        }
        act = best >= 0 ? best : rng.randint(5);
      } else {
        act = rng.randint(5);                                    // :183
      }
      const double r = sim_step(a, cw, lg, nlog, s, total, act, w, te, tr);
      tot += r;
      if (te || tr) {
        if (((double)s.expl / (double)total) * 100.0 >= 100.0) tot += 500.0;  // :160-163
        break;
      }
    }
    // 4. backpropagation (:130-134)
    for (int i = node; i != 0xFFFF;) {
      MNode b = load_node(T, i);
      b.visits += 1;
      b.value += tot;
      store_node(T, i, b);
      i = b.parent;
    }
    // restore the sim env for the next simulation (a new _copy_env_state)
    for (int k = nlog - 1; k >= 0; --k) {
      const uint2 u = lg[k];
      cw[u.x] = u.y;
    }
  }
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

struct pe_mcts {
  pe_handle* h;
  int n_sims, max_depth;
  double c;
  void* mem;
  uint32_t* cellw;
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
  const size_t b_cell = al(n * GG * 4), b_log = al(n * (size_t)(max_depth + 4) * 8),
               b_node = al(n * (size_t)(n_simulations + 1) * sizeof(MNode)), b_rng = al(n * kRngStride * 4),
               b_log_t = al((size_t)(n_simulations + 1) * 8);
  pe_mcts* m = new (std::nothrow) pe_mcts();
  if (!m) return fail(PE_ERR_NOMEM, "host allocation failed");
  hipError_t e = hipMalloc(&m->mem, b_cell + b_log + b_node + b_rng + b_log_t);
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
  m->h = h;
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
  if (cells > 0) {
    hipLaunchKernelGGL(pe_mcts_clone_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(pe_mcts_search_kernel, dim3((unsigned)((h->n + 63) / 64)), dim3(64), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? PE_OK : hip_fail(e, "pe_mcts_search");
}

}  // extern "C"
