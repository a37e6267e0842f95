// pe_coop.hpp -- wave-cooperative auto-reset: one env's reset() by all 64 lanes.
//
// The lane-per-env reset (gen_map + build_obs_fresh in pe_device.hpp /
// plantos_batch.hip) is a serial chain of ~60k instructions per env: scans of
// the grid image per plant pick, rejection loops, per-lane row stores.  That is
// fine when every lane of the commit wave has an env to reset (a synchronized
// batch truncating together), but inside a step it is the whole block's latency:
// a step in which ANY env of a block auto-resets took ~100 us instead of ~11 us,
// and steady-state training (episodes ending at different steps) resets a few
// envs in every step.
//
// Here the wave that owns a done env generates its map cooperatively: lane r
// holds grid row r in registers (G <= 64), the per-row counts of candidate cells
// are prefix-summed across lanes once, and each draw of random.sample /
// random.choice (plantos_env.py:366-372) finds its row with one ballot and its
// column with a ballot over the row word's set bits.  The draws are the same
// device-rng (Philox) stream in the same order as gen_map, so the map is the one
// gen_map / the oracle's po_reset_philox produce (the GPU parity tests check it).
// The stream itself is generated 64 blocks at a time (lane k: block base+k) and
// each draw is one readlane.  The terminal info, the fresh observation (lane i
// marches ray i over rows fetched from their owner lanes) and the row stores are
// wave-parallel too.
//
// MAXW: grid-row words a lane holds (1 when G + 2R <= 32, else up to kCoopWPR).
#pragma once
#include "../../include/plantos_batch.h"
#include "pe_device.hpp"

namespace pe {

#ifdef PE_COOP_TIMING  // tools/diag/coop_bench.hip only: phase cycle stamps of block 0
// (each stamp is a global read-modify-write: a few hundred cycles of its own)
__device__ unsigned long long g_coop_t[8];
#define PE_COOP_T(k)                                                     \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    const unsigned long long _t = __builtin_readcyclecounter();          \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_coop_t[k] += _t;          \
  } while (0)
#else
#define PE_COOP_T(k) \
  do {               \
  } while (0)
#endif

constexpr int kCoopWPR = 4;     // row words per lane: G + 2R <= 128
constexpr int kCoopMaxDone = 8;  // done envs per block up to which the cooperative path is taken
constexpr int kPrefetchEvery = 256;  // steps between prefetch launches (queue mode): desynchronized
                                     // 20x20 step 12.41 / 12.22 / 12.13 / 12.11 us at 64 / 128 / 256 / 512
                                     // (profiles/r2b_ab_prefetch.jsonl)

// The cooperative path covers the original map generator with one grid row per
// lane; everything else takes the lane-per-env path.
// The step kernel gives each of its 4 waves G x WPR words of LDS scratch after the
// reset staging (1296 B) in the window-row region, (2R+3) x 512 + 7 x 256 B.
__host__ __device__ constexpr bool coop_reset_ok(int G, int R, int WPR, int NW, int P, int C, int map_algo) {
  return G <= 64 && WPR <= kCoopWPR && NW <= kMaxNW && P <= 128 && C <= 64 && map_algo == 0 &&
         1296 + 4 * 8 * G * WPR <= (2 * R + 3) * 512 + 7 * 256;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ void lds_or64(uint64_t* p, uint64_t v) {
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, src) |
         ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), src) << 32);
}

// bit position of the jj-th (0-based) set bit of the wave-uniform mask m
__device__ __forceinline__ int nth_set_bit(uint64_t m, int jj, int lane) {
  const bool bit = (m >> lane) & 1ull;
  const int rank = __popcll(m & ((1ull << lane) - 1ull));
  const uint64_t hit = __ballot(bit && rank == jj);
  return __ffsll((unsigned long long)hit) - 1;
}

// A lane's grid row: MAXW named words, read and written by mask-selects.  (A
// word array indexed by a computed word number becomes a dynamically indexed
// stack array, i.e. scratch memory for the whole kernel.)
template <int MAXW>
struct Row4 {
  uint64_t w0, w1, w2, w3;
  __device__ __forceinline__ uint64_t get(int i) const {
    if constexpr (MAXW == 1) {
      return w0;
    } else {
      const uint64_t m0 = 0ull - (uint64_t)(i == 0), m1 = 0ull - (uint64_t)(i == 1);
      const uint64_t m2 = 0ull - (uint64_t)(i == 2), m3 = 0ull - (uint64_t)(i == 3);
      return (w0 & m0) | (w1 & m1) | (w2 & m2) | (w3 & m3);
    }
  }
  __device__ __forceinline__ void set(int i, uint64_t v) {
    if constexpr (MAXW == 1) {
      w0 = v;
    } else {
      w0 = i == 0 ? v : w0;
      w1 = i == 1 ? v : w1;
      w2 = i == 2 ? v : w2;
      w3 = i == 3 ? v : w3;
    }
  }
};

// The device-rng reset stream (pe_device.hpp Stream: Philox4x32-10 blocks 0, 1,
// 2, ... keyed by (seed, env, episode), words x, y, z, w in order) for a whole
// wave: lane k computes block base+k (one VALU Philox pass = 256 words; a map
// takes ~50), transposed once so that word 64j+k sits in register cj of lane k;
// a draw is then one uniform register select and one readlane -- no branches,
// no serial scalar multiply chain.  (The selects are mask arithmetic: a
// divergent branch around them would make the cursor look divergent.)
struct WaveStream {
  uint32_t k0, k1, env, episode, base;
  uint32_t c0, c1, c2, c3;  // lane k: words k, 64+k, 128+k, 192+k of blocks base..base+63
  int pos;                  // next word (uniform)
  __device__ __forceinline__ static uint32_t pick4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int i) {
    const uint32_t m0 = 0u - (uint32_t)(i == 0), m1 = 0u - (uint32_t)(i == 1);
    const uint32_t m2 = 0u - (uint32_t)(i == 2), m3 = 0u - (uint32_t)(i == 3);
    return (a & m0) | (b & m1) | (c & m2) | (d & m3);
  }
  __device__ __forceinline__ void fill(int lane) {
    const uint4 b = philox(make_uint4(base + (uint32_t)lane, env, episode, kDomainReset), k0, k1);
    uint32_t t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // word 64j + lane = component lane&3 of block 16j + lane/4
      const int src = 16 * j + (lane >> 2);
      t[j] = pick4((uint32_t)__shfl((int)b.x, src), (uint32_t)__shfl((int)b.y, src),
                   (uint32_t)__shfl((int)b.z, src), (uint32_t)__shfl((int)b.w, src), lane & 3);
    }
    c0 = t[0];
    c1 = t[1];
    c2 = t[2];
    c3 = t[3];
    pos = 0;
  }
  // restart the batch at the block holding word `pos`: words pos .. pos+252 available
  __device__ __forceinline__ void realign(int lane) {
    const uint32_t a = base * 4u + (uint32_t)pos;  // absolute word index
    base = a >> 2;
    fill(lane);
    pos = (int)(a & 3u);
  }
  // word q (< 256) of the batch, for each lane its own q
  __device__ __forceinline__ uint32_t word_at(int q) const {
    const int src = q & 63;
    return pick4((uint32_t)__shfl((int)c0, src), (uint32_t)__shfl((int)c1, src), (uint32_t)__shfl((int)c2, src),
                 (uint32_t)__shfl((int)c3, src), q >> 6);
  }
  __device__ __forceinline__ void init(uint64_t seed, uint32_t env_id, uint32_t ep, int lane) {
    k0 = (uint32_t)seed;
    k1 = (uint32_t)(seed >> 32);
    env = env_id;
    episode = ep;
    base = 0;
    fill(lane);
  }
  __device__ __forceinline__ uint32_t next(int lane) {
    if (pos == 256) {  // rare: a map takes ~50 words
      base += 64;
      fill(lane);
    }
    const int p = pos++;
    return (uint32_t)__builtin_amdgcn_readlane((int)pick4(c0, c1, c2, c3, p >> 6), p & 63);
  }
  // random.py:239-248 _randbelow_with_getrandbits (getrandbits(k) = u32 >> (32-k))
  __device__ __forceinline__ uint32_t below(uint32_t n, int lane) {
    if (!n) return 0;
    const int k = 32 - __clz(n);
    uint32_t r = next(lane) >> (32 - k);
    while (r >= n) r = next(lane) >> (32 - k);
    return r;
  }
  // random.random()
  __device__ __forceinline__ double random53(int lane) {
    const uint32_t a = next(lane) >> 5, b = next(lane) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }
};

// per-lane position of the jj-th (0-based) set bit of m (jj < popcount(m))
__device__ __forceinline__ int select_bit(uint64_t m, int jj) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int low = __popcll(m & ((1ull << w) - 1ull));
    const bool up = jj >= low;
    jj -= up ? low : 0;
    m = up ? (m >> w) : m;
    pos += up ? w : 0;
  }
  return pos;
}

// code `code` at padded column pcol of this lane's row words
template <int MAXW>
__device__ __forceinline__ void coop_set(Row4<MAXW>& rw, int pcol, int code) {
  const int bit = 2 * pcol;
  const uint64_t v = rw.get(bit >> 6);
  rw.set(bit >> 6, (v & ~(3ull << (bit & 63))) | ((uint64_t)code << (bit & 63)));
}

// Candidate-cell mask of one row word: kind 0 = not an obstacle (random.sample's
// `available`, :358-366), kind 1 = empty (the rover's `available - plants`, :370-372)
__device__ __forceinline__ uint64_t cand_mask(uint64_t v, uint64_t real, int kind) {
  const uint64_t lo = v & kEven64, hi = (v >> 1) & kEven64;
  return kind == 0 ? (real & ~(lo & ~hi)) : (real & ~(lo | hi));
}

// The j-th candidate cell (row-major) given this lane's inclusive/exclusive
// prefix counts; returns the row and the padded column (both uniform).
template <int MAXW>
__device__ __forceinline__ void coop_nth_cell(const Row4<MAXW>& rw, int WPR, const uint64_t* real, int incl,
                                              int excl, int j, int kind, int lane, int& row, int& pcol) {
  row = __popcll(__ballot(incl <= j));  // rows before it hold <= j candidates
  int jj = j - __builtin_amdgcn_readlane(excl, row);
  pcol = 0;
#pragma unroll
  for (int w = 0; w < MAXW; ++w) {
    if (MAXW == 1 || w < WPR) {
      const uint64_t m = cand_mask(readlane64(rw.get(w), row), real[w], kind);
      const int c = __popcll(m);
      if (MAXW == 1 || (jj >= 0 && jj < c)) pcol = w * 32 + nth_set_bit(m, jj, lane) / 2;
      jj -= c;
    }
  }
}

// gen_map (pe_device.hpp, original algorithm) for one env by one wave: the same
// Philox draws in the same order, rows in the lanes' registers.  Returns the new
// scalars (uniform); rw holds the lane's grid row.  tab: the handle's tables in
// global memory (uniform words: scalar loads).
// The obstacle clusters of gen_map for G >= 5 (see coop_gen_map): OR-s the
// cluster cells into scr (the caller merges); dbg (diagnostics, may be NULL)
// receives cx, cy, size of each cluster.
__device__ inline void coop_clusters(const Geo& g, int clusters, WaveStream& rng, uint64_t* scr, int lane,
                                     int* dbg) {
  const int G = g.G, R = g.R;
  const int k1 = 32 - __clz((uint32_t)(G - 4));
  int state = 0, emitted = 0;  // uniform: draw state at the round start, values emitted
  int carry1 = 0, carry2 = 0;  // the last two values emitted before this round (cy, cx)
  while (emitted < 3 * clusters) {
    if (rng.pos + 64 > 256) rng.realign(lane);
    const uint32_t wd = rng.word_at(rng.pos + lane);
    const bool a1 = (wd >> (32 - k1)) < (uint32_t)(G - 4), a2 = (wd >> 30) < 2u;
    // map: s -> next state; 2 bits per state
    int f = (a1 ? 1 : 0) | ((a1 ? 2 : 1) << 2) | ((a2 ? 0 : 2) << 4);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // F(lane) = f(lane) o F(lane - 1)
      const int t = __shfl_up(f, o);
      if (lane >= o)
        f = ((f >> (2 * (t & 3))) & 3) | (((f >> (2 * ((t >> 2) & 3))) & 3) << 2) |
            (((f >> (2 * ((t >> 4) & 3))) & 3) << 4);
    }
    // (the shuffle outside the select: inside `lane == 0 ? ... : __shfl_up()` it is
    // evaluated with lane 0 inactive, and lane 1 then reads an inactive lane)
    const int fup = __shfl_up(f, 1);
    const int fprev = lane == 0 ? (0 | (1 << 2) | (2 << 4)) : fup;
    const int st = (fprev >> (2 * state)) & 3;  // draw state before this word
    const bool emit = st < 2 ? a1 : a2;
    const int val = 2 + (int)(st < 2 ? (wd >> (32 - k1)) : (wd >> 30));
    const uint64_t em = __ballot(emit);
    const int rank = emitted + __popcll(em & ((1ull << lane) - 1ull));
    const bool use = emit && rank < 3 * clusters;
    // the two emitting lanes before this one (or the carried values)
    const uint64_t before = em & ((1ull << lane) - 1ull);
    const int p1 = before ? 63 - __clzll((long long)before) : -1;
    const uint64_t before2 = p1 >= 0 ? (before & ~(1ull << p1)) : 0ull;
    const int p2 = before2 ? 63 - __clzll((long long)before2) : -1;
    const int v1 = __shfl(val, p1 < 0 ? 0 : p1), v2 = __shfl(val, p2 < 0 ? 0 : p2);
    if (use && st == 2) {  // this lane completes a cluster
      const int cy = p1 >= 0 ? v1 : carry1;
      const int cx = p2 >= 0 ? v2 : (p1 >= 0 ? carry1 : carry2);
      const int size = val;
      if (dbg) {
        dbg[3 * (rank / 3)] = cx;
        dbg[3 * (rank / 3) + 1] = cy;
        dbg[3 * (rank / 3) + 2] = size;
      }
      for (int dx = 0; dx < size; ++dx) {
        const int ox = cx + dx - size / 2;
        if (ox < 0 || ox >= G) continue;
        for (int dy = 0; dy < size; ++dy) {
          const int oy = cy + dy - size / 2;
          if (0 <= oy && oy < G) {
            const int bit = 2 * (oy + R);
            lds_or64(scr + ox * g.WPR + (bit >> 6), 1ull << (bit & 63));  // code OBST
          }
        }
      }
    }
    const int nem = __popcll(em), take = 3 * clusters - emitted;
    if (nem >= take) {  // the last cluster's size: consume through that word
      rng.pos += nth_set_bit(em, take - 1, lane) + 1;
      emitted += take;
    } else {
      // carry the last two emitted values (by rank) into the next round
      if (nem >= 2) {
        const int l1 = 63 - __clzll((long long)em), l2 = 63 - __clzll((long long)(em & ~(1ull << l1)));
        carry1 = __shfl(val, l1);
        carry2 = __shfl(val, l2);
      } else if (nem == 1) {
        carry2 = carry1;
        carry1 = __shfl(val, 63 - __clzll((long long)em));
      }
      state = (__builtin_amdgcn_readlane(f, 63) >> (2 * state)) & 3;  // through all 64 words
      rng.pos += 64;
      emitted += nem;
    }
  }
}

// LDS scratch of one wave for the cooperative reset: G rows x WPR words (the
// obstacle / plant bits of a round, OR-ed in by the lanes that drew them).
__host__ __device__ constexpr int coop_scratch_words(int G, int WPR) { return G * WPR; }

// OR the round's bits (scr, G x WPR words, written with LDS atomics) into each
// lane's row, and clear them for the next round.
template <int MAXW>
__device__ __forceinline__ void coop_merge(Row4<MAXW>& rw, uint64_t* scr, int WPR, int G, int lane) {
  if (lane < G) {
#pragma unroll
    for (int w = 0; w < MAXW; ++w)
      if (MAXW == 1 || w < WPR) {
        rw.set(w, rw.get(w) | scr[lane * WPR + w]);
        scr[lane * WPR + w] = 0ull;
      }
  }
}

// LT: `tab` is the caller's LDS copy of the tables, read as LDS.  (A generic pointer that may
// hold it or st.tab turns every table read into a flat load, whose wait is vmcnt(0) as well:
// behind every store the wave has in flight.)
typedef const __attribute__((address_space(3))) Tables* LdsTables;

template <int MAXW, bool LT = false>
__device__ inline Scal coop_gen_map(const Geo& g, const Rules& rl, const Tables* tab, Row4<MAXW>& rw,
                                    uint32_t env_id, uint32_t episode, int lane, uint64_t* scr) {
  const int G = g.G, R = g.R;
  const bool own = lane < G;
  uint64_t real[MAXW];
#pragma unroll
  for (int w = 0; w < MAXW; ++w) {
    const bool in = MAXW == 1 || w < g.WPR;
    real[w] = in ? (LT ? ((LdsTables)tab)->grid_real[w] : tab->grid_real[w]) : 0ull;
    rw.set(w, own && in ? (LT ? ((LdsTables)tab)->grid_pad[w] : tab->grid_pad[w]) : 0ull);
  }
  PE_COOP_T(0);
  WaveStream rng;
  rng.init(rl.seed, env_id, episode, lane);
  PE_COOP_T(1);
  if (own)
    for (int w = 0; w < g.WPR; ++w) scr[lane * g.WPR + w] = 0ull;
  // obstacle clusters, plantos_env.py:341-354: cx = 2 + below(G-4), cy = 2 +
  // below(G-4), size = 2 + below(2) per cluster.  64 words per round: which draw
  // a word serves depends on the words before it (rejections), so each word's
  // effect on the draw state {cx, cy, size} is a 3-state map, and an inclusive
  // scan of map compositions gives every lane its state; the accepting lanes
  // emit the values, each size-lane assembles its cluster from the two emitting
  // lanes before it (or the previous round's carry) and ORs its obstacle bits in.
  const int clusters = rl.O / 3;
  if (G - 4 >= 1) {
    coop_clusters(g, clusters, rng, scr, lane, nullptr);
    coop_merge(rw, scr, g.WPR, G, lane);
  } else {  // G <= 4: below(0) draws nothing; the plain sequential form
    for (int q = 0; q < clusters; ++q) {
      const int cx = 2 + (int)rng.below((uint32_t)(G - 4), lane);
      const int cy = 2 + (int)rng.below((uint32_t)(G - 4), lane);
      const int size = 2 + (int)rng.below(2u, lane);
      const int x0 = cx - size / 2;
      if (own && lane >= x0 && lane < x0 + size)
        for (int dy = 0; dy < size; ++dy) {
          const int oy = cy + dy - size / 2;
          if (0 <= oy && oy < G) coop_set(rw, oy + R, OBST);
        }
    }
  }
  PE_COOP_T(2);
  int c0 = 0, nob = 0;
#pragma unroll
  for (int w = 0; w < MAXW; ++w) {
    const uint64_t v = rw.get(w), rl_w = own ? real[w] : 0ull;
    nob += __popcll(v & ~(v >> 1) & rl_w & kEven64);
    c0 += __popcll(cand_mask(v, rl_w, 0));
  }
  const int nfree = g.GG - wave_sum(nob);
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
  // random.sample(list(available), P) (:366), 64 draws per round.  The sequential
  // form is: below(nfree) (words whose top k bits are >= nfree are skipped), map
  // to the j-th non-obstacle cell, redraw if that cell is already chosen.  Plants
  // are not obstacles, so the per-row counts stay valid for every pick; the
  // accepted values are the stream's words in order, so 64 consecutive words are
  // mapped to cells at once (row: binary search over the rows' prefix counts;
  // column: per-lane bit select in the row word fetched from its owner lane), and
  // the first (P - picked) of them whose cell is free and not hit by an earlier
  // lane of the round become the next picks -- the sequential loop's result.
  // Pick i is kept in lane i % 64 (registers pk0 / pk1).
  const int i0 = wave_incl_scan(c0, lane), e0 = i0 - c0;
  PE_COOP_T(3);
  int pk0 = 0, pk1 = 0;
  {
    const int kb = 32 - __clz((uint32_t)nfree);
    int picked = 0;
    while (picked < rl.P) {
      if (rng.pos + 64 > 256) rng.realign(lane);
      const uint32_t jv = rng.word_at(rng.pos + lane) >> (32 - kb);
      const bool acc = jv < (uint32_t)nfree;
      int row = 0;  // rows whose inclusive count is <= jv
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1) {
        const int probe = __shfl(i0, row + st - 1);
        row += (uint32_t)probe <= jv ? st : 0;
      }
      row = acc ? row : 0;
      int jj = (int)jv - __shfl(e0, row);
      Row4<MAXW> rv{0ull, 0ull, 0ull, 0ull};
#pragma unroll
      for (int w = 0; w < MAXW; ++w)
        if (MAXW == 1 || w < g.WPR) rv.set(w, shfl64(rw.get(w), row));
      int col = 0;
#pragma unroll
      for (int w = 0; w < MAXW; ++w) {
        if (MAXW == 1 || w < g.WPR) {
          const uint64_t m = cand_mask(rv.get(w), real[w], 0);
          const int c = __popcll(m);
          if (jj >= 0 && jj < c) col = w * 32 + select_bit(m, jj) / 2;
          jj -= c;
        }
      }
      const bool valid = acc && ((rv.get((2 * col) >> 6) >> ((2 * col) & 63)) & 3u) == EMPTY;
      const int cell = row * G + col - R;
      bool dup = false;  // an earlier valid lane of this round chose the same cell
      for (uint64_t um = __ballot(valid); um;) {
        const int t = __ffsll((unsigned long long)um) - 1;
        um &= um - 1;
        dup = dup || (t < lane && __builtin_amdgcn_readlane(cell, t) == cell);
      }
      const bool surv = valid && !dup;
      const uint64_t sm = __ballot(surv);
      const int need = rl.P - picked, nsurv = __popcll(sm);
      const int rank = __popcll(sm & ((1ull << lane) - 1ull));
      const bool take = surv && rank < need;
      // words consumed: through the last pick taken, else the whole round
      rng.pos += nsurv >= need ? nth_set_bit(sm, need - 1, lane) + 1 : 64;
      // the picks of the round: plant bits into the owner rows (LDS atomics); lane L
      // keeps pick L (pk0) / L + 64 (pk1), pulled from the lane that took it (the
      // rho-th survivor, rho = its rank in the round)
      if (take) {
        const int bit = 2 * col;
        lds_or64(scr + row * g.WPR + (bit >> 6), (uint64_t)HYD << (bit & 63));
      }
      const int ntake = nsurv < need ? nsurv : need;
      const int rho = (lane - picked) & 63;
      const int got = __shfl(cell, rho < ntake ? select_bit(sm, rho) : 0);
      pk0 = lane >= picked && lane < picked + ntake ? got : pk0;
      pk1 = lane + 64 >= picked && lane + 64 < picked + ntake ? got : pk1;
      coop_merge(rw, scr, g.WPR, G, lane);
      picked += ntake;
    }
  }
  PE_COOP_T(4);
  // thirsty draws in sample order, plantos_env.py:367-369: random() = 2 words
  // each, no rejection -- pick i draws words 2i, 2i+1 after the sample
  for (int base_i = 0; base_i < rl.P; base_i += 64) {
    const int cnt = rl.P - base_i < 64 ? rl.P - base_i : 64;
    if (rng.pos + 2 * cnt > 256) rng.realign(lane);
    const uint32_t a = rng.word_at(rng.pos + 2 * lane) >> 5, b = rng.word_at(rng.pos + 2 * lane + 1) >> 6;
    const double r = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
    const bool th = lane < cnt && r < rl.p_thirsty;
    const int cell = base_i == 0 ? pk0 : pk1;
    rng.pos += 2 * cnt;
    if (th) {  // hydrated (2) -> thirsty (3): the low bit of the plant's code
      const int bit = 2 * (cell % G + R);
      lds_or64(scr + (cell / G) * g.WPR + (bit >> 6), 1ull << (bit & 63));
    }
    coop_merge(rw, scr, g.WPR, G, lane);
  }
  PE_COOP_T(5);
  // rover: choice(list(available - plants)), plantos_env.py:370-372
  int c1 = 0;
#pragma unroll
  for (int w = 0; w < MAXW; ++w) c1 += __popcll(cand_mask(rw.get(w), own ? real[w] : 0ull, 1));
  const int i1 = wave_incl_scan(c1, lane);
  int row, pcol;
  coop_nth_cell(rw, g.WPR, real, i1, i1 - c1, (int)rng.below((uint32_t)(nfree - rl.P), lane), 1, lane, row, pcol);
  s.x = row;
  s.y = pcol - R;
  PE_COOP_T(6);
  return s;
}

// _get_info (plantos_env.py:317-336) of env e's current state by one wave
// (write_info's columns), in two halves so that a caller can issue the row loads
// before other memory work and wait for them later: coop_info_rows loads lane r's
// grid row r (sc1 load (L2): the row may hold a word another lane of this wave just
// stored), coop_info_store reduces and writes the row.  s: the env's scalars
// (uniform); wfix: see write_info.
template <int MAXW>
__device__ __forceinline__ Row4<MAXW> coop_info_rows(const State& st, const Geo& g, int64_t e, int lane) {
  Row4<MAXW> r{0ull, 0ull, 0ull, 0ull};
  if (lane < g.G) {
#pragma unroll
    for (int w = 0; w < MAXW; ++w)
      if (MAXW == 1 || w < g.WPR)
        r.set(w, __hip_atomic_load(st.grid + e * g.gstride + (int64_t)lane * g.WPR + w, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT));
  }
  return r;
}

template <int MAXW, bool LT = false>
__device__ inline void coop_info_store(const State& st, const Geo& g, const Row4<MAXW>& rows, const Scal& s, int32_t* o,
                                       int lane, int wfix = 0, const Tables* tab = nullptr) {
  const Tables* T = tab ? tab : st.tab;  // the caller's LDS copy, if it has one
  int th = 0, hy = 0;
  if (lane < g.G) {
#pragma unroll
    for (int w = 0; w < MAXW; ++w)
      if (MAXW == 1 || w < g.WPR) {
        const uint64_t v = rows.get(w);
        const uint64_t lo = v & kEven64, hi = (v >> 1) & kEven64;
        const uint64_t real = LT ? ((LdsTables)tab)->grid_real[w] : T->grid_real[w];
        th += __popcll(lo & hi & real);   // sum(plants.values())     :318
        hy += __popcll(~lo & hi & real);  // len(plants) - thirsty    :319
      }
  }
  th = wave_sum(th) - wfix;
  hy = wave_sum(hy) + wfix;
  int v = 0;
  switch (lane) {
    case 0: v = s.x; break;                             // rover_position     :324
    case 1: v = s.y; break;
    case 2: v = th; break;
    case 3: v = hy; break;
    case 4: v = th + hy; break;                         // total_plants       :327
    case 5: v = s.step; break;                          // step_count         :328
    case 6: v = s.expl; break;                          // explored_cells     :320
    case 7: v = s.total; break;                         // total_cells        :321
    case 8: v = (s.flags & F_COLLIDED) ? 1 : 0; break;  // collided_with_wall :333
    case 9: v = s.coll; break;                          // total_collisions   :334
    case 10: v = (int)((s.flags >> 2) & 7u); break;     // error flags (PE_S_POISONED layout)
    default: break;
  }
  if (lane < PE_NINFO) o[lane] = v;
}

template <int MAXW, bool LT = false>
__device__ inline void coop_write_info(const State& st, const Geo& g, int64_t e, const Scal& s, int32_t* o, int lane,
                                       int wfix = 0, const Tables* tab = nullptr) {
  coop_info_store<MAXW, LT>(st, g, coop_info_rows<MAXW>(st, g, e, lane), s, o, lane, wfix, tab);
}

// Prefetched resets: the map of an env's NEXT reset depends only on (seed, env,
// episode counter) -- never on how the current episode goes -- so it is generated
// ahead of time, in batches, by pe_prefetch_kernel (one wave per env, thousands of
// envs per launch: throughput, not latency), and the step kernel's auto-reset
// copies it in (one memory round trip) instead of generating it on the critical
// path of its block.  A record is valid for the reset whose episode counter is
// scal.w - 1 (coop_gen_map returns episode + 1); scal.w == 0: no record
// (struct Prefetch, pe_device.hpp).

// Env e's prefetched reset record, loaded (PfLoad) before the caller's other
// memory round trips (terminal info) and taken (coop_take_prefetched) after them:
// if the record holds the reset of episode counter `episode`, its scalars go to s,
// its rows to rw and its fresh obs row (D <= 64 * KD floats) to out.  Short rows
// come in with the record (one round trip); longer ones after the check
// (registers).
// OT: the record's obs row type -- floats, or (a byte-coded handle) D byte codes,
// loaded early as 4-code words (lane k: codes 4k..4k+3; the row is 16-B aligned and
// padded to ostride, so the last word stays inside it) and written to a byte-coded
// tile row at the take.
template <int MAXW, int KD>
struct PfLoad {
  static constexpr bool kEarly = KD <= 2;
  uint4 ps;
  Row4<MAXW> rw;
  float ov[kEarly ? KD : 1];  // (codes: 4-code words, bit-cast)
};

template <int MAXW, int KD, typename OT = float>
__device__ __forceinline__ void coop_load_prefetched(const Prefetch& pf, const Geo& g, int64_t e,
                                                     PfLoad<MAXW, KD>& L, int lane) {
  L.ps = pf.scal[e];
  L.rw = Row4<MAXW>{0ull, 0ull, 0ull, 0ull};
  if (lane < g.G) {
    const uint64_t* src = pf.grid + e * g.gstride + (int64_t)lane * g.WPR;
#pragma unroll
    for (int w = 0; w < MAXW; ++w)
      if (MAXW == 1 || w < g.WPR) L.rw.set(w, src[w]);
  }
  if constexpr (PfLoad<MAXW, KD>::kEarly) {
    if constexpr (sizeof(OT) == 1) {
      const uint32_t* osrc = reinterpret_cast<const uint32_t*>(pf_obs_row(pf, e));
      const int nw = (g.D + 3) >> 2;
#pragma unroll
      for (int j = 0; j < KD; ++j) {  // (unconditional, clamped: a select on the loaded word was waited out
                                      // at once; the take writes only the codes k < D)
        const int kk = lane + 64 * j;
        L.ov[j] = __uint_as_float(osrc[kk < nw ? kk : nw - 1]);
      }
    } else {
      const float* osrc = pf_obs_row(pf, e);
#pragma unroll
      for (int j = 0; j < KD; ++j) L.ov[j] = lane + 64 * j < g.D ? osrc[lane + 64 * j] : 0.0f;
    }
  }
}

template <int MAXW, int KD, typename OT = float>
__device__ __forceinline__ bool coop_take_prefetched(const Prefetch& pf, const Geo& g, int64_t e, uint32_t episode,
                                                     const PfLoad<MAXW, KD>& L, Row4<MAXW>& rw, Scal& s, OT* out,
                                                     int lane) {
  const uint32_t key = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.ps.w);
  if (key != episode + 1u) return false;
  s = unpack(make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)L.ps.x),
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)L.ps.y),
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)L.ps.z), key));
  rw = L.rw;
  if constexpr (PfLoad<MAXW, KD>::kEarly) {
    if constexpr (sizeof(OT) == 1) {
#pragma unroll
      for (int j = 0; j < KD; ++j) {
        const int k = 4 * (lane + 64 * j);
        const uint32_t w = __float_as_uint(L.ov[j]);
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (k + b < g.D) out[k + b] = (OT)(w >> (8 * b));
      }
    } else {
#pragma unroll
      for (int j = 0; j < KD; ++j)
        if (lane + 64 * j < g.D) out[lane + 64 * j] = L.ov[j];
    }
  } else {
    const OT* osrc = reinterpret_cast<const OT*>(pf_obs_row(pf, e));
    for (int k = lane; k < g.D; k += 64) out[k] = osrc[k];
  }
  return true;
}

// The state writes of reset() for env e by one wave, given its new map (rows in
// the lanes' registers) and scalars s: grid rows and visit rows (the new episode's
// slot) to HBM (lane r writes row r), the curriculum's carried-visits mode as
// new_episode_visits.
// keep: CurriculumWrapper keeps the previous visit counts.
// Fresh visit rows of a new episode (all zero, pads 10, visit[rover] = 1,
// plantos_env.py:146-147) into its slot, lane r writing row r.
template <bool LT = false>
__device__ inline void coop_fresh_visits(const State& st, const Geo& g, int64_t e, const Scal& s, int lane,
                                         const Tables* tab) {
  if (lane < g.G) {
    uint32_t* vb = vis_env(st, g, e, s.episode) + (int64_t)lane * g.NW;
    const int bit = 4 * (s.y + 2);
    const bool rover = lane == s.x && !(s.flags & F_NOROOM);
    for (int w = 0; w < g.NW; ++w) {
      uint32_t v = LT ? ((LdsTables)tab)->vis_pad[w] : (tab ? tab : st.tab)->vis_pad[w];
      if (rover && w == (bit >> 5)) v = (v & ~(0xFu << (bit & 31))) | (1u << (bit & 31));
      vb[w] = v;
    }
  }
}

// taken: s is a prefetched record's, whose fresh visit rows the prefetch kernel already
// wrote into the new episode's slot (pe_device.hpp vis_env): no visit row is stored.
template <int MAXW, bool LT = false>
__device__ inline Scal coop_apply_reset(const State& st, const Geo& g, int64_t e, Scal s, bool keep,
                                        const Row4<MAXW>& rw, int lane,
                                        const Tables* tab = nullptr, bool taken = false) {
  if ((s.flags & F_NOROOM) && lane == 0) atomicOr(st.err_bits, F_NOROOM);
  if (lane < g.G) {
    uint64_t* gb = st.grid + e * g.gstride + (int64_t)lane * g.WPR;
#pragma unroll
    for (int w = 0; w < MAXW; ++w)
      if (MAXW == 1 || w < g.WPR) gb[w] = rw.get(w);
  }
  if (!keep && !taken) {  // reset_visits: all zero (pads 10), visit[rover] = 1 (:146-147)
    coop_fresh_visits<LT>(st, g, e, s, lane, tab);
  } else if (keep) {  // the previous episode's rows carried into the new slot, explored map restarted
    if (lane < g.G) {
      const uint32_t* src = vis_env(st, g, e, s.episode - 1u) + (int64_t)lane * g.NW;
      uint32_t* dst = vis_env(st, g, e, s.episode) + (int64_t)lane * g.NW;
      for (int w = 0; w < g.NW; ++w) dst[w] = src[w];
    }
    const int rc = s.x * g.G + s.y;
    for (int w = lane; w < g.estride; w += 64)
      st.expl[e * g.estride + w] = (!(s.flags & F_NOROOM) && w == (rc >> 5)) ? (1u << (rc & 31)) : 0u;
    s.flags |= F_EXPL_BITMAP;
  }
  return s;
}

// reset() of env e (plantos_env.py:125-158) by one wave: map generation, then
// coop_apply_reset.
template <int MAXW, bool LT = false>
__device__ inline Scal coop_reset_env(const State& st, const Geo& g, const Rules& rl, int64_t e, uint32_t episode,
                                      bool keep, Row4<MAXW>& rw, int lane, uint64_t* scr,
                                      const Tables* tab = nullptr) {
  const Scal s = coop_gen_map<MAXW, LT>(g, rl, LT ? tab : (tab ? tab : st.tab), rw, rl.env_off + (uint32_t)e, episode, lane, scr);
  return coop_apply_reset<MAXW, LT>(st, g, e, s, keep, rw, lane, tab);
}

// Obs writers: an obs row of f32 values (HBM or an f32 LDS tile row), or of byte
// CODES (the byte-coded LDS obs tile of the sector kernel, pe_step_quad<..., BT>;
// the prefetched records of such a handle).  Every obs value is one of the tables'
// floats, so a byte names it: code c <= R+1 = dist[c] (dist[R+1] = 1.0; the
// one-hot's 0.0 / 1.0 are codes 0 / R+1), kCodeVis + v = vis[v], kCodePos + x =
// pos[x] (obs_code_table expands them at the tile store).
constexpr int kCodeVis = 80, kCodePos = 96;  // R + 1 < 80, 96 + G - 1 <= 255 (G <= 128)

template <typename T>
struct ObsW;
template <>
struct ObsW<float> {
  const float *tdist, *tpos, *tvis;
  int R;
  __device__ __forceinline__ float dist(int r) const { return tdist[r]; }
  __device__ __forceinline__ float one(bool b) const { return b ? 1.0f : 0.0f; }
  __device__ __forceinline__ float vis(int v) const { return tvis[v]; }
  __device__ __forceinline__ float pos(int x) const { return tpos[x]; }
};
template <>
struct ObsW<uint8_t> {
  const float *tdist, *tpos, *tvis;  // unused
  int R;
  __device__ __forceinline__ uint8_t dist(int r) const { return (uint8_t)r; }
  __device__ __forceinline__ uint8_t one(bool b) const { return b ? (uint8_t)(R + 1) : (uint8_t)0; }
  __device__ __forceinline__ uint8_t vis(int v) const { return (uint8_t)(kCodeVis + v); }
  __device__ __forceinline__ uint8_t pos(int x) const { return (uint8_t)(kCodePos + x); }
};

// The code table entry c from global memory in two halves (the expansion kernel and the
// runtime-(C,R) byte-tile kernel's first round): obs_code_loads issues
// every candidate load unconditionally (with the kernel's other loads: a load inside the
// branches of a per-code `if` chain was waited out at once -- three dependent round trips in
// the byte-coded kernels' first round, ~1.2 us, profiles/r5s/), obs_code_pick selects.
struct CodeLd {
  float d, v, p;
};
__device__ __forceinline__ CodeLd obs_code_loads(const Tables* tab, int R, int G, int c) {
  const int px = c - kCodePos;
  return CodeLd{tab->dist[c <= R ? c : 0], tab->vis[(c - kCodeVis) & 15], tab->pos[px >= 0 && px < G ? px : 0]};
}
// The code table entry c from the step kernels' LDS tables (load_tables_hot's dist[0..R],
// pos[0..G), vis[0..16), the kernel's dist[R+1] = 1.0 and one-hot zeros at kOneHotF):
// one LDS read, no global load -- filled by each thread after a barrier that completes
// round 1's LDS writes, read after the next one.
__device__ __forceinline__ void ctab_from_lds(const float* smem, float* ctab, int R, int G, int c, int onehot_zero) {
  const int f = c <= R + 1 ? c
                           : ((c >= kCodeVis && c < kCodeVis + 16)
                                  ? 328 + (c - kCodeVis)
                                  : ((c >= kCodePos && c < kCodePos + G) ? 72 + (c - kCodePos) : onehot_zero));
  ctab[c] = smem[f];
}

// The float of code c as one call: a per-code if-chain of global loads (each waited out at
// once: three dependent round trips where a kernel's first round issues it -- the C = 64 and
// far kernels, measured faster so, see pe_step_quad).
__device__ __forceinline__ float obs_code_value(const Tables* tab, int R, int G, int c) {
  if (c <= R) return tab->dist[c];
  if (c == R + 1) return 1.0f;
  if (c >= kCodeVis && c < kCodeVis + 16) return tab->vis[c - kCodeVis];
  if (c >= kCodePos && c < kCodePos + G) return tab->pos[c - kCodePos];
  return 0.0f;
}
__device__ __forceinline__ float obs_code_pick(const CodeLd& l, int R, int G, int c) {
  return c <= R ? l.d
                : (c == R + 1 ? 1.0f
                              : ((c >= kCodeVis && c < kCodeVis + 16) ? l.v
                                                                      : ((c >= kCodePos && c < kCodePos + G) ? l.p : 0.0f)));
}


// build_obs_fresh by one wave from the rows in the lanes' registers: lane i
// marches ray i (plantos_env.py:260-292), lanes 0..26 the position and the 5x5
// slice of a fresh episode (visit 1 at the rover, :294-313).  out: the env's obs
// row (floats: LDS tile row or HBM; codes: a byte-coded tile row or record);
// ldx/ldy: the handle's LIDAR offset tables.
template <int MAXW, typename T = float>
__device__ inline void coop_fresh_obs(const Geo& g, const Row4<MAXW>& rw, const Scal& s, T* out,
                                      const float* tdist, const float* tpos, const float* tvis,
                                      const signed char* ldx, const signed char* ldy, int lane) {
  const int R = g.R, C = g.C, G = g.G;
  const ObsW<T> w{tdist, tpos, tvis, R};
  // every lane takes part in every row fetch (a lane that left the loop could not
  // serve its row to the others): first hits are latched, not broken out of
  const int li = lane < C ? lane : 0;
  int dist = R, ent = EMPTY;
  bool hit = false;
  for (int r = 1; r <= R; ++r) {
    const int cx = s.x + ldx[li * R + r - 1];
    const int cy = s.y + ldy[li * R + r - 1];
    const bool inr = cx >= 0 && cx < G;
    const int src = inr ? cx : 0;
    const int bit = 2 * (cy + R);
    Row4<MAXW> fetched{0ull, 0ull, 0ull, 0ull};
#pragma unroll
    for (int k = 0; k < MAXW; ++k)
      if (MAXW == 1 || k < g.WPR) fetched.set(k, shfl64(rw.get(k), src));
    const uint64_t word = fetched.get(bit >> 6);
    const int code = inr ? (int)((word >> (bit & 63)) & 3u) : OBST;  // :271-284
    if (!hit && code != EMPTY) {
      hit = true;
      dist = r;
      ent = code;
    }
  }
  if (lane < C) {
    out[5 * lane] = w.dist(dist);
    out[5 * lane + 1] = w.one(ent == 0);
    out[5 * lane + 2] = w.one(ent == 1);
    out[5 * lane + 3] = w.one(ent == 2);
    out[5 * lane + 4] = w.one(ent == 3);
  }
  if (lane < 25) {
    const int lx = lane / 5, ly = lane % 5;
    const int gx = s.x + lx - 2, gy = s.y + ly - 2;
    const bool in = gx >= 0 && gx < G && gy >= 0 && gy < G;  // :307-311
    const bool rover = lane == 12 && !(s.flags & F_NOROOM);
    out[5 * C + 2 + lane] = w.vis(!in ? 10 : (rover ? 1 : 0));
  } else if (lane < 27) {
    out[5 * C + lane - 25] = w.pos(lane == 25 ? s.x : s.y);  // :294-296
  }
}

// ---- A block's single done env: its prefetched record staged into LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, so it can be issued by the commit wave before
// the done barrier, at the end of the commit, and land during the barrier and the
// other waves' last work instead of after it).  16-B units, in lane order:
//   [0] record scalars  [1, 1+NG) record grid rows  [1+NG, 1+NG+NO) record obs row
//   [1+NG+NO, 1+2NG+NO) the env's current grid rows (for the terminal info; staged when
//   all of it fits one instruction, and without the curriculum, whose commit stores rows)
__host__ __device__ constexpr int pf_grid_units(int G, int WPR) { return (G * WPR + 1) / 2; }
__host__ __device__ constexpr int pf_stage_units(int G, int WPR, int ostride, bool info) {
  return 1 + pf_grid_units(G, WPR) * (info ? 2 : 1) + ostride / 16;
}
__host__ __device__ constexpr bool pf_stage_info_fits(int G, int WPR, int ostride) {
  return pf_stage_units(G, WPR, ostride, true) <= 64;
}
__host__ __device__ constexpr int pf_stage_bytes(int G, int WPR, int ostride) {
  return ((pf_stage_units(G, WPR, ostride, pf_stage_info_fits(G, WPR, ostride)) + 63) / 64) * 1024;
}

// Issue the staging loads of env e's record into lds (wave-uniform; all 64 lanes).
__device__ __forceinline__ void pf_stage_issue(const Prefetch& pf, const State& st, const Geo& g, int64_t e,
                                               float* lds, int lane, bool info) {
  const int ng = pf_grid_units(g.G, g.WPR), no = (int)pf.ostride / 16;
  const int total = 1 + ng * (info ? 2 : 1) + no;
  // unit u's address, branch-free (selects on 64-bit integers)
  const uint64_t rs = reinterpret_cast<uint64_t>(pf.scal + e);
  const uint64_t rg = reinterpret_cast<uint64_t>(pf.grid + e * g.gstride) - 16u;
  const uint64_t ro = reinterpret_cast<uint64_t>(pf_obs_row(pf, e)) - 16u * (uint64_t)(1 + ng);
  const uint64_t cg = reinterpret_cast<uint64_t>(st.grid + e * g.gstride) - 16u * (uint64_t)(1 + ng + no);
  for (int c = 0; c < total; c += 64) {
    const int u = c + lane < total ? c + lane : total - 1;
    const uint64_t b = u == 0 ? rs : (u <= ng ? rg : (u <= ng + no ? ro : cg));
    const uint64_t ad = b + (u == 0 ? 0u : 16u * (uint64_t)u);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ad),
                                     (__attribute__((address_space(3))) void*)(lds + 4 * c), 16, 0, 0);
  }
}

// Lane r's grid row r from staged rows (words [G][WPR]).
template <int MAXW>
__device__ __forceinline__ Row4<MAXW> pf_stage_rows(const uint64_t* w, const Geo& g, int lane) {
  Row4<MAXW> r{0ull, 0ull, 0ull, 0ull};
  if (lane < g.G) {
#pragma unroll
    for (int k = 0; k < MAXW; ++k)
      if (MAXW == 1 || k < g.WPR) r.set(k, w[lane * g.WPR + k]);
  }
  return r;
}

// coop_take_prefetched from the staged record (after the wave's vmcnt(0)).  KD > 0: the obs
// row (at most 64 * KD values) copied as batched reads, then writes.
template <int MAXW, typename OT, int KD = 0>
__device__ __forceinline__ bool pf_stage_take(const float* lds, const Geo& g, int ostride, uint32_t episode,
                                              Row4<MAXW>& rw, Scal& s, OT* out, int lane) {
  const uint4 ps = *reinterpret_cast<const uint4*>(lds);
  const uint32_t key = (uint32_t)__builtin_amdgcn_readfirstlane((int)ps.w);
  if (key != episode + 1u) return false;
  s = unpack(make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)ps.x),
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)ps.y),
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)ps.z), key));
  const int ng = pf_grid_units(g.G, g.WPR);
  rw = pf_stage_rows<MAXW>(reinterpret_cast<const uint64_t*>(lds + 4), g, lane);
  const OT* o = reinterpret_cast<const OT*>(lds + 4 + 4 * ng);
  if constexpr (KD > 0) {
    OT v[KD];
#pragma unroll
    for (int j = 0; j < KD; ++j) v[j] = lane + 64 * j < g.D ? o[lane + 64 * j] : OT(0);
#pragma unroll
    for (int j = 0; j < KD; ++j)
      if (lane + 64 * j < g.D) out[lane + 64 * j] = v[j];
  } else {
    for (int k = lane; k < g.D; k += 64) out[k] = o[k];
  }
  (void)ostride;
  return true;
}

}  // namespace pe
