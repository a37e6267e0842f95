// pe_far.hpp -- the sector step kernel for long LIDAR ranges: pe_step_far<C, R>
// (compile-time C, R with C % 4 == 0 and 15 <= R <= 32, e.g. SURVEY §8(d)'s 64x64 /
// 64 rays / R = 32 stress variant).  Included by plantos_batch.hip after pe_step_quad,
// whose auto-reset slow path and tile stores it shares.
//
// The sector kernel's LDS window ([2R+3 rows][64 envs] of one funnel-shifted word) does
// not reach R > 14, and a (2R+1)^2 window of 64 envs does not fit LDS.  Here every
// wave holds its sector's window in REGISTERS:
//
//   one workgroup = 4 waves = 64 envs, lane l of every wave works on env e0+l, and
//   wave w owns the rays of compass quadrant w ([wC/4, (w+1)C/4): dx and dy keep one
//   sign, so the cells its rays probe lie in the (R+1) x (R+1) quadrant of the window,
//   plantos_env.py:260-267 truncating toward zero);
//   round 1  packed scalars + action (every wave);
//   round 2  the grid word of the move's target and of the rover's cell, and the
//            target's visit word (every wave derives the transition itself, no
//            barrier: plantos_env.py:160-222);
//   round 3  the quadrant's grid rows around the POST-move position, 3 words per row
//            funnel-shifted per lane so that window column c is bit 2c of the row's
//            words, in batches of kFarRowBatch rows (the next batch's loads in flight
//            while a batch is marched); each probe of the quadrant's rays is then one
//            bit-field extract at a compile-time register and offset, packed 2 bits per
//            probe into the ray's 64-bit code word (first hit: one find-first-set, as
//            pe_quad.hpp quad_rays);
//   the non-commit waves build the 5x5 visit slice and position, the commit wave
//   (3) stores the state; the obs row is a byte-coded LDS tile row (pe_coop.hpp
//   ObsW<uint8_t>), expanded to floats at the tile store; a block with a done env
//   takes pe_step_quad's auto-reset path (quad_done_path, byte-tile form).
//
// No LDS window: the workgroup's LDS is the tables, the done path's scratch and the
// byte tile (~34 KB at 64x64 / 64 rays), so the 1024 workgroups of a 65536-env batch
// are resident at once (4 per CU); the cost that remains is the grid rows
// (~2 KB per env-step with the 2R pad) and the obs stream.
// (a fragment of plantos_batch.hip's anonymous namespace, like pe_pipe.hpp)
#pragma once

constexpr int kFarWaves = 4;
#ifndef PE_FAR_INFO_REG
#define PE_FAR_INFO_REG 0  // the terminal-info rows register-staged by the info wave (round 6 A/B: slower)
#endif
#ifndef PE_FAR_ROW_BATCH
#define PE_FAR_ROW_BATCH 33  // one batch: the compiler's schedule (9: 55.1 us, 12: 54.3, 17: 54.6, 33: 53.7 at
                             // 64x64/C64/R32, same box, profiles/r5f/, r5h/)
#endif
constexpr int kFarRowBatch = PE_FAR_ROW_BATCH;  // quadrant rows per load batch
constexpr int kFarRow32 = 2 * kCoopWPR;  // u32 words per padded grid row: the kernel takes G + 2R in (96, 128]

template <int C, int R>
constexpr int ray_dy_min(int i0, int i1) {
  int m = 0;
  for (int i = i0; i < i1; ++i)
    for (int r = 0; r < R; ++r) m = LidarTab<C, R>::dy[i][r] < m ? LidarTab<C, R>::dy[i][r] : m;
  return m;
}
template <int C, int R>
constexpr int ray_dy_max(int i0, int i1) {
  int m = 0;
  for (int i = i0; i < i1; ++i)
    for (int r = 0; r < R; ++r) m = LidarTab<C, R>::dy[i][r] > m ? LidarTab<C, R>::dy[i][r] : m;
  return m;
}

// The window of quadrant W: rows dx in [LO, HI], columns dy in [DLO, DHI] (both
// include 0: the rover's own cell, r = 1 of every non-axis ray).
template <int C, int R, int W>
struct FarQ {
  static constexpr int I0 = W * C / 4, I1 = (W + 1) * C / 4, NI = I1 - I0;
  static constexpr int LO = ray_dx_min<C, R>(I0, I1), HI = ray_dx_max<C, R>(I0, I1);
  static constexpr int DLO = ray_dy_min<C, R>(I0, I1), DHI = ray_dy_max<C, R>(I0, I1);
  static constexpr int NR = HI - LO + 1, NCOL = DHI - DLO + 1;
  static constexpr int NWD = (2 * NCOL + 31) / 32;        // aligned window words per row
  static constexpr int NRAW = (30 + 2 * NCOL + 31) / 32;  // raw words per row (any even shift <= 30)
  static constexpr int NB = (NR + kFarRowBatch - 1) / kFarRowBatch;
  static_assert(NWD <= 3 && NRAW <= 3, "window rows of at most 33 cells");
};

// LDS layout (floats): tables | the done path's scratch (quad_done_path: its staging
// words, then one cooperative-reset scratch per wave; the lane path's LIDAR offsets) |
// byte tile [64 x D] | code table [256]
// The region also ends in the commit wave's park words (far_park_off, 6 x 64 floats): the
// lane-per-env done path's LIDAR offsets (2CR bytes from its start, written by waves that
// pass the done barrier while the commit wave may still read its park words) must stay
// below them, so the region holds both side by side whatever the cooperative scratch.
__host__ __device__ constexpr int far_scr_floats(int G, int WPR, int C, int R) {
  const int coop = 2 * (162 + kFarWaves * coop_scratch_words(G, WPR));
  const int lane = (2 * C * R + 3) / 4 + 6 * kQuadEnvs;
  return ((coop > lane ? coop : lane) + 3) & ~3;
}
static_assert(far_scr_floats(33, kCoopWPR, 64, 32) - 6 * kQuadEnvs >= (2 * 64 * 32 + 3) / 4 &&
                  far_scr_floats(64, kCoopWPR, 64, 32) - 6 * kQuadEnvs >= (2 * 64 * 32 + 3) / 4,
              "far kernel: the park words overlap the lane path's LIDAR offsets");
__host__ __device__ constexpr int far_tile_off(int G, int WPR, int C, int R) {
  return kTabFloats + far_scr_floats(G, WPR, C, R);
}
__host__ __device__ constexpr int far_ctab_off(int G, int WPR, int C, int R) {
  return far_tile_off(G, WPR, C, R) + ((kQuadEnvs * (5 * C + 27) + 15) / 16) * 4;
}
// the commit wave's post-step scalars and return, parked in LDS for the done path
// ([6][64] words: packed scalars x4, return x2) -- not held in registers across the
// rays.  In the tail of the done path's scratch: read back before the done path runs.
__host__ __device__ constexpr int far_park_off(int G, int WPR, int C, int R) {
  return far_tile_off(G, WPR, C, R) - 6 * kQuadEnvs;
}
// the single-done record's LDS-DMA staging region (pe_coop.hpp pf_stage_issue; the
// byte-coded records' obs rows: 5C+27 codes rounded up to 16 B).  Not the env's current
// rows for the terminal info: 5 LDS-DMA instructions instead of 3 were slower
// (desynchronized 60.7 -> 61.4 us at 64x64/C64/R32, profiles/r5j/)
__host__ __device__ constexpr int far_stage_units(int G, int WPR, int C) {
  return pf_stage_units(G, WPR, ((5 * C + 27) + 15) & ~15, false);
}
__host__ __device__ constexpr int far_stage_off(int G, int WPR, int C, int R) { return far_ctab_off(G, WPR, C, R) + 256; }
// (round 6) after the record: the env's current grid rows for its terminal info, register-
// staged by the info wave in round 2 (pe_step_far info_reg), then one unit of the done env's
// post-step scalars and one of its wfix, parked by the commit wave for the info wave
__host__ __device__ constexpr int far_info_park_unit(int G, int WPR, int C) {
  return far_stage_units(G, WPR, C) + pf_grid_units(G, WPR);
}
__host__ __device__ constexpr int far_lds_floats(int G, int WPR, int C, int R) {
  // (whole 64-unit LDS-DMA instructions: every lane of the last one writes its unit)
  return far_stage_off(G, WPR, C, R) +
         4 * 64 * (((PE_FAR_INFO_REG ? far_info_park_unit(G, WPR, C) + 2 : far_stage_units(G, WPR, C)) + 63) / 64);
}

// Quadrant W's rays for this lane's env at the post-move position (xp, yp): first hit
// per ray (plantos_env.py:260-292), written as byte codes obs[5i .. 5i+4] of `row`.
// gb32: the env's grid block as u32 words (rw32 words per padded row).
template <int C, int R, int W>
__device__ __forceinline__ void far_sector(const uint32_t* gb32, int G, int xp, int yp, bool watered, uint8_t* row) {
  using Q = FarQ<C, R, W>;
  using T = LidarTab<C, R>;
  constexpr int NB = Q::NB, RB = kFarRowBatch, NRAW = Q::NRAW, NWD = Q::NWD, NI = Q::NI;
  // window column 0 = padded column yp + DLO + R: its bit b0 of the padded row
  const int b0 = 2 * (yp + Q::DLO + R);
  // window row j = grid row xp + LO + j: one base per lane, the row as an immediate offset.
  // Rows off the map are loaded UNCLAMPED (a neighbouring env's rows, or the arrays
  // around the grid in the handle's one allocation: pe_create carves scal / ep_ret
  // before and vis after it) and selected away; so is the raw word a row may read one
  // word past its end when the shift is small.
  const uint32_t* cb = gb32 + (xp + Q::LO) * kFarRow32 + (b0 >> 5);
  const uint32_t sh = (uint32_t)(b0 & 31);
  uint32_t lo[NI], hi[NI];  // probe r at bits 2(r-1) of lo (r <= 16) / 2(r-17) of hi
#pragma unroll
  for (int i = 0; i < NI; ++i) lo[i] = hi[i] = 0u;
  constexpr int J0 = -Q::LO, C0 = -Q::DLO;  // the rover's cell in the window
  uint32_t raw[RB][NRAW];
  auto load_batch = [&](int b) {
#pragma unroll
    for (int jj = 0; jj < RB; ++jj) {
      const int j = b * RB + jj;
      if (j < Q::NR) {
        const uint32_t* p = cb + j * kFarRow32;
#pragma unroll
        for (int k = 0; k < NRAW; ++k) raw[jj][k] = p[k];
      }
    }
  };
  load_batch(0);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint32_t w[RB][NWD];
#pragma unroll
    for (int jj = 0; jj < RB; ++jj) {
      const int j = b * RB + jj;
      if (j < Q::NR) {
        const int xr = xp + Q::LO + j;
        const bool in = (unsigned)xr < (unsigned)G;  // off-map rows read as obstacles (:271-274)
#pragma unroll
        for (int k = 0; k < NWD; ++k) {
          const uint32_t v = k + 1 < NRAW ? __builtin_amdgcn_alignbit(raw[jj][k + 1], raw[jj][k], sh) : raw[jj][k] >> sh;
          w[jj][k] = in ? v : 0x55555555u;
        }
        if (j == J0 && watered) w[jj][C0 >> 4] &= ~(1u << (2 * (C0 & 15)));  // the watered cell: 3 -> 2
      }
    }
    if (b + 1 < NB) load_batch(b + 1);  // in flight while this batch is marched
#pragma unroll
    for (int i = Q::I0; i < Q::I1; ++i) {
#pragma unroll
      for (int r = 1; r <= R; ++r) {
        const int j = T::dx[i][r - 1] - Q::LO;
        if (j / RB == b) {
          const int c = T::dy[i][r - 1] - Q::DLO;
          const uint32_t code = __builtin_amdgcn_ubfe(w[j - b * RB][c >> 4], 2 * (c & 15), 2);
          if (r <= 16)
            lo[i - Q::I0] |= code << (2 * (r - 1));
          else
            hi[i - Q::I0] |= code << (2 * (r - 17));
        }
      }
    }
  }
  // first hit per ray: find-first-set over the probes' nonzero codes (sentinel: none hit
  // -> range R, EMPTY); byte codes as quad_rays
#pragma unroll
  for (int i = Q::I0; i < Q::I1; ++i) {
    const uint32_t l = lo[i - Q::I0], h = hi[i - Q::I0];
    const uint32_t nl = (l | (l >> 1)) & 0x55555555u, nh = (h | (h >> 1)) & 0x55555555u;
    const int al = __ffs(nl), ah = __ffs(nh);  // 1 + bit index, 0: none
    const int f = al ? al - 1 : (ah ? 31 + ah : 2 * R);
    const uint32_t ent = al ? (l >> (al - 1)) & 3u : (ah ? (h >> (ah - 1)) & 3u : 0u);
    row[5 * i] = (uint8_t)((f >> 1) + 1);  // code r = dist[r] (R+1: 1.0, nothing hit)
    const uint32_t oh = (uint32_t)(R + 1) << (8 * ent);  // one-hot as codes {0, R+1}
    row[5 * i + 1] = (uint8_t)oh;
    row[5 * i + 2] = (uint8_t)(oh >> 8);
    row[5 * i + 3] = (uint8_t)(oh >> 16);
    row[5 * i + 4] = (uint8_t)(oh >> 24);
  }
}


// The step of one env of a far-kernel block before its rays, by the COMMIT wave: the
// state commit of plantos_env.py:160-222 (as pe_step_quad's quad_compute) from the
// round-2 words: gt / gc the grid words of the target and of the rover's cell, vt the
// target's visit word (its row vrow_t).  Returns done; wfix: its watering not stored.
__device__ __forceinline__ bool far_commit(const StepArgs& a, int64_t e, Scal& s, double& ret, const QuadMove& m,
                                           bool ok, uint32_t n, uint32_t nib, bool watered, bool wet_hyd, int xp,
                                           int yp, uint32_t gc, int cbit, uint32_t vt, int tvp, uint32_t* vrow_t,
                                           const uint32_t* gb32, int rw32, int R, uint32_t eo, uint32_t en,
                                           double cthr, bool& wfix) {
  const Geo& g = a.g;
  const Rules rl = a.rl;  // by value (see quad_compute)
  const State& st = a.st;
  uint32_t wo = eo, wn = en;
  if (ok) {
    if (s.flags & F_EXPL_BITMAP) {                                  // explored[old]=1, [new]=2 (:198-200)
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
  double h = 0.0;
  if (m.mv) {
    if (ok) {
      h = n == 0u ? rl.r_exploration : rl.r_revisit;               // :197, 204-207
    } else {
      s.flags |= F_COLLIDED;                                        // :209
      s.coll = s.coll < 65535 ? s.coll + 1 : 65535;                 // :210
      h = rl.r_invalid;                                             // :211
    }
  } else if (m.water) {
    h = watered ? rl.r_goal : (wet_hyd ? rl.r_mistake : rl.r_water_empty);  // :216-222 (fork's -10)
  }
  const int ox = s.x, oy = s.y;
  s.x = xp;                                                         // :199
  s.y = yp;
  double rew = rl.r_step;                                           // :164
  rew += h;
  bool term = s.expl >= s.total;                                    // :176, 244-246, 331
  const bool trunc = s.step >= rl.max_steps;                        // :177
  if (term && !(s.flags & F_BONUS)) {                               // :179-181
    rew += rl.r_complete;
    s.flags |= F_BONUS;
  }
  if (st.cur) term = curriculum_hit(st.cur, e, cthr, s.expl, s.total, rl.cur_term) || term;  // A2C_training.py:101-103
  const bool done = term || trunc;
  // an env about to be auto-reset gets new rows: its last move / watering is not stored
  // (the terminal info accounts for the watering), unless the curriculum carries its
  // visits over
  wfix = watered && done && a.autoreset && !st.cur;
  if (!(done && a.autoreset && !st.cur)) {
    if (ok) {
      // the byte of the target's visit nibble (padded column tvp), from its word
      const int pos = (4 * tvp) & 31, bsh = 8 * ((tvp >> 1) & 3);
      const uint32_t wnew = (vt & ~(0xFu << pos)) | (nib << pos);
      st_wt(reinterpret_cast<uint8_t*>(vrow_t) + (tvp >> 1), (uint8_t)(wnew >> bsh));
      visit_bump_exact(st, g, e, m.cell_n, n);
      if (s.flags & F_EXPL_BITMAP) {
        uint32_t* ep_o = st.expl + e * g.estride + (m.cell_o >> 5);
        uint32_t* ep_n = st.expl + e * g.estride + (m.cell_n >> 5);
        if (wo != eo) *ep_o = wo;
        if ((m.cell_o >> 5) != (m.cell_n >> 5) && wn != en) *ep_n = wn;
      }
    }
    if (watered) {  // the byte of the rover cell's code (padded column oy + R): 3 -> 2
      const int c = oy + R;
      const uint32_t wr = gc & ~(1u << (cbit & 31));
      st_wt(reinterpret_cast<uint8_t*>(const_cast<uint32_t*>(gb32) + ox * rw32) + (c >> 2),
            (uint8_t)(wr >> (8 * ((c >> 2) & 3))));
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
  if (!(done && a.autoreset && !st.cur)) {  // else the reset path stores the new episode's
    st_wt(st.ep_ret + e, ret);
    st_wt(st.scal + e, pack(s));
  }
  return done;
}

// The auto-reset slow path of a far-kernel block (pe_step_quad's, byte-tile form) out of
// line: a call, so that its register demand is its own (spilled on entry, cold) instead of
// the hot path's -- inlined, the values live into it spilled in the kernel's prologue.
// ka: the kernel's argument segment, taken in the kernel body (a noinline callee's own
// kernarg pointer is 0 on gfx950 / ROCm 7.2).  stage: the done env's prefetched record,
// staged into LDS by LDS-DMA (or nullptr).
template <int C, int R>
__device__ __attribute__((noinline)) uint4 far_done(const void* ka, int tile_off, int lane, int wv, int64_t e0,
                                                    bool done, uint4 sp, double ret, int ndone, bool wfix,
                                                    const float* ctab, const float* stage, bool stage_info) {
  constexpr int D = 5 * C + 27;
  return quad_done_path<kFarWaves, false, (D + 63) / 64, true, true>(ka, tile_off, C, R, lane, wv, kFarWaves - 1, e0,
                                                                     done, sp, ret, ndone, wfix, ctab, stage, stage_info);
}
#if PE_FAR_INFO_REG
// (the A/B form: the info wave writes the terminal info from the rows it staged)
template <int C, int R>
__device__ __attribute__((noinline)) uint4 far_done_iw(const void* ka, int tile_off, int lane, int wv, int64_t e0,
                                                       bool done, uint4 sp, double ret, int ndone, bool wfix,
                                                       const float* ctab, const float* stage, bool stage_info,
                                                       bool info_iw, int park_unit) {
  constexpr int D = 5 * C + 27;
  return quad_done_path<kFarWaves, false, (D + 63) / 64, true>(
      ka, tile_off, C, R, lane, wv, kFarWaves - 1, e0, done, sp, ret, ndone, wfix, ctab, stage, stage_info, -1,
      nullptr, nullptr, -1, false, info_iw, stage ? stage + 4 * park_unit : nullptr);
}
#endif

template <int C, int R>
__global__ __launch_bounds__(64 * kFarWaves, 4) void pe_step_far(StepArgs a) {
  constexpr int NW = kFarWaves, LS = kQuadEnvs, CW = NW - 1, D = 5 * C + 27;
  static_assert(C % 4 == 0 && C >= 4, "quadrant sectors");
  static_assert(R >= 2 && R <= 32, "64-bit packed probe codes");
  static_assert(R + 2 <= kOneHotF, "ray tables inside dist[]");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const Geo& g = a.g;
  const State& st = a.st;
  const int tile_off = far_tile_off(g.G, g.WPR, C, R);
  uint8_t* rows = reinterpret_cast<uint8_t*>(smem + tile_off);
  float* ctab = smem + far_ctab_off(g.G, g.WPR, C, R);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t e0 = (int64_t)blockIdx.x * LS;
  const int64_t e = e0 + lane;
  const bool live = e < a.n;
  if (a.stagger) {  // de-phase the resident workgroups of a CU (speed only), as pe_step_quad
    const int qg = (int)(blockIdx.x * PE_STAGGER_GROUPS / gridDim.x);
    for (int i = 0; i < qg * a.stagger; ++i) __builtin_amdgcn_s_sleep(8);
  }
  // ---- round 1 (every wave; unconditional loads at an index clamped into the batch)
  const int64_t ec = live ? e : (int64_t)a.n - 1;
  const uint4 sw = st.scal[ec];
  const int ash = a.act_bytes == 8 ? 1 : 0;
  const int32_t* ap = reinterpret_cast<const int32_t*>(a.actions);
  const int32_t alo = ap[ec << ash], ahi = ap[(ec << ash) + ash];
  double ret = st.ep_ret[wv == CW ? ec : 0];  // (the commit wave's; the others read one shared word)
  load_tables_hot(smem, st.tab, g.G, R);
  if (threadIdx.x < 16) smem[kOneHotF + threadIdx.x] = (threadIdx.x >> 2) == (threadIdx.x & 3) ? 1.0f : 0.0f;
  if (threadIdx.x == 16) smem[R + 1] = 1.0f;
  // (its code table after round 1's wait: the candidate loads issued with round 1 measured
  // 53.8 -> 55.4 us here -- three more live VGPRs in a kernel at its register cap -- and the
  // table filled from the LDS tables after the round-2 barrier 53.7 -> 54.4;
  // profiles/r5s/ab_code_table_*.txt)
  ctab[threadIdx.x] = obs_code_value(st.tab, R, g.G, (int)threadIdx.x);  // (256 threads)
  Scal s = unpack(sw);
  const int64_t action = ash ? (int64_t)(((uint64_t)(uint32_t)ahi << 32) | (uint32_t)alo) : (int64_t)alo;
  QuadMove m = quad_move<false>(s, action, g.G);
  quad_move_cells<false>(m, s, g.G);
  // ---- round 2: the target's grid and visit words, the rover cell's grid word; the
  // slice waves (0..2) also the candidate visit rows of their slice rows (rows x-3+lx ..
  // x-1+lx of slice row lx, 7 nibbles from padded column ybv: whatever the move, the
  // post-move slice row is among them)
  const uint32_t* gb32 = reinterpret_cast<const uint32_t*>(st.grid + ec * g.gstride);
  const int rw32 = kFarRow32;  // (g.WPR == kCoopWPR: pe_create)
  const int tx = m.inb ? m.nx : s.x, ty = m.nyc;  // (a move off the map is no move)
  const int tb = 2 * (ty + R), cbit = 2 * (s.y + R);
  const uint32_t gt = gb32[tx * rw32 + (tb >> 5)];
  const uint32_t gc = gb32[s.x * rw32 + (cbit >> 5)];
  uint32_t* vbase = vis_env(st, g, ec, s.episode);
  uint32_t* vrow_t = vbase + (int64_t)tx * g.NW;
  const int tvp = ty + 2;  // padded nibble column of the target
  const uint32_t vt = vrow_t[(4 * tvp) >> 5];
  // A block whose only env to truncate this step is known from its step count (:177;
  // ~6 % of the blocks of a desynchronized batch): the commit wave stages that env's
  // prefetched record into LDS by LDS-DMA now, so that its auto-reset makes no memory
  // round trip of its own (as pe_step_quad's byte-coded kernel; issued right after this
  // round's loads, see there)
  float* stage = smem + far_stage_off(g.G, g.WPR, C, R);
  const bool stage_ok = a.pf.scal && quad_coop(a, 1) && e0 + LS <= a.n;  // full block: every lane live
  constexpr bool stage_info = false;  // (see far_stage_units)
  int npred = 0;
  // (round 6) the predicted env's current grid rows for its terminal info, register-staged
  // by the info wave (two 16-B units per lane, written to LDS before the march): the info
  // wave then writes the terminal info beside the commit wave's reset, instead of the commit
  // wave loading the rows after the done barrier (a round trip on the one-done block's path)
  const int ng_s = pf_grid_units(g.G, g.WPR);
  // (measured slower here: 64x64/C64/R32 desync 60.0 -> 61.0 us, sync 52.8 -> 53.2, profiles/r6e/ --
  // the kernel is at its register cap; A/B: -DPE_FAR_INFO_REG=1)
  const bool info_reg = PE_FAR_INFO_REG && stage_ok && !st.cur && a.tinfo != nullptr && ng_s <= 128;
  uint4 iq0 = make_uint4(0u, 0u, 0u, 0u), iq1 = iq0;
  if (stage_ok) {
    const uint64_t pm = __ballot(s.step + 1 >= a.rl.max_steps);
    npred = __popcll(pm);
    if (wv == CW && npred == 1)
      pf_stage_issue(a.pf, st, g, e0 + (__ffsll((unsigned long long)pm) - 1), stage, lane, stage_info);
    if (info_reg && wv == kQuadInfoWave && npred == 1) {
      const uint4* src = reinterpret_cast<const uint4*>(st.grid + (e0 + (__ffsll((unsigned long long)pm) - 1)) * g.gstride);
      iq0 = src[lane < ng_s ? lane : ng_s - 1];
      iq1 = src[lane + 64 < ng_s ? lane + 64 : ng_s - 1];
    }
  }
  const int vw0 = (4 * m.ybv) >> 5, vo = (4 * m.ybv) & 31;
  uint32_t cv[2][3][2];  // [slice row t][candidate k][word]
  if (wv != CW) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int xr = s.x - 3 + (wv + 3 * t) + k;
        const int xc = xr < 0 ? 0 : (xr >= g.G ? g.G - 1 : xr);
        const uint32_t* p = vbase + (int64_t)xc * g.NW + vw0;
        cv[t][k][0] = p[0];
        cv[t][k][1] = p[1];
      }
  }
  double cthr = 0.0;
  uint32_t eo = 0u, en = 0u;
  if (live && wv == CW) {
    if (st.cur) cthr = st.cur[e].thr;  // CurriculumWrapper threshold
    if (m.inb && (s.flags & F_EXPL_BITMAP)) {
      eo = st.expl[e * g.estride + (m.cell_o >> 5)];
      en = st.expl[e * g.estride + (m.cell_n >> 5)];
    }
  }
  // ---- the transition (plantos_env.py:160-222), every wave
  s.step = s.step < 65535 ? s.step + 1 : 65535;                        // :162
  const bool ok = m.inb && ((gt >> (tb & 31)) & 3u) != OBST;            // :193-195 (plants walkable)
  const uint32_t n = ok ? (vt >> ((4 * tvp) & 31)) & 15u : 0u;         // :197
  const int ccode = (int)((gc >> (cbit & 31)) & 3u);
  const bool watered = m.water && ccode == THIRSTY;                    // fork plantos_env_new.py:237-240
  const bool wet_hyd = m.water && ccode == HYD;                        // fork :241-242 (root raises)
  const int xp = ok ? m.nx : s.x, yp = ok ? m.ny : s.y;
  const int dxv = xp - s.x;
  const uint32_t nib = n < 15u ? n + 1u : 15u;                         // :203
  // Every wave's round-2 words consumed before the commit wave stores: its visit byte
  // would otherwise reach a lagging wave's load of the same word (that wave then reads
  // n + 1 and shows n + 2 at the slice centre -- seen with 4 workgroups per CU, never at
  // one).  (The candidate slice rows and the rays' rows may see the new bytes: the slice
  // centre is rebuilt from nib, the watered cell's fix is idempotent.)
  asm volatile("s_barrier" ::"v"(vt), "v"(gt), "v"(gc) : "memory");
  if (info_reg && wv == kQuadInfoWave && npred == 1) {  // (into LDS before the march: no registers across it)
    uint4* d = reinterpret_cast<uint4*>(stage) + far_stage_units(g.G, g.WPR, C);
    if (lane < ng_s) d[lane] = iq0;
    if (lane + 64 < ng_s) d[lane + 64] = iq1;
  }
  uint8_t* row = rows + lane * D;
  bool done = false, wfix = false;
  uint32_t* park = reinterpret_cast<uint32_t*>(smem + far_park_off(g.G, g.WPR, C, R));
  if (live) {
    if (wv == CW) {
      done = far_commit(a, e, s, ret, m, ok, n, nib, watered, wet_hyd, xp, yp, gc, cbit, vt, tvp, vrow_t, gb32, rw32,
                        R, eo, en, cthr, wfix);
      // the post-step scalars and return for the done path, parked in LDS: in registers
      // they were live across the rays (and spilled there)
      const uint4 sp = pack(s);
      park[lane] = sp.x;
      park[64 + lane] = sp.y;
      park[128 + lane] = sp.z;
      park[192 + lane] = sp.w;
      park[256 + lane] = (uint32_t)__double2loint(ret);
      park[320 + lane] = (uint32_t)__double2hiint(ret);
    } else {
      // 5x5 slice rows lx = wv, wv + 3 (plantos_env.py:298-313) and the position (:294-296)
      const int vs = vo + 4 * (yp - m.ybv);  // bit of padded nibble column yp in the candidate words
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int lx = wv + 3 * t;
        if (lx < 5) {
          const int xr = xp - 2 + lx;
          const uint32_t w0 = dxv < 0 ? cv[t][0][0] : (dxv > 0 ? cv[t][2][0] : cv[t][1][0]);
          const uint32_t w1 = dxv < 0 ? cv[t][0][1] : (dxv > 0 ? cv[t][2][1] : cv[t][1][1]);
          uint32_t v = (uint32_t)((((uint64_t)w1 << 32) | w0) >> vs) & 0xFFFFFu;
          if ((unsigned)xr >= (unsigned)g.G) v = 0xAAAAAu;  // off-map rows: visit 10 (reads 1.0, :307-311)
          if (lx == 2 && ok) v = (v & ~0xF00u) | (nib << 8);  // the move's own visit (:203)
#pragma unroll
          for (int ly = 0; ly < 5; ++ly) row[5 * C + 2 + 5 * lx + ly] = (uint8_t)(kCodeVis + ((v >> (4 * ly)) & 15u));
        }
      }
      if (wv == 2) {
        row[5 * C] = (uint8_t)(kCodePos + xp);
        row[5 * C + 1] = (uint8_t)(kCodePos + yp);
      }
    }
    // ---- round 3 + the rays of this wave's quadrant
#if defined(PE_FAR_PROBE) && PE_FAR_PROBE == 1  // timing probe (wrong obs): no rays
    if (false)
#endif
    switch (wv) {
      case 0: far_sector<C, R, 0>(gb32, g.G, xp, yp, watered, row); break;
      case 1: far_sector<C, R, 1>(gb32, g.G, xp, yp, watered, row); break;
      case 2: far_sector<C, R, 2>(gb32, g.G, xp, yp, watered, row); break;
      default: far_sector<C, R, 3>(gb32, g.G, xp, yp, watered, row); break;
    }
  }
  // ---- DummyVecEnv auto-reset (rare): the commit wave's done mask in dist[70..71]
  const int park_unit = far_info_park_unit(g.G, g.WPR, C);
  if (wv == CW) {
    const uint64_t dm = __ballot(done);
    if (lane == 0) reinterpret_cast<uint64_t*>(smem)[35] = dm;
    if (info_reg && npred == 1 && __popcll(dm) == 1 && done) {  // the one done env's scalars for the info wave
      float* pk = stage + 4 * park_unit;  // (from the commit wave's park words: no registers across the march)
      pk[0] = __int_as_float((int)park[lane]);
      pk[1] = __int_as_float((int)park[64 + lane]);
      pk[2] = __int_as_float((int)park[128 + lane]);
      pk[3] = __int_as_float((int)park[192 + lane]);
      pk[4] = __int_as_float((int)wfix);
    }
  }
  // the block barrier without a memory fence (see pe_step_quad)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const uint64_t dmask = reinterpret_cast<const uint64_t*>(smem)[35];
  const uint64_t dmu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dmask) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(dmask >> 32)) << 32);
  const bool any_done = dmu != 0ull;
  const int ndone = __popcll(dmu);
  const int64_t valid = a.n - e0 < LS ? a.n - e0 : LS;
  uint4 sp = make_uint4(0u, 0u, 0u, 0u);
  if (__builtin_expect(any_done, 0)) {
    double rv = 0.0;
    if (wv == CW) {  // (the other waves' values are not used by the done path)
      sp = make_uint4(park[lane], park[64 + lane], park[128 + lane], park[192 + lane]);
      rv = __hiloint2double((int)park[320 + lane], (int)park[256 + lane]);
    }
    const bool staged = stage_ok && npred == 1 && ndone == 1;  // then the done env is the predicted one
#if PE_FAR_INFO_REG
    sp = far_done_iw<C, R>(kernargs(), tile_off, lane, wv, e0, done, sp, rv, ndone, wfix, ctab, staged ? stage : nullptr,
                           staged && stage_info, staged && info_reg, park_unit);
#else
    sp = far_done<C, R>(kernargs(), tile_off, lane, wv, e0, done, sp, rv, ndone, wfix, ctab, staged ? stage : nullptr,
                        staged && stage_info);
#endif
  }
  if (wv == CW) __builtin_amdgcn_s_waitcnt(0x0F70);  // tracked vmcnt(0): no wait inside the store loop
#if defined(PE_FAR_PROBE) && PE_FAR_PROBE == 2  // timing probe (no obs): no tile store
  if (false)
#endif
  if (a.obs_codes)
    store_tile_bytes(rows, a.obs_codes + e0 * D, (int)valid, D, (int)threadIdx.x, (int)blockDim.x);
  else
    store_tile_codes(rows, ctab, a.obs + e0 * D, (int)valid, D, (int)threadIdx.x, (int)blockDim.x);
  if (any_done && a.autoreset && !quad_coop(a, ndone)) {
    // the tile store wrote the terminal codes of the done rows: drain it, then overwrite
    // them with the fresh obs built from the env's rows in HBM (quad_done_obs)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    quad_done_obs<NW, true>(kernargs(), tile_off, lane, e, done, sp);
  }
}
