// pe_pipe.hpp -- the persistent, software-pipelined sector step kernel (pe_step_pipe).
// Included by plantos_batch.hip after pe_step_quad, whose StepArgs, LDS layout
// (quad_tile_off), compute phase (quad_compute) and auto-reset path (quad_done_path)
// it uses unchanged: per 64-env block it computes exactly what pe_step_quad<C, R,
// one-word, 4 waves> computes (plantos_env.py:160-315 + the DummyVecEnv auto-reset).
//
// pe_step_quad runs the 1024 workgroups of a 65536-env batch at once (4 per CU), each
// through two dependent load rounds, the compute phase and then its 27 KB obs tile --
// in lockstep, so the write stream (2/3 of the kernel's bytes) starts only after every
// block's prelude.  Here a resident grid of WPC workgroups per CU walks the blocks
// b = blockIdx.x, b + gridDim.x, ...: block b+1's round-1 loads are issued before
// block b's compute, its round-2 loads before block b's tile stores, so the stores of
// one block drain while the next one loads and computes.  The tile goes out as buffer
// stores the compiler counts (sc1 through the cache-policy operand, the store policy
// of store_tile), so the wait for the next block's round 2 is vmcnt(#tile stores
// issued after it), not vmcnt(0).
#pragma once

// Round-1 values of one block: the lane's env (scalars, action, return) and the
// loader env's (scalars, whole one-word grid block: gstride / 2 <= 10 16-B units,
// JG1 per loader thread).
template <int LT>
struct PipeR1 {
  static constexpr int JG1 = (10 + LT - 1) / LT;
  uint4 sw, lw, q[JG1];
  int32_t alo, ahi;
  double ret;
  uint32_t vp;  // the commit wave's: the deferred overflow write (pe_device.hpp vx_pending)
};

// The auto-reset path of a block with a done env, out of line: inlined into the loop
// its registers (map generation, the cooperative reset) would be the loop's.  `ka`:
// the kernel's argument segment, taken by the KERNEL (kernargs()) -- in a called
// function the kernarg-segment-pointer builtin reads as 0 on gfx950 / ROCm 7.2.
__device__ __attribute__((noinline)) uint4 pipe_done(const void* ka, int tile_off, int lane, int wv, int64_t e0,
                                                     bool done, uint4 sp, double ret, int ndone, bool wfix) {
  return quad_done_path<4, true, 2, false>(ka, tile_off, 16, 6, lane, wv, 3, e0, done, sp, ret, ndone, wfix);
}

// The kernel argument re-read per iteration through an opaque copy of the kernarg
// pointer (address space 4: scalar loads): otherwise the loop keeps every field it
// uses in SGPRs across iterations and spills them.
typedef __attribute__((address_space(4))) const StepArgs KArgs;
__device__ __forceinline__ const StepArgs& pipe_args() {
  KArgs* kp = (KArgs*)(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(kp));
  return *(const StepArgs*)kp;
}

// round 1 of block bb (every load unconditional, indices clamped into the batch, as
// in pe_step_quad): the lane's env and the loader env (le, part sub of LT)
template <int LT>
__device__ __forceinline__ void pipe_r1(const StepArgs& a, int64_t bb, int lane, int le, int sub, bool cw,
                                        PipeR1<LT>& r) {
  const State& st = a.st;
  const int ash = a.act_bytes == 8 ? 1 : 0;  // 8-byte actions: two words, low first
  const int32_t* ap = reinterpret_cast<const int32_t*>(a.actions);
  const int nq = (int)(a.g.gstride >> 1);
  const int64_t e = bb * kQuadEnvs + lane, el = bb * kQuadEnvs + le;
  const int64_t ec = e < a.n ? e : (int64_t)a.n - 1, elc = el < a.n ? el : (int64_t)a.n - 1;
  r.sw = st.scal[ec];
  r.alo = ap[ec << ash];
  r.ahi = ap[(ec << ash) + ash];
  r.ret = st.ep_ret[cw ? ec : 0];  // (the commit wave's; the others read one shared word)
  r.vp = st.vpend[cw ? ec : 0];
  r.lw = st.scal[elc];
  const uint4* lgq = reinterpret_cast<const uint4*>(st.grid + elc * a.g.gstride);
#pragma unroll
  for (int j = 0; j < PipeR1<LT>::JG1; ++j) {
    const int q = sub + LT * j;
    r.q[j] = lgq[q < nq ? q : nq - 1];
  }
}

// round 2 of block bb: the loader env's 7 visit rows (16 B each) around its rover
template <int LT, int JV>
__device__ __forceinline__ void pipe_r2(const StepArgs& a, int64_t bb, int le, int sub, const PipeR1<LT>& r,
                                        uint4 (&qv)[JV]) {
  const int64_t el = bb * kQuadEnvs + le;
  const int64_t elc = el < a.n ? el : (int64_t)a.n - 1;
  const int lx = (int)(r.lw.x & 0xFF);
  const uint32_t* lvb = vis_env(a.st, a.g, elc, r.lw.w);  // (the loader env's episode: its visit slot)
#pragma unroll
  for (int j = 0; j < JV; ++j) {
    const int xr = lx - 3 + sub + LT * j;
    const int xc = xr < 0 ? 0 : (xr >= a.g.G ? a.g.G - 1 : xr);
    qv[j] = *reinterpret_cast<const uint4*>(lvb + (int64_t)xc * 4);  // g.NW == 4
  }
}

// block bb's window into LDS [row][env]: the grid rows inside it from round 1's block
// (row pairs 2q, 2q+1), off-map rows as obstacles, the visit rows funnel-shifted to
// ybv (pe_step_quad's one-word round 2)
template <int R, int LT, int JV>
__device__ __forceinline__ void pipe_window(const StepArgs& a, int64_t bb, int le, int sub, const PipeR1<LT>& r,
                                            const uint4 (&qv)[JV], uint64_t* lrow, uint32_t* lvis) {
  constexpr int NR = 2 * R + 3, NV = 7, LS = kQuadEnvs;
  if (bb * LS + le >= a.n) return;
  const int G = a.g.G, nq = (int)(a.g.gstride >> 1);
  const int lx = (int)(r.lw.x & 0xFF), ly = (int)((r.lw.x >> 8) & 0xFF);
  const int base = lx - R - 1;  // grid row of LDS row 0
#pragma unroll
  for (int j = 0; j < PipeR1<LT>::JG1; ++j) {
    const int q = sub + LT * j, ka = 2 * q - base;
    if (q < nq) {
      const uint64_t lo = (uint64_t)r.q[j].x | ((uint64_t)r.q[j].y << 32);
      const uint64_t hi = (uint64_t)r.q[j].z | ((uint64_t)r.q[j].w << 32);
      if (ka >= 0 && ka < NR) lrow[ka * LS + le] = lo;
      if (ka + 1 >= 0 && ka + 1 < NR && 2 * q + 1 < G) lrow[(ka + 1) * LS + le] = hi;
    }
  }
#pragma unroll
  for (int j = 0; j < (NR + LT - 1) / LT; ++j) {
    const int k = sub + LT * j, xr = base + k;
    if (k < NR && (xr < 0 || xr >= G)) lrow[k * LS + le] = kEven64;  // off-map rows: obstacles
  }
  const int lybv = ly > 0 ? ly - 1 : 0;
  const int vw = (4 * lybv) >> 5, vo = (4 * lybv) & 31;
#pragma unroll
  for (int j = 0; j < JV; ++j) {
    const int k = sub + LT * j;
    if (k < NV) {
      const int xr = lx - 3 + k;
      uint32_t lo = 0xAAAAAAAAu, hi = 0xAAAAAAAAu;  // off-map row: visit 10 (reads 1.0)
      if (xr >= 0 && xr < G) {
        const uint4 q = qv[j];
        lo = vw == 0 ? q.x : (vw == 1 ? q.y : q.z);
        hi = vw == 0 ? q.y : (vw == 1 ? q.z : q.w);
      }
      lvis[k * LS + le] = vo ? ((lo >> vo) | (hi << (32 - vo))) : lo;
    }
  }
}

template <int C, int R, int WPC>
__global__ __launch_bounds__(256, WPC) void pe_step_pipe(StepArgs a0) {
  static_assert(C == 16 && R == 6, "pipe_done is the C16R6 one-word done path");
  constexpr int NW = 4, NR = 2 * R + 3, NV = 7, LS = kQuadEnvs, CW = NW - 1, LT = NW, D = 5 * C + 27;
  constexpr int JV = (NV + LT - 1) / LT;
  static_assert(2 * C * R <= (NR * 8 + NV * 4) * LS && 5 * 4 * LS + 8 <= (NR * 8 + NV * 4) * LS,
                "the done path's staging fits the window region");
  const int tile_off = quad_tile_off<R>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tdist = smem;
  float* tpos = smem + 72;
  float* tvis = smem + 328;
  uint64_t* lrow = reinterpret_cast<uint64_t*>(smem + kTabFloats);  // [NR][LS]
  uint32_t* lvis = reinterpret_cast<uint32_t*>(lrow + NR * LS);     // [NV][LS]
  float* rows = smem + tile_off;                                     // [LS][D]
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int le = threadIdx.x / LT, sub = threadIdx.x % LT;
  const int64_t nblk = ((int64_t)a0.n + LS - 1) / LS;

  // tables, once per workgroup (dist[R+1] = 1.0 and the one-hot rows: pe_quad.hpp quad_rays)
  load_tables_hot(smem, a0.st.tab, a0.g.G, R);
  if (threadIdx.x < 16) smem[kOneHotF + threadIdx.x] = (threadIdx.x >> 2) == (threadIdx.x & 3) ? 1.0f : 0.0f;
  if (threadIdx.x == 16) smem[R + 1] = 1.0f;

  // prologue: block blockIdx.x's two rounds, unpipelined
  int64_t b = blockIdx.x;
  PipeR1<LT> cur;
  pipe_r1<LT>(a0, b, lane, le, sub, wv == CW, cur);
  {
    uint4 qv[JV];
    pipe_r2<LT, JV>(a0, b, le, sub, cur, qv);
    pipe_window<R, LT, JV>(a0, b, le, sub, cur, qv, lrow, lvis);
  }
  // Waits the compiler tracks (__builtin_amdgcn_s_waitcnt, not asm) at the points where
  // every load before them is due anyway: its model of what is in flight then stays
  // exact across iterations -- otherwise a register loaded one iteration earlier gets
  // a conservative vmcnt at its first use that also waits for the next block's loads
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
  for (;;) {
    const StepArgs& a = pipe_args();
    const int64_t e0 = b * LS, e = e0 + lane;
    const bool live = e < a.n;
    const int64_t bn = b + gridDim.x;
    const bool more = bn < nblk;  // (uniform)
    // block b's window in LDS; the previous tile read out by its stores.  A barrier
    // without a memory fence: __syncthreads() would wait (vmcnt(0)) for the previous
    // block's tile stores and this block's round-2 loads -- the overlap itself
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- block bn's round 1, in flight through block b's compute
    PipeR1<LT> nxt;
    if (more) pipe_r1<LT>(a, bn, lane, le, sub, wv == CW, nxt);
    // ---- block b's compute phase (pe_step_quad's, unchanged)
    const int ash = a.act_bytes == 8 ? 1 : 0;
    Scal s = unpack(cur.sw);
    const int64_t action = ash ? (int64_t)(((uint64_t)(uint32_t)cur.ahi << 32) | (uint32_t)cur.alo) : (int64_t)cur.alo;
    QuadMove m = quad_move<true>(s, action, a.g.G);
    quad_move_cells<true>(m, s, a.g.G);
    double ret = cur.ret;
    if (wv == CW) __builtin_amdgcn_s_setprio(2);  // the commit wave is the laggard (pe_step_quad)
    bool done = false, wfix = false;
    quad_compute<C, R, true, NW, false, false, true, true>(a, lrow, lvis, rows, tdist, tpos, tvis, lane, wv, e, live, C, R,
                                                     m, 0u, 0u, 0.0, cur.vp, s, ret, done, wfix);
    if (wv == CW) {
      const uint64_t dm = __ballot(done);
      if (lane == 0) reinterpret_cast<uint64_t*>(smem)[35] = dm;
      __builtin_amdgcn_s_setprio(0);
    }
    // the done barrier, without a memory fence (see pe_step_quad)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const uint64_t dmask = reinterpret_cast<const uint64_t*>(smem)[35];
    const uint64_t dmu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dmask) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(dmask >> 32)) << 32);
    const bool any_done = dmu != 0ull;
    const int ndone = __popcll(dmu);
    if (__builtin_expect(any_done, 0))
      s = unpack(pipe_done(kernargs(), tile_off, lane, wv, e0, done, pack(s), ret, ndone, wfix));
    // ---- block bn's round 2 (its addresses need round 1), then block b's tile stores
    __builtin_amdgcn_s_waitcnt(kVmcnt0);  // block bn's round 1 landed (issued before the compute phase)
    uint4 qv[JV];
    if (more) pipe_r2<LT, JV>(a, bn, le, sub, nxt, qv);
    const int64_t valid = a.n - e0 < LS ? a.n - e0 : LS;
    if (wv != CW) {  // (the commit wave's state stores are in flight: see pe_step_quad)
      float* dst = a.obs + e0 * D;
      if (valid == LS && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        store_tile_buf<D, 64 * (NW - 1)>(rows, dst, (int)threadIdx.x);
        // round 2 landed: all but this wave's tile stores (issued after it) done
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(tile_buf_stores<D, 64 * (NW - 1)>()));
      } else {
        store_tile(rows, dst, (int)valid, D, D, (int)threadIdx.x, 64 * (NW - 1));
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
      }
    } else {
      __builtin_amdgcn_s_waitcnt(kVmcnt0);
    }
    if (any_done && a.autoreset && !quad_coop(a, ndone) && reset_scratch_bytes(a.g.G, a.g.WPR, a.rl.P) <= 4 * a.g.D) {
      // the lane-per-env reset's fresh obs over the stale tile rows (see pe_step_quad)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      quad_done_obs<NW, false>(kernargs(), tile_off, lane, e, done, pack(s));
      __syncthreads();  // its reads of the window region (LIDAR offsets) before block bn's rows
    }
    if (!more) break;
    pipe_window<R, LT, JV>(a, bn, le, sub, nxt, qv, lrow, lvis);
    cur = nxt;
    b = bn;
  }
}
