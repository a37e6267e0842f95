#!/usr/bin/env python3
"""Phase timeline of the sector step kernel from in-kernel s_memrealtime stamps
(diagnostics; the stamped build is a separate library, its run time is not a
bench number -- read the SHARES and the timeline shape, not the length).

  python tools/stamps.py build                 # CPU: build/stamps/libplantos_hip_stamps.so
  python tools/stamps.py run [--grid 20 --rays 16 --range 6 --envs 65536] [--codes] [--desync] [--lib build/ab/lib_X.so]   # GPU

Stamps (lane 0 of each wave, 100 MHz = 10 ns ticks):
  0 entry  1 round-1 data in  2 round-2 loads landed + LDS written  3 after barrier
  4 rays/slice/commit done  5 after barrier_or  6 tile stores issued  7 stores drained
"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "build", "stamps", "libplantos_hip_stamps.so")
NAMES = ["entry", "round1", "round2+lds", "barrier", "compute", "barrier_or", "store_issue", "store_drain"]


def build(ablate=0):
    so = SO if not ablate else SO.replace(".so", f"_abl{ablate}.so")
    sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
    import build as B
    B.build(force=True, out=so, extra_flags=["-DPE_STAMPS", "-DPE_DEBUG_KNOBS"],
            obj_dir=os.path.join(os.path.dirname(so), f"obj{ablate}"))
    print(so)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def run(argv):
    abl = int(argv[argv.index("--ablate") + 1]) if "--ablate" in argv else 0
    os.environ["PLANTOS_HIP_LIB"] = SO if not abl else SO.replace(".so", f"_abl{abl}.so")
    if "--lib" in argv:  # a stamped A/B library (tools/ab_build.sh with EXTRA_FLAGS=-DPE_STAMPS)
        os.environ["PLANTOS_HIP_LIB"] = argv[argv.index("--lib") + 1]
    sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
    import numpy as np
    import torch
    from plantos_amd import PlantOSBatch
    from plantos_amd import _capi

    def arg(name, default):
        return int(argv[argv.index(name) + 1]) if name in argv else default

    G, C, n, Rg = arg("--grid", 20), arg("--rays", 16), arg("--envs", 65536), arg("--range", 6)
    P, O = (10, 12) if G <= 32 else (100, 120)
    codes = "--codes" in argv  # the byte-coded step (pe_step_codes)
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=O, lidar_range=Rg, lidar_channels=C,
                     device="cuda:0", obs_codes=codes)
    desync = "--desync" in argv
    if desync:  # every env at its own step count (bench.py --desync)
        st = b.get_state()
        sc = st["scalars"]
        g = torch.Generator(device="cpu").manual_seed(1)
        sc[:, _capi.PE_S_STEP] = torch.randint(0, 1000, (n,), generator=g, dtype=torch.int32).to(sc.device)
        b.set_state(scalars=sc)
    acts = torch.empty((64, n), dtype=torch.int32, device="cuda:0")
    for t in range(64):
        b.synth_actions(0, t, out=acts[t])
    for t in range(300):
        b.step(acts[t % 64])
    torch.cuda.synchronize()
    _, _, te, tr = b.step(acts[7])
    torch.cuda.synchronize()
    done = (te.bool() | tr.bool()).cpu().numpy()
    L = _capi.lib()
    L.pe_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    # envs per workgroup and waves per workgroup of the stamped kernel (the small-batch shapes:
    # E16 with 8 waves at <= 4096 envs, E16 / E32 with 4 waves up to 32768; --epb / --waves)
    EPB = arg("--epb", 64)
    NWQ = arg("--waves", int(os.environ.get("PE_QUAD_WAVES", "4")))
    nw = (n + EPB - 1) // EPB * NWQ
    buf = np.zeros(nw * 8, np.uint64)
    _capi.check(L.pe_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size), "stamps")
    st = buf.reshape(nw, 8).astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 10  # ns
    out = {"kernel": b.kernel_name, "envs": n, "waves": nw,
           "span_ns": int(rel[:, 7].max()),
           "abs_ns": {NAMES[k]: {"p0": int(rel[:, k].min()), "p50": int(np.median(rel[:, k])),
                                  "p100": int(rel[:, k].max())} for k in range(8)},
           "phase_ns": {f"{NAMES[k - 1]}->{NAMES[k]}": {"p50": int(np.median(rel[:, k] - rel[:, k - 1])),
                                                         "p90": int(np.percentile(rel[:, k] - rel[:, k - 1], 90))}
                        for k in range(1, 8)}}
    if desync:
        nb = (n + EPB - 1) // EPB
        dpb = np.add.reduceat(done.astype(np.int64), np.arange(0, n, EPB))
        L.pe_debug_dstamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        dbuf = np.zeros(nb * 8, np.uint64)
        _capi.check(L.pe_debug_dstamps(dbuf.ctypes.data_as(ctypes.c_void_p), dbuf.size), "dstamps")
        ds = (dbuf.reshape(nb, 8).astype(np.int64) - t0) * 10
        cw = rel.reshape(nb, NWQ, 8)[:, NWQ - 1, :]  # the commit wave of every block
        one = np.where(dpb == 1)[0]
        none = np.where(dpb == 0)[0]
        out["desync"] = {
            "blocks_done": {int(k): int((dpb == k).sum()) for k in np.unique(dpb)},
            "commit_wave_no_done_p50": {NAMES[k]: int(np.median(cw[none, k])) for k in range(8)},
            "commit_wave_one_done_p50": {NAMES[k]: int(np.median(cw[one, k])) for k in range(8)},
            "done_path_p50": {f"d{k}": int(np.median(ds[one, k])) for k in range(6)},
            "done_path_p90": {f"d{k}": int(np.percentile(ds[one, k], 90)) for k in range(6)},
            "block_end_no_done_p50": int(np.median(rel.reshape(nb, NWQ, 8)[none, :, 7].max(1))),
            "block_end_one_done_p50": int(np.median(rel.reshape(nb, NWQ, 8)[one, :, 7].max(1))),
            "block_end_one_done_p90": int(np.percentile(rel.reshape(nb, NWQ, 8)[one, :, 7].max(1), 90)),
            # the last block of each done count (the step ends with the slowest block)
            "block_end_max_by_done": {int(k): int(rel.reshape(nb, NWQ, 8)[dpb == k, :, 7].max())
                                      for k in np.unique(dpb)},
            "done_points": "single-done path (commit wave): d0 entry, d1 tobs copied, d2 info written, "
                           "d3 reset taken+applied, d4 queue flag, d5 scalars stored"}
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    else:
        run(sys.argv[2:])
