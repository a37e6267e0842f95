#!/usr/bin/env python3
"""Summarize rocprofv3 output for the step kernel into profiles/.

  python tools/pmc_summary.py TAG [--prefix pmc] [--stats-dir gpurun_out/stats_TAG]

Reads the two PMC passes (FETCH_SIZE and WRITE_SIZE, collected in SEPARATE runs as
MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots prescribe) and the kernel-trace
stats, and writes profiles/<prefix>_<TAG>.json with per-launch HBM bytes of the
dominant kernel:

  FETCH_SIZE, WRITE_SIZE are in KiB (calibrated: pe_synth_kernel writes exactly
  n_envs * 4 B and reports n_envs * 4 / 1024).
  fetch_bytes_raw      = FETCH_SIZE * 1024
  fetch_bytes_x2       = 2 * FETCH_SIZE * 1024  (gfx950: FETCH_SIZE counts half of a
                         wide coalesced streaming read; upper bound for our mix of
                         16-B coalesced and 4/8-B gathered loads)
  traffic             = fetch_bytes_raw + write_bytes (raw counters);
  traffic_hi          = fetch_bytes_x2 + write_bytes: every read treated as streamed (upper bound);
  traffic_cal         = fetch_bytes_raw + streamed/2 + write_bytes: the calibrated figure bench.py
                        reports as roofline.traffic (for a profile whose lib_sha is the benched
                        library's).  profiles/r3r_fetch_calibration.json measured FETCH_SIZE on
                        known byte counts: streamed 16-B / 4-B reads report 1/2 of their bytes,
                        random 64-B segments and 16-B / 8-B gathers their full request bytes --
                        so only the kernel's streamed reads (--streamed-bytes per env: the sector
                        kernels' packed scalars 16 B + int32 action 4 B + return 8 B = 28 B) need
                        the x2, the gathered rows are counted as they are.
"""
import argparse
import collections
import csv
import json
import os
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        d[k].append(float(r["Counter_Value"]))
        meta[k] = {"grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                   "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"])}
    return d, meta


def stats_rows(stats_dir):
    p = os.path.join(stats_dir, "run_kernel_stats.csv")
    if not os.path.exists(p):
        return {}
    return {r["Name"]: r for r in csv.DictReader(open(p))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--prefix", default="pmc")
    ap.add_argument("--out-prefix", default=None)
    ap.add_argument("--kernel", default="pe_step")
    ap.add_argument("--stats-dir", default=None)
    ap.add_argument("--bench-json", default=None, help="bench line of the profiled run (config)")
    ap.add_argument("--fetch-dir", default=None, help="FETCH_SIZE pass dir under gpurun_out (tools/gpu_session.sh: pmcf_TAG)")
    ap.add_argument("--write-dir", default=None, help="WRITE_SIZE pass dir under gpurun_out (tools/gpu_session.sh: pmcw_TAG)")
    ap.add_argument("--streamed-bytes", type=float, default=28.0,
                    help="streamed (coalesced, 16-B / 4-B per lane) read bytes per env-step of the kernel")
    a = ap.parse_args()
    g = os.path.join(REPO, "gpurun_out")
    fd = a.fetch_dir or f"{a.prefix}_fetch_{a.tag}"
    wd = a.write_dir or f"{a.prefix}_write_{a.tag}"
    fetch, meta = per_kernel(os.path.join(g, fd, "run_counter_collection.csv"), "FETCH_SIZE")
    write, _ = per_kernel(os.path.join(g, wd, "run_counter_collection.csv"), "WRITE_SIZE")
    names = [k for k in fetch if a.kernel in k]
    if not names:
        raise SystemExit(f"no kernel matching {a.kernel}")
    # dominant = most launches
    k = max(names, key=lambda n: len(fetch[n]))
    f_kib = statistics.mean(fetch[k])
    w_kib = statistics.mean(write[k])
    out = {
        "kernel": k, "launches_fetch_pass": len(fetch[k]), "launches_write_pass": len(write[k]),
        "FETCH_SIZE_KiB_mean": f_kib, "WRITE_SIZE_KiB_mean": w_kib,
        "fetch_bytes_raw": f_kib * 1024, "fetch_bytes_x2": 2 * f_kib * 1024, "write_bytes": w_kib * 1024,
        "traffic": (f_kib + w_kib) * 1024, "traffic_hi": (2 * f_kib + w_kib) * 1024,
        "resources": meta[k],
        "write_calibration": {n: statistics.mean(write[n]) for n in write if "synth" in n},
        "method": "rocprofv3 --pmc FETCH_SIZE --kernel-trace, then --pmc WRITE_SIZE --kernel-trace (separate passes)",
    }
    if a.bench_json:
        try:
            line = [ln for ln in open(a.bench_json) if ln.startswith("{")][-1]
            b = json.loads(line)
            n = b["config"]["envs_per_gpu"]
            out["config"] = b["config"]
            out["lib_sha"] = b.get("lib_sha")  # bench.py cites this profile only for this exact library
            out["traffic_per_env_step"] = out["traffic"] / n
            out["traffic_hi_per_env_step"] = out["traffic_hi"] / n
            out["streamed_read_bytes_per_env_step"] = a.streamed_bytes
            out["traffic_cal"] = out["traffic"] + a.streamed_bytes * n / 2
            out["traffic_cal_per_env_step"] = out["traffic_cal"] / n
            out["calibration"] = "profiles/r3r_fetch_calibration.json"
        except (OSError, IndexError, KeyError, ValueError):
            pass
    sd = a.stats_dir
    if sd:
        rows = stats_rows(os.path.join(g, sd) if not os.path.isabs(sd) else sd)
        if k in rows:
            out["stats_avg_ns"] = float(rows[k]["AverageNs"])
            out["stats_calls"] = int(rows[k]["Calls"])
    dst = os.path.join(REPO, "profiles", f"{a.out_prefix or a.prefix}_{a.tag}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
