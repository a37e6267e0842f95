#!/usr/bin/env python3
"""Summarize one `rocprofv3 --kernel-trace --stats` run of bench.py as the record
bench.py's roofline cites (rocprof_kernel_ns): the step kernel's average launch
duration, keyed by the benched library's hash and the bench config.

  python tools/kstats_summary.py OUT.json run_kernel_stats.csv bench_line.json [substring]

substring (default "pe_step"): the kernel is the stats row with the largest total
duration among the names holding it.
"""
import csv
import json
import os
import sys


def main():
    out, csv_path, bench_path = sys.argv[1:4]
    sub = sys.argv[4] if len(sys.argv) > 4 else "pe_step"
    line = None
    for ln in open(bench_path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        raise SystemExit(f"no bench line in {bench_path}")
    rows = [r for r in csv.DictReader(open(csv_path)) if sub in r["Name"]]
    if not rows:
        raise SystemExit(f"no kernel matching {sub!r} in {csv_path}")
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    rec = {"lib_sha": line["lib_sha"], "config": line["config"], "kernel_symbol": r["Name"],
           "avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]), "min_ns": float(r["MinNs"]),
           "max_ns": float(r["MaxNs"]), "source": os.path.relpath(csv_path),
           "desync": "desynchronized" in line.get("data", ""),
           "method": "rocprofv3 --kernel-trace --stats -f csv -- python3 bench.py ... (the bench line of the same run)"}
    json.dump(rec, open(out, "w"), indent=1)
    print(out, rec["avg_ns"], rec["kernel_symbol"][:80])


if __name__ == "__main__":
    main()
