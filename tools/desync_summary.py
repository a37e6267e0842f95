#!/usr/bin/env python3
"""Per-step cost of the desynchronized steady state from one `rocprofv3 --kernel-trace
--stats` run of `bench.py --desync` (tools/measure_desync.sh): the step kernel's average
launch plus the prefetch launches (pe_prefetch_kernel, every prefetch_every steps) and
their queue compaction (pe_pf_compact_kernel) spread over the step launches.  Writes a
kstats-style record (desync: true) keyed like tools/kstats_summary.py.

  python tools/desync_summary.py OUT.json run_kernel_stats.csv bench_line.json
"""
import csv
import json
import os
import sys


def main():
    out, csv_path, bench_path = sys.argv[1:4]
    line = None
    for ln in open(bench_path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    rows = list(csv.DictReader(open(csv_path)))
    steps = [r for r in rows if "pe_step" in r["Name"]]
    step = max(steps, key=lambda r: float(r["TotalDurationNs"]))
    n_step = int(step["Calls"])
    extra = {}
    for key, sub in (("prefetch", "pe_prefetch_kernel"), ("compaction", "pe_pf_compact_kernel")):
        rr = [r for r in rows if sub in r["Name"]]
        extra[key] = sum(float(r["TotalDurationNs"]) for r in rr) / n_step
    rec = {"lib_sha": line["lib_sha"], "config": line["config"], "kernel_symbol": step["Name"],
           "desync": True, "avg_ns": float(step["AverageNs"]), "calls": n_step,
           "prefetch_ns_per_step": extra["prefetch"], "compaction_ns_per_step": extra["compaction"],
           "per_step_ns": float(step["AverageNs"]) + extra["prefetch"] + extra["compaction"],
           "bench_us_per_step": line.get("ms_per_step", 0) * 1e3,
           "source": os.path.relpath(csv_path),
           "method": "rocprofv3 --kernel-trace --stats -- python3 bench.py --desync ... (tools/measure_desync.sh); "
                     "per_step = step kernel average + (prefetch + compaction total) / step launches"}
    json.dump(rec, open(out, "w"), indent=1)
    print(out, round(rec["avg_ns"]), "+", round(extra["prefetch"]), "+", round(extra["compaction"]), "=",
          round(rec["per_step_ns"]), "ns/step;", step["Name"][:60])


if __name__ == "__main__":
    main()
