#!/usr/bin/env python3
"""Per-wave SQ instruction counts of one kernel from a rocprofv3 --pmc pass.

  python tools/sq_summary.py gpurun_out/sq_TAG/run_counter_collection.csv [--kernel pe_step_quad]
"""
import argparse
import collections
import csv
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--kernel", default="pe_step_quad")
a = ap.parse_args()
d = collections.defaultdict(list)
for r in csv.DictReader(open(a.csv)):
    if a.kernel in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.mean(v) for k, v in d.items()}
w = m.get("SQ_WAVES", 1.0)
out = {"kernel": a.kernel, "launches": len(d.get("SQ_WAVES", [])), "per_launch": m,
       "per_wave": {k: v / w for k, v in m.items() if k != "SQ_WAVES"}}
print(json.dumps(out, indent=1))
