#!/usr/bin/env python3
"""The root's 8-block expansion (bench.py gather leg, expand_w8_us) from a rocprofv3
--kernel-trace run of bench.py: the pe_expand_codes_kernel dispatches of the 8-block
expansion (told apart by duration: more than 4x the short launches), their average duration, beside the
1-block expansion and the codes step of the same run.  Writes the rows it used as a CSV
and one JSON record.
  python tools/expand_w8_summary.py run_kernel_trace.csv OUT.csv OUT.json bench_line.json"""
import csv
import json
import sys


def main():
    trace, out_csv, out_json, bench = sys.argv[1:5]
    rows = list(csv.DictReader(open(trace)))
    ex = [r for r in rows if "pe_expand_codes_kernel" in r["Kernel_Name"]]
    # (the expansion kernel's grid does not grow with the blocks -- a grid-stride loop -- so the
    # 8-block launches are told apart by duration: ~8x the 1-block ones)
    d = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    lo = sorted(d(r) for r in ex)[len(ex) // 10]
    w8 = [r for r in ex if d(r) > 4 * lo]
    w1 = [r for r in ex if d(r) <= 4 * lo]
    gmax = gmin = int(ex[0]["Grid_Size_X"])
    step = [r for r in rows if "pe_step_quad<16, 6, true, 4, true" in r["Kernel_Name"]]
    dur = lambda rr: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rr) / max(1, len(rr)) / 1e3
    with open(out_csv, "w") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(w8)
    line = None
    for ln in open(bench):
        if ln.strip().startswith("{"):
            line = json.loads(ln)
    g = (line or {}).get("gather", {})
    rec = {"lib_sha": (line or {}).get("lib_sha"), "expand_w8_us_rocprof": dur(w8), "expand_w8_calls": len(w8),
           "expand_w8_grid": gmax, "expand_w1_us_rocprof": dur(w1), "expand_w1_grid": gmin,
           "codes_step_us_rocprof": dur(step), "codes_step_calls": len(step),
           "root_step_w8_us_rocprof": dur(step) + dur(w8),
           "bench_expand_w8_us_events": g.get("expand_w8_us"), "bench_root_step_w8_us": g.get("root_step_w8_us"),
           "expand_w8_bytes": g.get("expand_w8_bytes"), "source": trace,
           "note": "8 copies of one rank's gathered codes slot expanded by one launch (the root's per-step expansion "
                   "at 8 ranks, BASELINE config 5); root_step_w8 = its own codes step + that expansion"}
    json.dump(rec, open(out_json, "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if "us" in k}))


if __name__ == "__main__":
    main()
