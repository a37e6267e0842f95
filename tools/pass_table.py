#!/usr/bin/env python3
"""The DESIGN / README results table of one measurement pass from its committed files
(profiles/<TAG>_bench*.json, kstats_<TAG>*.json, pmc*_<TAG>.json, <TAG>_expand_w8.json).
  python tools/pass_table.py TAG > table.md"""
import json
import sys

T = sys.argv[1]
P = "profiles/"


def bl(name):
    return json.loads([ln for ln in open(P + f"{T}_{name}.json") if ln.startswith("{")][-1])


def ks(name):
    try:
        return json.load(open(P + f"kstats_{T}{name}.json"))
    except FileNotFoundError:
        return None


def pmc(name):
    try:
        d = json.load(open(P + name.replace("TAG", T)))
        return d.get("traffic_cal", d["traffic_hi"]) / d["config"]["envs_per_gpu"]
    except FileNotFoundError:
        return None


def B(C, R):
    return 4 + 4 * (5 * C + 27) + 4 + 2 + 8 + 50 + 2 + C * R + 16


rows = [("headline 20×20 / C16 / R6", "bench", "", "_desync_head", "pmc_TAG.json"),
        ("BASELINE config 2: 4096 envs", "bench_n4096", "_n4096", "_desync_n4096", "pmc_n4096_TAG.json"),
        ("25×25 / C16 / R6 (the training scripts' grid)", "bench_g25", "_g25", "_desync_g25", "pmc_g25_TAG.json"),
        ("21×21 / C10 / R2 (constructor default)", "bench_g21", None, "_desync_g21", None),
        ("15×15 / C16 / R4", "bench_g15", None, "_desync_g15", None),
        ("64×64 / C64 / R6 (config 4)", "bench64", "_64", "_desync_g64", "pmc64_TAG.json"),
        ("32×32 / C24 / R9", "bench_g32", "_g32", "_desync_g32", "pmc_g32_TAG.json"),
        ("40×40 / C48 / R8", "bench_g40c48", "_g40c48", "_desync_g40c48", "pmc_g40c48_TAG.json"),
        ("64×64 / C64 / R32", "bench_g64r32", "_g64r32", "_desync_g64r32", "pmc_g64r32_TAG.json")]
print("| Workload (65536 envs unless noted) | kernel | env-steps/s | µs per step (bench window) | HIP events (frac) | "
      "rocprof avg (frac) | desync: bench window | desync: rocprof step + prefetch + compaction | measured HBM "
      "B/env-step (algorithmic) |")
print("|---|---|---|---|---|---|---|---|---|")
for lab, b, k, kd, pm in rows:
    d = bl(b)
    c = d["config"]
    C, R, n = c["rays"], c["lidar_range"], c["envs_per_gpu"]
    Bb = B(C, R)
    ev = d["roofline"]["kernel_us_events"]
    fe = Bb * n / (ev * 1e-6) / 8e12
    kk = ks(k) if k is not None else None
    kr = f"{kk['avg_ns'] / 1e3:.2f} ({Bb * n / (kk['avg_ns'] * 1e-9) / 8e12:.3f})" if kk else "—"
    dd = ks(kd)
    dsr = (f"{dd['avg_ns'] / 1e3:.2f} + {dd['prefetch_ns_per_step'] / 1e3:.2f} + {dd['compaction_ns_per_step'] / 1e3:.2f}"
           f" = **{dd['per_step_ns'] / 1e3:.2f}**") if dd else "—"
    ds = d.get("desync", {})
    t = pmc(pm) if pm else None
    print(f"| {lab} | `{c['kernel']}` | {d['value']:.3g} | {d['ms_per_step'] * 1e3:.2f} | {ev:.2f} ({fe:.3f}) | {kr} | "
          f"{ds.get('us_per_step', 0):.2f} | {dsr} | {f'{t:.0f}' if t else '—'} ({Bb}) |")
d = bl("bench_drv")
print(f"| the driver's window (`--steps 20 --warmup 5`), headline | same | {d['value']:.3g} | "
      f"{d['ms_per_step'] * 1e3:.2f} | {d['roofline']['kernel_us_events']:.2f} | — | — | — | — |")
g = bl("bench")["gather"]
w = json.load(open(P + f"{T}_expand_w8.json"))
print(f"| config 5's gather leg, one rank (codes step into a slot + expansion of the previous, one graph) | "
      f"`…,bytetile` + `pe_expand_codes_kernel` | — | {g['us_per_step']:.2f} per pair | step {g['step_us']:.2f}, "
      f"expansion {g['expand_us']:.2f} | {w['codes_step_us_rocprof']:.2f} + {w['expand_w1_us_rocprof']:.2f} | "
      f"(desynchronized) | — | — |")
rd = w["expand_w8_bytes"] if w.get("expand_w8_bytes") else {"read": 0, "written": 0}
tb = (rd["read"] + rd["written"]) / (w["expand_w8_us_rocprof"] * 1e-6) / 1e12
print(f"| config 5's root at 8 ranks: its codes step + the expansion of 8 gathered blocks (59 MB codes in, 227.5 MB f32 "
      f"out) | same | — | — | {g['step_us']:.2f} + {g['expand_w8_us']:.2f} = {g['root_step_w8_us']:.2f} | "
      f"{w['codes_step_us_rocprof']:.2f} + {w['expand_w8_us_rocprof']:.2f} = {w['root_step_w8_us_rocprof']:.2f} "
      f"(expansion at {tb:.2f} TB/s) | — | — | — |")
cb = bl("bench")["cpu_baseline"]
print()
print(f"cpu_baseline of the same pass: {cb['value']:.3g} env-steps/s ({cb['sample']}).")
