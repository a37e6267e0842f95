#!/usr/bin/env bash
# Copy a measurement pass (tools/measure_pass1.sh TAG, then tools/measure_pass2.sh TAG) from gpurun_out/ into
# profiles/ under the names the docs cite, and write the PMC summaries (tools/pmc_summary.py).
#   usage: bash tools/summarize_pass.sh TAG
set -euo pipefail
T=$1
G=gpurun_out
P=profiles
cp $G/tests_$T.log $P/${T}_gpu_tests.log
cp $G/smoke_$T.log $P/${T}_smoke.log
cp $G/bench_$T.json $P/${T}_bench.json
cp $G/bench64_$T.json $P/${T}_bench64.json
for x in drv n4096 g25 g21 g15 g32 g64r32 g40c48; do cp $G/benchx_${x}_$T.json $P/${T}_bench_${x}.json; done
cp $G/stats_$T/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $G/statsd_$T/run_kernel_stats.csv $P/${T}_kernel_stats_desync.csv
cp $G/stats64_$T/run_kernel_stats.csv $P/${T}_kernel_stats_64.csv
for x in n4096 g25 g64r32 g40c48 g32 gather; do cp $G/statsx_${x}_$T/run_kernel_stats.csv $P/${T}_kernel_stats_${x}.csv; done
# the gather leg's kernel trace (the step into the slot, the expansion, the gaps between them)
python3 - $G/statsx_gather_$T/run_kernel_trace.csv $P/${T}_gather_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keep = [r for r in rows if "bytetile" in r.get("Kernel_Name", "") or "expand" in r.get("Kernel_Name", "")
        or "pe_step_quad<16, 6, true, 4, true" in r.get("Kernel_Name", "")][-400:]
if keep:
    w = csv.DictWriter(open(sys.argv[2], "w"), fieldnames=list(keep[0].keys()))
    w.writeheader()
    w.writerows(keep)
PY
# the step kernel's rocprof average per stats run, keyed by lib_sha + config (bench.py rocprof_kernel_ns)
python3 tools/kstats_summary.py $P/kstats_${T}.json $P/${T}_kernel_stats.csv $G/stats_bench_$T.json
python3 tools/kstats_summary.py $P/kstats_${T}_desync.json $P/${T}_kernel_stats_desync.csv $G/statsd_bench_$T.json
python3 tools/kstats_summary.py $P/kstats_${T}_64.json $P/${T}_kernel_stats_64.csv $G/stats64_bench_$T.json
for x in n4096 g25 g64r32 g40c48 g32; do
  python3 tools/kstats_summary.py $P/kstats_${T}_$x.json $P/${T}_kernel_stats_$x.csv $G/statsx_${x}_$T.json
done
python3 tools/pmc_summary.py $T --fetch-dir pmcf_$T --write-dir pmcw_$T --bench-json $G/pmcf_$T.json \
  --stats-dir stats_$T > /dev/null
python3 tools/pmc_summary.py $T --out-prefix pmc64 --fetch-dir pmcf64_$T --write-dir pmcw64_$T \
  --bench-json $G/pmcf64_$T.json --stats-dir stats64_$T > /dev/null
for x in g25 n4096; do
  python3 tools/pmc_summary.py $T --out-prefix pmc_$x --fetch-dir pmcx_${x}_FETCH_SIZE_$T \
    --write-dir pmcx_${x}_WRITE_SIZE_$T --bench-json $G/pmcx_${x}_FETCH_SIZE_$T.json --stats-dir statsx_${x}_$T > /dev/null
done
for x in g64r32 g40c48 g32; do
  python3 tools/pmc_summary.py $T --out-prefix pmc_$x --fetch-dir pmcx_${x}_FETCH_SIZE_$T \
    --write-dir pmcx_${x}_WRITE_SIZE_$T --bench-json $G/pmcx_${x}_FETCH_SIZE_$T.json --stats-dir statsx_${x}_$T > /dev/null
done
# the root's 8-block expansion of config 5 (bench.py gather leg expand_w8_us), from the gather trace
python3 tools/expand_w8_summary.py $G/statsx_gather_$T/run_kernel_trace.csv $P/${T}_expand_w8_trace.csv \
  $P/${T}_expand_w8.json $G/statsx_gather_$T.json
# the desynchronized steady state of every geometry (tools/measure_desync.sh): step + prefetch + compaction
for x in head n4096 g25 g21 g15 g64 g64r32 g32 g40c48; do
  d=$G/statsx_d${x}_$T
  [ -f $d/run_kernel_stats.csv ] || continue
  cp $d/run_kernel_stats.csv $P/${T}_kernel_stats_desync_$x.csv
  python3 tools/desync_summary.py $P/kstats_${T}_desync_$x.json $P/${T}_kernel_stats_desync_$x.csv $G/statsx_d${x}_$T.json
done
ls -la $P/*_$T.json $P/${T}_* | wc -l
