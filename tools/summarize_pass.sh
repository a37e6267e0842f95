#!/usr/bin/env bash
# Copy a measurement pass (tools/measure_pass.sh TAG) from gpurun_out/ into
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
for x in n4096 g25 g64r32 g40c48; do cp $G/statsx_${x}_$T/run_kernel_stats.csv $P/${T}_kernel_stats_${x}.csv; done
python3 tools/pmc_summary.py $T --fetch-dir pmcf_$T --write-dir pmcw_$T --bench-json $G/pmcf_$T.json \
  --stats-dir stats_$T > /dev/null
python3 tools/pmc_summary.py $T --out-prefix pmc64 --fetch-dir pmcf64_$T --write-dir pmcw64_$T \
  --bench-json $G/pmcf64_$T.json --stats-dir stats64_$T > /dev/null
for x in g25 n4096; do
  python3 tools/pmc_summary.py $T --out-prefix pmc_$x --fetch-dir pmcx_${x}_FETCH_SIZE_$T \
    --write-dir pmcx_${x}_WRITE_SIZE_$T --bench-json $G/pmcx_${x}_FETCH_SIZE_$T.json --stats-dir statsx_${x}_$T > /dev/null
done
# the wave kernel's window span and visit rows are streamed reads too
python3 tools/pmc_summary.py $T --out-prefix pmc_g64r32 --fetch-dir pmcx_g64r32_FETCH_SIZE_$T \
  --write-dir pmcx_g64r32_WRITE_SIZE_$T --bench-json $G/pmcx_g64r32_FETCH_SIZE_$T.json \
  --stats-dir statsx_g64r32_$T --streamed-bytes 1820 --kernel pe_step_wave > /dev/null
ls -la $P/*_$T.json $P/${T}_* | wc -l
