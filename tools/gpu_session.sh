#!/usr/bin/env bash
# A GPU-box session of named steps, each under its own time limit; the chain stops
# at the first failure (set -e).  Libraries for A/B steps are built beforehand on
# the CPU (tools/ab_build.sh) and travel with the tree.
#   usage: bash tools/gpu_session.sh TAG step [step ...]
#   steps: tests | smoke | bench | benchd | bench64 | stats | statsd | stats64 |
#          pmcf | pmcw | pmcf64 | pmcw64 | stamps | stampsd | benchx:<name>:<args> | statsx:<name>:<args> |
#          pmcx:<name>:<FETCH_SIZE|WRITE_SIZE>:<bench args with _ for spaces> |
#          ab:<name>:<rounds>:<lib,lib,...>:<bench args with _ for spaces>
set -euo pipefail
TAG=$1
shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
HEAD_ARGS="--steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 --no-cpu-baseline"
for w in "$@"; do
  case $w in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err ;;
    benchd)
      timeout -k 10 300 python bench.py --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
        > $OUT/benchd_$TAG.json 2> $OUT/benchd_$TAG.err ;;
    bench64)
      timeout -k 10 300 python bench.py --grid 64 --rays 64 --range 6 --steps 3000 --warmup 100 --desync-steps 3000 \
        --cpu-seconds 5 > $OUT/bench64_$TAG.json 2> $OUT/bench64_$TAG.err ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_$TAG -o run -- \
        python3 bench.py $HEAD_ARGS > $OUT/stats_bench_$TAG.json 2> $OUT/stats_$TAG.err ;;
    statsd)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/statsd_$TAG -o run -- \
        python3 bench.py --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
        > $OUT/statsd_bench_$TAG.json 2> $OUT/statsd_$TAG.err ;;
    stats64)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats64_$TAG -o run -- \
        python3 bench.py --grid 64 --rays 64 --range 6 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
        > $OUT/stats64_bench_$TAG.json 2> $OUT/stats64_$TAG.err ;;
    pmcf|pmcw|pmcf64|pmcw64)
      ctr=FETCH_SIZE; [[ $w == pmcw* ]] && ctr=WRITE_SIZE
      geo=""; [[ $w == *64 ]] && geo="--grid 64 --rays 64 --range 6"
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${w}_$TAG -o run -- \
        python3 bench.py $geo --steps 50 --warmup 10 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
        > $OUT/${w}_$TAG.json 2> $OUT/${w}_$TAG.err ;;
    stamps|stampsd)
      flag=""; [ $w = stampsd ] && flag="--desync"
      timeout -k 10 180 python tools/stamps.py run $flag > $OUT/${w}_$TAG.json 2> $OUT/${w}_$TAG.err ;;
    benchx:*)  # benchx:<name>:<bench args with _ for spaces>
      IFS=: read -r _ name args <<< "$w"
      timeout -k 10 300 python bench.py ${args//_/ } > $OUT/benchx_${name}_$TAG.json 2> $OUT/benchx_${name}_$TAG.err ;;
    statsx:*)  # statsx:<name>:<bench args with _ for spaces> under rocprofv3 --kernel-trace --stats
      IFS=: read -r _ name args <<< "$w"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/statsx_${name}_$TAG -o run -- \
        python3 bench.py ${args//_/ } > $OUT/statsx_${name}_$TAG.json 2> $OUT/statsx_${name}_$TAG.err ;;
    pmcx:*)  # one PMC pass (one counter) over a short bench run of the given geometry
      IFS=: read -r _ name ctr args <<< "$w"
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/pmcx_${name}_${ctr}_$TAG -o run -- \
        python3 bench.py ${args//_/ } --steps 50 --warmup 10 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
        > $OUT/pmcx_${name}_${ctr}_$TAG.json 2> $OUT/pmcx_${name}_${ctr}_$TAG.err ;;
    ab:*)
      IFS=: read -r _ name rounds libs args <<< "$w"
      libs=${libs//,/ }  # lib[+VAR=VAL]: ab_bench.sh's lib,VAR=VAL
      bash tools/ab_bench.sh "${name}_$TAG" "$rounds" ${libs//+/,} -- ${args//_/ } > /dev/null ;;
    *) echo "unknown step $w" >&2; exit 2 ;;
  esac
  echo "step $w done"
done
echo "all done"
