#!/usr/bin/env bash
# One GPU-box session: parity tests, bench lines, rocprofv3 kernel stats and the
# two PMC passes (FETCH_SIZE / WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# §HBM) for the headline step kernel.  Every GPU step has its own time limit and
# the chain stops at the first failure.
#   usage: bash tools/gpu_profile.sh [tag] [what...]   what in {tests,bench,bench64,stats,pmc,micro}
set -euo pipefail
TAG=${1:-r1}
shift || true
WHAT=${*:-tests bench bench64 stats pmc}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
python rl-env_amd/build.py > $OUT/build_$TAG.log 2>&1
make -s -C oracle >> $OUT/build_$TAG.log 2>&1
BENCH_ARGS="--steps 2000 --warmup 200 --no-cpu-baseline"
for w in $WHAT; do
  case $w in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err ;;
    benchd)
      timeout -k 10 300 python bench.py --desync --steps 20000 --warmup 200 --no-cpu-baseline > $OUT/benchd_$TAG.json 2> $OUT/benchd_$TAG.err ;;
    benchq)
      timeout -k 10 300 python bench.py --steps 4000 --warmup 200 --no-cpu-baseline > $OUT/benchq_$TAG.json 2> $OUT/benchq_$TAG.err ;;
    bench64)
      timeout -k 10 300 python bench.py --grid 64 --rays 64 --range 6 --steps 3000 --warmup 100 \
        --cpu-seconds 5 > $OUT/bench64_$TAG.json 2> $OUT/bench64_$TAG.err ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_$TAG -o run -- \
        python3 bench.py $BENCH_ARGS > $OUT/stats_bench_$TAG.json 2> $OUT/stats_$TAG.err ;;
    pmc)
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc_fetch_$TAG -o run -- \
        python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/pmc_fetch_$TAG.json 2> $OUT/pmc_fetch_$TAG.err
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_write_$TAG -o run -- \
        python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/pmc_write_$TAG.json 2> $OUT/pmc_write_$TAG.err ;;
    pmc64)
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc64_fetch_$TAG -o run -- \
        python3 bench.py --grid 64 --rays 64 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/pmc64_fetch_$TAG.json 2> $OUT/pmc64_fetch_$TAG.err
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc64_write_$TAG -o run -- \
        python3 bench.py --grid 64 --rays 64 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/pmc64_write_$TAG.json 2> $OUT/pmc64_write_$TAG.err ;;
    sq)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -f csv -d $OUT/sq_$TAG -o run -- \
        python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/sq_$TAG.json 2> $OUT/sq_$TAG.err ;;
    sq64)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -f csv -d $OUT/sq64_$TAG -o run -- \
        python3 bench.py --grid 64 --rays 64 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/sq64_$TAG.json 2> $OUT/sq64_$TAG.err ;;
    micro)
      timeout -k 10 300 python tools/micro_step.py > $OUT/micro_$TAG.json 2> $OUT/micro_$TAG.err ;;
    *) echo "unknown step $w" >&2; exit 2 ;;
  esac
  echo "step $w done"
done
echo "all done: $WHAT"
