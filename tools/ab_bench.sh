#!/usr/bin/env bash
# Same-box A/B of step-kernel variants: alternate bench runs over the given
# libraries (paths; "tree" = the in-tree build), ROUNDS times, one JSON per line
# with the kernel time.   usage: bash tools/ab_bench.sh TAG ROUNDS lib1 lib2 ... [-- bench args]
set -euo pipefail
TAG=$1; ROUNDS=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
ARGS=${*:---steps 2000 --warmup 200}
OUT=gpurun_out/ab_$TAG.jsonl
mkdir -p gpurun_out; : > $OUT
for r in $(seq 1 $ROUNDS); do
  for L in "${LIBS[@]}"; do
    IFS=, read -r LP ENVS <<< "$L"   # "path[,VAR=VAL ...]" (space-separated env assignments)
    if [ "$LP" = tree ]; then unset PLANTOS_HIP_LIB; else export PLANTOS_HIP_LIB=$LP; fi
    env ${ENVS:-} timeout -k 10 120 python bench.py --no-cpu-baseline $ARGS > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_one.json')); rf=d['roofline']; g=d.get('gather', {}); print(json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), 'kernel_us': rf['kernel_us_window'], 'events_us': rf['kernel_us_events'], 'wall_us': d['ms_per_step']*1e3, 'desync_us': d.get('desync', {}).get('us_per_step'), 'gather_us': g.get('us_per_step'), 'gather_step_us': g.get('step_us'), 'expand_us': g.get('expand_us'), 'value': d['value'], 'kernel': d['config']['kernel']}))" "$L" "$r" >> $OUT
  done
done
unset PLANTOS_HIP_LIB
cat $OUT
