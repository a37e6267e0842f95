#!/usr/bin/env bash
# start-delay stagger (PE_STAGGER, debug library) across the non-headline geometries:
#   bash tools/diag/stagger_geo.sh build/ab/lib_dbg.so
set -euo pipefail
LIB=$1
OUT=gpurun_out/stagger_geo.jsonl
: > "$OUT"
run() {  # tag stagger args...
  local tag=$1 st=$2; shift 2
  PE_STAGGER=$st PLANTOS_HIP_LIB=$LIB timeout -k 10 150 python bench.py --no-cpu-baseline --desync-steps 0 \
    --gather-steps 0 "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(json.dumps({'tag':'$tag','stagger':$st,'us':d['ms_per_step']*1e3,'frac':d['roofline']['frac']}))" >> "$OUT"
  tail -1 "$OUT"
}
for st in 0 2 4 8; do
  run g40c48 $st --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100
  run g32 $st --grid 32 --rays 24 --range 9 --steps 2000 --warmup 100
  run g25 $st --grid 25 --steps 4000 --warmup 200
done
