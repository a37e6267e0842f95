#!/usr/bin/env bash
# same-box A/B of two libraries over the runtime-(C, R) sector kernel's geometries:
#   bash tools/diag/rt_ab.sh OUT.jsonl LIB_A LIB_B
set -euo pipefail
OUT=$1; shift
LIBS=("$@")
: > "$OUT"
for rep in 1 2; do
  for lib in "${LIBS[@]}"; do
    for geo in "40 48 8" "32 24 9" "64 64 6"; do
      read -r G C R <<< "$geo"
      PLANTOS_HIP_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --desync-steps 0 --gather-steps 0 \
        --grid $G --rays $C --range $R --steps 2000 --warmup 100 |
        python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(json.dumps({'lib':'$(basename $lib)','geo':'$geo','us':round(d['ms_per_step']*1e3,3),'frac':round(d['roofline']['frac'],4)}))" >> "$OUT"
      tail -1 "$OUT"
    done
  done
done
