#!/usr/bin/env bash
# rocprof kernel stats of the DESYNCHRONIZED steady state (bench.py --desync: every env at
# its own step count, ~n/1000 auto-resets per step) for every geometry of the measurement
# pass; the per-step cost is the step kernel + the prefetch launches + the queue compaction
# (tools/desync_summary.py).   usage: bash tools/measure_desync.sh TAG [geo ...]
set -euo pipefail
T=$1; shift
D="--desync_--warmup_1300_--desync-steps_0_--gather-steps_0_--no-cpu-baseline"
declare -A G=(
  [head]="--steps_20480_$D"
  [n4096]="--envs_4096_--steps_20480_$D"
  [g25]="--grid_25_--steps_20480_$D"
  [g21]="--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_--steps_20480_$D"
  [g15]="--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_--steps_20480_$D"
  [g64]="--grid_64_--rays_64_--range_6_--steps_4096_$D"
  [g64r32]="--grid_64_--rays_64_--range_32_--steps_2048_$D"
  [g32]="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_4096_$D"
  [g40c48]="--grid_40_--rays_48_--range_8_--steps_2048_$D"
)
GEOS=${*:-head n4096 g25 g21 g15 g64 g64r32 g32 g40c48}
STEPS=()
for g in $GEOS; do STEPS+=("statsx:d${g}:${G[$g]}"); done
bash tools/gpu_session.sh $T "${STEPS[@]}"
