#!/usr/bin/env bash
# The measurement pass's profiling half (tools/measure_pass.sh, split in two gpurun calls):
# rocprof kernel stats of every geometry and the FETCH / WRITE PMC passes.
#   usage: bash tools/measure_pass2.sh TAG
set -euo pipefail
T=$1
bash tools/gpu_session.sh $T stats statsd stats64 \
  statsx:n4096:--envs_4096_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g25:--grid_25_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g64r32:--grid_64_--rays_64_--range_32_--steps_1000_--warmup_50_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g40c48:--grid_40_--rays_48_--range_8_--steps_1000_--warmup_50_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g32:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:gather:--steps_20_--warmup_5_--desync-steps_0_--no-cpu-baseline \
  pmcf pmcw pmcf64 pmcw64 pmcx:g25:FETCH_SIZE:--grid_25 pmcx:g25:WRITE_SIZE:--grid_25 \
  pmcx:n4096:FETCH_SIZE:--envs_4096 pmcx:n4096:WRITE_SIZE:--envs_4096 \
  pmcx:g64r32:FETCH_SIZE:--grid_64_--rays_64_--range_32 pmcx:g64r32:WRITE_SIZE:--grid_64_--rays_64_--range_32 \
  pmcx:g40c48:FETCH_SIZE:--grid_40_--rays_48_--range_8 pmcx:g40c48:WRITE_SIZE:--grid_40_--rays_48_--range_8 \
  pmcx:g32:FETCH_SIZE:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30 \
  pmcx:g32:WRITE_SIZE:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30
echo pass2 done
