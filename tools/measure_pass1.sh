#!/usr/bin/env bash
# The measurement pass's first half (tools/measure_pass.sh, split in two gpurun calls):
# the GPU suite, smoke and the bench lines of every geometry.   usage: bash tools/measure_pass1.sh TAG
set -euo pipefail
T=$1
bash tools/gpu_session.sh $T tests
tail -n 1 gpurun_out/tests_$T.log
bash tools/gpu_session.sh $T smoke bench benchx:drv:--steps_20_--warmup_5 bench64 \
  benchx:n4096:--envs_4096_--steps_20000_--warmup_1000_--desync-steps_20000_--cpu-seconds_5 \
  benchx:g25:--grid_25_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g21:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g15:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g32:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_4000_--warmup_200_--desync-steps_4000_--cpu-seconds_5 \
  benchx:g64r32:--grid_64_--rays_64_--range_32_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5 \
  benchx:g40c48:--grid_40_--rays_48_--range_8_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5
echo pass1 done
