#!/usr/bin/env bash
# round-6 session g: the suite on the in-tree library (the candidate: lib w8's source), same-
# box A/B of lib_w8 (product flags = w8 + debug knobs) against lib_head on every geometry
set -euo pipefail
T=r6g
mkdir -p gpurun_out
bash tools/gpu_session.sh $T tests smoke
tail -n 1 gpurun_out/tests_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
W=build/ab/lib_w8.so
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G40="--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:2:$H,$W:$A" \
  "ab:n4096:2:$H,$W:--envs_4096_$A" \
  "ab:g25:2:$H,$W:--grid_25_$A" \
  "ab:g21:2:$H,$W:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:g15:2:$H,$W:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_$A" \
  "ab:codes:2:$H,$W:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g32:2:$H,$W:$G32" \
  "ab:g40c48:2:$H,$W:$G40" \
  "ab:g64:2:$H,$W:$G64" \
  "ab:far:2:$H,$W:$GF"
timeout -k 10 120 python tools/stamps.py run --lib build/ab/lib_stamps_rss.so --envs 4096 --epb 16 --waves 8 --desync \
  > gpurun_out/stamps_n4096d_rss_$T.json 2> gpurun_out/stamps_n4096d_rss_$T.err || true
echo all-g done
