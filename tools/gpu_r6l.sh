#!/usr/bin/env bash
# round-6 session l: the suite on lib_w15 (the done path's in-place map generation out of line),
# A/B against lib_w11 (the tree's source) on every geometry
set -euo pipefail
T=r6l
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w15.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w15_$T.log 2>&1
echo "w15 tests done"; tail -n 1 gpurun_out/tests_w15_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
L=build/ab/lib_w11.so,build/ab/lib_w15.so
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G40="--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:2:$L:$A" \
  "ab:n4096:2:$L:--envs_4096_$A" \
  "ab:g25:2:$L:--grid_25_$A" \
  "ab:g21:2:$L:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:codes:2:$L:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g32:2:$L:$G32" \
  "ab:g40c48:2:$L:$G40" \
  "ab:g64:2:$L:$G64" \
  "ab:far:2:$L:$GF"
echo all-l done
