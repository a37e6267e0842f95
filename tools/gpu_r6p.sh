#!/usr/bin/env bash
# round-6 session p: the done path's table reads as LDS reads (no flat loads: lt1, with the
# one-wait path of the one-word f32 kernels) against ow0 (round-6 source) and ow1 (one-wait only)
set -euo pipefail
T=r6p
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_lt1.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_$T.log 2>&1
tail -n 3 gpurun_out/tests_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
L=build/ab/lib_ow0.so,build/ab/lib_ow1.so,build/ab/lib_lt1.so
L2=build/ab/lib_ow0.so,build/ab/lib_lt1.so
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G40="--grid_40_--rays_48_--range_8_--plants_20_--obstacles_40_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:3:$L:$A" \
  "ab:n4096:2:$L:--envs_4096_$A" \
  "ab:g25:2:$L2:--grid_25_$A" \
  "ab:g21:2:$L2:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:g15:2:$L2:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_$A" \
  "ab:codes:2:$L2:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g64:2:$L2:$G64" \
  "ab:g32:1:$L2:$G32" \
  "ab:g40:1:$L2:$G40"
echo all-p done
