#!/usr/bin/env bash
# round-6 session q: the one-wait done path and the LDS table reads restricted to the one-word
# f32 kernels (lt2) against the round-6 source (ow0); parity of lt2 first
set -euo pipefail
T=r6q
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_lt2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_$T.log 2>&1
tail -n 3 gpurun_out/tests_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
L=build/ab/lib_ow0.so,build/ab/lib_lt2.so
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:4:$L:$A" \
  "ab:n4096:3:$L:--envs_4096_$A" \
  "ab:g21:2:$L:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:g15:2:$L:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_$A" \
  "ab:codes:2:$L:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:far:2:$L:$GF"
echo all-q done
