#!/usr/bin/env bash
# round-6 session i: the suite on lib_w12 (a done block's tile stored without the waves that wait
# for their done-path stores), A/B against lib_w11 (the tree's source) and lib_head
set -euo pipefail
T=r6i
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w12.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w12_$T.log 2>&1
echo "w12 tests done"; tail -n 1 gpurun_out/tests_w12_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
W11=build/ab/lib_w11.so
W12=build/ab/lib_w12.so
G40="--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:g64:2:$W11,$W12:$G64" \
  "ab:head:2:$W11,$W12:$A" \
  "ab:codes:2:$W11,$W12:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:far:2:$H,$W11,$W12:$GF" \
  "ab:g40c48:2:$W11,$W12:$G40" \
  "ab:g32:2:$W11,$W12:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
echo all-i done
