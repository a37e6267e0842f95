#!/usr/bin/env bash
# round-6 session d: the suite on the in-tree library (current source), same-box A/B of
# lib_w4 (register-staged record for the multi-word / runtime f32 kernels, register-window
# runtime rays, info-wave staging in the LDS-DMA byte-tile kernels, no stagger for the C16
# codes kernel) against lib_head, the far kernel's stagger, the round-5 hazard repro
set -euo pipefail
T=r6d
mkdir -p gpurun_out
bash tools/gpu_session.sh $T tests
tail -n 1 gpurun_out/tests_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
W=build/ab/lib_w4.so
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G40="--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:g64:2:$H,$W:$G64" \
  "ab:g32:2:$H,$W:$G32" \
  "ab:g40c48:2:$H,$W:$G40" \
  "ab:codes:2:$H,$W:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g25:2:$H,$W:--grid_25_$A" \
  "ab:head:2:$H,$W:$A" \
  "ab:farstag:2:$H,$H+PE_STAGGER=0,$H+PE_STAGGER=8:$GF" \
  "ab:g64stag:2:$H+PE_STAGGER=2,$H+PE_STAGGER=8:$G64"
PLANTOS_HIP_LIB=build/ab/lib_gridc.so timeout -k 10 120 python tools/diag/g64_diag.py > gpurun_out/regreuse_g64_diag_$T.log 2>&1 || true
PLANTOS_HIP_LIB=build/ab/lib_gridc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_coop_reset.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "test_desync_autoreset_parity and g64" > gpurun_out/regreuse_tests_$T.log 2>&1 || true
echo all-d done
