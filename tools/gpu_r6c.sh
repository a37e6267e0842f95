#!/usr/bin/env bash
# round-6 session c: the suite on lib_w2 (register-staged record with LDS flags, runtime
# kernel's probe table in round 1 + register-window rays), same-box A/B against lib_head
# (HEAD built the same way), the stagger knob on the byte-tile kernels, the hazard repro
set -euo pipefail
T=r6c
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w2_$T.log 2>&1
echo "w2 tests done"; tail -n 1 gpurun_out/tests_w2_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G40="--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:g32:2:$H,build/ab/lib_w.so,build/ab/lib_wnoreg.so,build/ab/lib_w2.so:$G32" \
  "ab:g40c48:2:$H,build/ab/lib_wnoreg.so,build/ab/lib_w2.so:$G40" \
  "ab:g25:3:$H,build/ab/lib_w2.so:--grid_25_$A" \
  "ab:n4096:3:$H,build/ab/lib_w2.so:--envs_4096_$A" \
  "ab:g21:2:$H,build/ab/lib_w2.so:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:codesstag:2:$H,$H+PE_STAGGER=0:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g32stag:2:$H,$H+PE_STAGGER=0:$G32" \
  "ab:g40stag:2:$H,$H+PE_STAGGER=0:$G40"
PLANTOS_HIP_LIB=build/ab/lib_gridc.so timeout -k 10 120 python tools/diag/g64_diag.py > gpurun_out/regreuse_g64_diag_$T.log 2>&1 || true
PLANTOS_HIP_LIB=build/ab/lib_gridc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_coop_reset.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "test_desync_autoreset_parity and g64" > gpurun_out/regreuse_tests_$T.log 2>&1 || true
echo all-c done
