#!/usr/bin/env bash
# round-6 session f: the suite on lib_w7 (w5 + two-record early path, two-word grid block in
# round 1, far stagger 8 without info staging), same-box A/B of each knob
set -euo pipefail
T=r6f
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w7.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w7_$T.log 2>&1
echo "w7 tests done"; tail -n 1 gpurun_out/tests_w7_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
W=build/ab/lib_w7.so
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:3:$H,$W,build/ab/lib_w7ne2.so:$A" \
  "ab:codes:2:$H,$W,build/ab/lib_w7ne2.so:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:g25:2:$H,$W,build/ab/lib_w7ngr2.so,build/ab/lib_w7nors.so:--grid_25_$A" \
  "ab:g21:2:$H,$W,build/ab/lib_w7nors.so:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:far:2:$H,$W:$GF"
echo all-f done
