#!/usr/bin/env bash
# round-6 first GPU session: the suite on the tree library and on the register-staged A/B
# library, the bench line, the gather leg's trace, same-box desync A/B, desync stats
set -euo pipefail
T=r6a
mkdir -p gpurun_out
bash tools/gpu_session.sh $T tests
PLANTOS_HIP_LIB=build/ab/lib_rs.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_rs_$T.log 2>&1
echo "rs tests done"
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
bash tools/gpu_session.sh $T smoke bench \
  statsx:gather:--steps_20_--warmup_5_--desync-steps_0_--gather-steps_500_--no-cpu-baseline \
  "ab:g25:3:tree,build/ab/lib_rs.so:--grid_25_$A" \
  "ab:n4096:3:tree,build/ab/lib_rs.so:--envs_4096_$A" \
  "ab:g21:2:tree,build/ab/lib_rs.so:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A"
bash tools/measure_desync.sh $T
