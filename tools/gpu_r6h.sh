#!/usr/bin/env bash
# round-6 session h: the suite on the in-tree library (commit 5b2bcc3) and on lib_w10 (batched
# done-path row copies), the far kernel's desync (w9 = the tree's source) and the w10 A/B
set -euo pipefail
T=r6h
mkdir -p gpurun_out
bash tools/gpu_session.sh $T tests
tail -n 1 gpurun_out/tests_$T.log
PLANTOS_HIP_LIB=build/ab/lib_w10.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w10_$T.log 2>&1
echo "w10 tests done"; tail -n 1 gpurun_out/tests_w10_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
H=build/ab/lib_head.so
W9=build/ab/lib_w9.so
W10=build/ab/lib_w10.so
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:far:2:$H,$W9,$W9+PE_STAGGER=4,$W10:$GF" \
  "ab:head:2:$W9,$W10:$A" \
  "ab:n4096:2:$W9,$W10:--envs_4096_$A" \
  "ab:g25:2:$W9,$W10:--grid_25_$A" \
  "ab:g64:2:$W9,$W10:$G64" \
  "ab:codes:2:$W9,$W10:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500"
echo all-h done
