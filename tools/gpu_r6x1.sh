#!/usr/bin/env bash
# round-6 final pass, call 1: the suite, smoke and every bench line on the in-tree library
# (tools/measure_pass1.sh), then a same-box confirmation against the round-5 library
set -euo pipefail
T=r6x
bash tools/measure_pass1.sh $T
H=build/ab/lib_head.so
W=build/ab/lib_w11.so
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:2:$H,$W:$A" \
  "ab:g64:2:$H,$W:$G64" \
  "ab:codes:2:$H,$W:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500" \
  "ab:far:2:$H,$W:$GF"
echo x1 done
