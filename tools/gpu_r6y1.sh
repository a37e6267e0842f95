#!/usr/bin/env bash
# round-6 final pass y (library after the done-path change), call 1: the suite, smoke and every
# bench line on the in-tree library (tools/measure_pass1.sh), then a same-box confirmation against
# the r6x library's source (w11)
set -euo pipefail
T=r6y
bash tools/measure_pass1.sh $T
W=build/ab/lib_w11.so
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:2:$W,tree:$A" \
  "ab:n4096:2:$W,tree:--envs_4096_$A"
echo y1 done
