#!/usr/bin/env bash
# round-6 session z: rocprof kernel stats of the 4096-env step, in-tree library (pass y) and the
# r6x library's source (w11) on one box, alternating
set -euo pipefail
S="statsx:n4096:--envs_4096_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline"
for i in 1 2; do
  bash tools/gpu_session.sh r6z_tree$i "$S"
  PLANTOS_HIP_LIB=build/ab/lib_w11.so bash tools/gpu_session.sh r6z_w11_$i "$S"
done
echo z done
