#!/usr/bin/env bash
# round-6 session m: the backend scheduler strategy (-mllvm -amdgpu-sched-strategy=...) of the
# final source: max-ilp (s1), max-memory-clause (s2), iterative-ilp (s3) against the default (w11)
set -euo pipefail
T=r6m
mkdir -p gpurun_out
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
L=build/ab/lib_w11.so,build/ab/lib_s1.so,build/ab/lib_s2.so,build/ab/lib_s3.so
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:head:2:$L:$A" \
  "ab:g25:2:$L:--grid_25_$A" \
  "ab:n4096:2:$L:--envs_4096_$A" \
  "ab:g64:1:$L:$G64" \
  "ab:g32:1:$L:$G32"
echo all-m done
