#!/usr/bin/env bash
# round-6 session k: the suite on lib_w14 (the f32 kernels' late LDS-DMA record staging + the
# done path out of line for the non-early kernels), A/B of w13 (late DMA), w14, w14b (out of line
# only) against lib_w11 (the tree's source)
set -euo pipefail
T=r6k
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w14.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w14_$T.log 2>&1
echo "w14 tests done"; tail -n 1 gpurun_out/tests_w14_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
W11=build/ab/lib_w11.so
L="$W11,build/ab/lib_w13.so,build/ab/lib_w14.so,build/ab/lib_w14b.so"
G64="--grid_64_--rays_64_--range_6_--steps_1000_--warmup_100_--desync-steps_2000_--gather-steps_0"
G32="--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:g25:2:$L:--grid_25_$A" \
  "ab:g21:2:$L:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:n4096:2:$L:--envs_4096_$A" \
  "ab:head:2:$W11,build/ab/lib_w14.so:$A" \
  "ab:g64:2:$W11,build/ab/lib_w14.so:$G64" \
  "ab:g32:2:$W11,build/ab/lib_w14.so:$G32"
echo all-k done
