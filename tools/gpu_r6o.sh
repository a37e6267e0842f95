#!/usr/bin/env bash
# round-6 session o: phase stamps of the one-wait done path (ow1st) against ow0st, desynchronized;
# A/B of the one-wait path restricted to the one-word f32 kernels (ow1) against ow0
set -euo pipefail
T=r6o
mkdir -p gpurun_out
st() { local nm=$1; shift; timeout -k 10 120 python tools/stamps.py run "$@" > gpurun_out/stamps_${nm}_$T.json 2> gpurun_out/stamps_${nm}_$T.err; }
for v in ow0st ow1st; do
  st n4096d_$v --desync --envs 4096 --epb 16 --waves 8 --lib build/ab/lib_$v.so
  st headd_$v --desync --lib build/ab/lib_$v.so
done
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
L=build/ab/lib_ow0.so,build/ab/lib_ow1.so
bash tools/gpu_session.sh $T \
  "ab:head:3:$L:$A" \
  "ab:n4096:3:$L:--envs_4096_$A" \
  "ab:g21:2:$L:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:g15:2:$L:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_$A" \
  "ab:g25:2:$L:--grid_25_$A" \
  "ab:codes:2:$L:--steps_200_--warmup_100_--desync-steps_0_--gather-steps_500"
echo all-o done
