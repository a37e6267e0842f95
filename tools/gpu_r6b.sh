#!/usr/bin/env bash
# round-6 session b: the suite on the register-staged A/B library (rs: kRegStage + the
# runtime kernel's probe table in round 1), same-box A/B against the tree library, phase
# stamps of the f32 and codes steps desynchronized, the visit-byte store A/B (visplain)
set -euo pipefail
T=r6b
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_rs.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_rs_$T.log 2>&1
echo "rs tests done"; tail -n 1 gpurun_out/tests_rs_$T.log
A="--steps_4096_--warmup_200_--desync-steps_8192_--gather-steps_0"
bash tools/gpu_session.sh $T \
  "ab:g25:3:tree,build/ab/lib_rs.so:--grid_25_$A" \
  "ab:n4096:3:tree,build/ab/lib_rs.so:--envs_4096_$A" \
  "ab:g21:2:tree,build/ab/lib_rs.so:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_$A" \
  "ab:g32:2:tree,build/ab/lib_rs.so:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_2000_--gather-steps_0" \
  "ab:g40c48:2:tree,build/ab/lib_rs.so:--grid_40_--rays_48_--range_8_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0" \
  "ab:head:3:tree,build/ab/lib_visplain.so:$A"
timeout -k 10 120 python tools/stamps.py run --desync > gpurun_out/stampsd_f32_$T.json 2> gpurun_out/stampsd_f32_$T.err
timeout -k 10 120 python tools/stamps.py run --desync --codes > gpurun_out/stampsd_codes_$T.json 2> gpurun_out/stampsd_codes_$T.err
echo stamps done
PLANTOS_HIP_LIB=build/ab/lib_visplain.so bash tools/gpu_session.sh ${T}_vp pmcf pmcw
bash tools/gpu_session.sh ${T}_tree pmcf pmcw
echo all-b done
