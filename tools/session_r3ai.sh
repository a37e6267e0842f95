#!/usr/bin/env bash
# round-3 GPU session ai: the measurement pass of the in-tree product library (w2's
# pe_step_wave round trips; the sector kernels' code is unchanged): the GPU suite, smoke,
# bench lines, rocprof kernel stats, FETCH / WRITE PMC passes (tools/session_r3aj.sh) --
# then a pe_step_wave A/B: aa1feb1 (base: the session-start source), w2 (= the product's source), w6 = w2 + ray
# rounds without the per-round early exit, w7 = w6 + re-staging slots past the window
# skipped (diff profiles/r3ai/uniform_ray_rounds_and_slot_skip.diff)
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/session_r3aj.sh
A=build/ab/lib_base.so; B=build/ab/lib_w2.so; C=build/ab/lib_w6.so; D=build/ab/lib_w7.so
PLANTOS_HIP_LIB=$D timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_geometry_sweep.py tests/test_gpu_parity.py > $OUT/r3ai_tests_w7.log 2>&1
tail -2 $OUT/r3ai_tests_w7.log
bash tools/ab_bench.sh r3ai_g64r32 2 $A $B $C $D -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 1000 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ai_g40c48 1 $A $B $C $D -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ai_g8r20 1 $A $B $C $D -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
