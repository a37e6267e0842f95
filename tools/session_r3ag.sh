#!/usr/bin/env bash
# round-3 GPU session ag: pe_step_wave round trips and re-staging, vs HEAD (base):
#   w1: round 1 (scalars + both action words) unconditional, round 2's visit rows and
#       first window pass landing in one wait
#   w2: w1 + round 1 issued before the shared header's copy
#   w3: w2 + the aligned re-staging with lane = (row, word) of a slot (one division per
#       lane, slots past the window skipped uniformly)
# wave parity with w3 first
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_w1.so; C=build/ab/lib_w2.so; D=build/ab/lib_w3.so
PLANTOS_HIP_LIB=$D timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_geometry_sweep.py tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_curriculum_autoreset.py > $OUT/r3ag_tests.log 2>&1
tail -2 $OUT/r3ag_tests.log
bash tools/ab_bench.sh r3ag_g64r32 2 $A $B $C $D -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 1000 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ag_g8r20 2 $A $B $C $D -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ag_g40c48 2 $A $B $C $D -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
