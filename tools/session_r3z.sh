#!/usr/bin/env bash
# round-3 GPU session z: pe_step_wave restage with a fixed lane -> (row, word) map, all
# slot reads in flight at once (wv5) vs wv4 (probe offsets + shifts, 16-B long-row
# stores) vs HEAD (base); wave parity first
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_wv4.so; C=build/ab/lib_wv5.so
PLANTOS_HIP_LIB=$C timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_geometry_sweep.py tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_curriculum_autoreset.py > $OUT/r3z_tests.log 2>&1
tail -2 $OUT/r3z_tests.log
bash tools/ab_bench.sh r3z_g64r32 2 $A $B $C -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3z_g8r20 2 $A $B $C -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3z_g40c48 2 $A $B $C -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
