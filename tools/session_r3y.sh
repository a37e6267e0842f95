#!/usr/bin/env bash
# round-3 GPU session y: pe_step_wave with the aligned-window probes as byte offsets +
# bit shifts (one SDWA add and one bfe per probe) and 16-B stores of long obs rows
# (wv4) vs HEAD (base) and the 16-B plain stores alone (wv3); wave parity first
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_wv3.so; C=build/ab/lib_wv4.so
PLANTOS_HIP_LIB=$C timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_geometry_sweep.py tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_curriculum_autoreset.py > $OUT/r3y_tests.log 2>&1
tail -2 $OUT/r3y_tests.log
bash tools/ab_bench.sh r3y_g64r32 2 $A $B $C -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3y_g8r20 2 $A $B $C -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3y_g40c48 2 $A $B $C -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
