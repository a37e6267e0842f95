#!/usr/bin/env bash
# round-3 GPU session ah: w5 = w3 + the single-done early-record reset's stores (info,
# state rows, terminal obs, scalars) issued after the done barrier, beside the other
# waves' tile stores, vs HEAD (base); desync parity with w5 first
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_w5.so
PLANTOS_HIP_LIB=$B timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_coop_reset.py tests/test_gpu_parity.py tests/test_gpu_curriculum_autoreset.py tests/test_gpu_vec_env.py > $OUT/r3ah_tests.log 2>&1
tail -2 $OUT/r3ah_tests.log
bash tools/ab_bench.sh r3ah_head 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ah_g15 2 $A $B -- --grid 15 --rays 16 --range 4 --plants 6 --obstacles 8 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
