#!/usr/bin/env bash
# round-3 GPU session ae: the done path's table reads from the step kernel's LDS copy
# as LDS reads (dq1) instead of flat loads through a select of an LDS and a global
# pointer (each waited vmcnt(0): for every store in flight) -- desynchronized steps
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_dq1.so
PLANTOS_HIP_LIB=$B timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_coop_reset.py tests/test_gpu_curriculum_autoreset.py tests/test_gpu_parity.py > $OUT/r3ae_tests.log 2>&1
tail -n 1 $OUT/r3ae_tests.log
bash tools/ab_bench.sh r3ae_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ae_g25d 2 $A $B -- --grid 25 --desync --steps 8192 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ae_g64d 2 $A $B -- --grid 64 --rays 64 --desync --steps 4096 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ae_sync 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
