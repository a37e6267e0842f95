#!/usr/bin/env bash
# round-3 GPU session u: the one-word sector kernel's rays run between two barriers
# rays overlapped nothing before: vmcnt(0) at the llive join) and a 2-chunk early store loop
# chunks stored before the visit half (PE_EARLY_STORE) -- vs base (HEAD) and the
# reordered source without either (re0); parity of re2 first
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_re1.so; C=build/ab/lib_re2.so; Z=build/ab/lib_re0.so
PLANTOS_HIP_LIB=$C timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_geometry_sweep.py tests/test_gpu_curriculum_autoreset.py > $OUT/r3v_tests.log 2>&1
tail -2 $OUT/r3v_tests.log
bash tools/ab_bench.sh r3v_head 3 $A $B $C -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3v_g15 2 $A $B $C -- --grid 15 --range 4 --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3v_n4096 2 $A $B $C -- --envs 4096 --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
