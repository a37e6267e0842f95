#!/usr/bin/env bash
# round-3 GPU session ak: the final candidate f1 = w2 (wave-kernel round trips) + the
# re-staging slots past the window skipped (w7's half that paid: 40x40/C48 72.9 -> 69.0 us;
# its other half, ray rounds without the early exit, made 8x8/R20 67 -> 78 us) + the
# 25x25 kernel's rows of 2 words at compile time (grid and visit rows in one round trip).
# f1 parity, the 25x25 A/B vs aa1feb1 (base) and w2, the measurement pass of the in-tree
# product (f1's source) with the full GPU suite, then the other A/Bs.
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_w2.so; C=build/ab/lib_f1.so
PLANTOS_HIP_LIB=$C timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_geometry_sweep.py > $OUT/r3ak_tests_f1.log 2>&1
tail -2 $OUT/r3ak_tests_f1.log
bash tools/ab_bench.sh r3ak_g25 3 $A $B $C -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
PASS_TAG=r3al bash tools/session_r3aj.sh
bash tools/ab_bench.sh r3ak_head 2 $A $C -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ak_g40c48 2 $A $B $C -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ak_g8r20 1 $A $B $C -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ak_g64r32 1 $A $B $C -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
