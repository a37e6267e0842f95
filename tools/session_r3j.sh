#!/usr/bin/env bash
# round-3 GPU session j: 4-word visit rows up to G=25 (knobs11) vs knobs9 at 25x25,
# 21x21/C10/R2 and the headline; tests of the product library
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs9.so; B=build/ab/lib_knobs11.so
bash tools/ab_bench.sh r3j_g25 3 $A $B -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3j_g21 2 $A $B -- --grid 21 --rays 10 --range 2 --plants 8 --obstacles 50 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3j_head 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
bash tools/gpu_session.sh r3j tests
