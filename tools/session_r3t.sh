#!/usr/bin/env bash
# round-3 GPU session t: 16-B visit rows for the multi-word kernel at G <= 25 (the
# V16 variant, NW = 4) vs 5-word rows, same source
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_nw16off.so; B=build/ab/lib_nw16on.so
bash tools/ab_bench.sh r3t_g25 3 $A $B -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3t_g25r4 2 $A $B -- --grid 25 --range 4 --steps 4096 --warmup 200 --desync-steps 4096 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3t_head 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 4096 --gather-steps 0 > /dev/null
echo ab done
