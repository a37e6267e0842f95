#!/usr/bin/env bash
# round-3 GPU session x: pe_step_wave's obs row store -- base (HEAD) vs the aligned-window
# offsets from pe_create with 16-B sc1 row stores (wv1), one float per lane (wv2),
# 16-B plain stores (wv3)
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_wv1.so; C=build/ab/lib_wv2.so; D=build/ab/lib_wv3.so
bash tools/ab_bench.sh r3x_g64r32 2 $A $B $C $D -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3x_g8r20 2 $A $B $C $D -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3x_g40c48 2 $A $B $C $D -- --grid 40 --rays 48 --range 8 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
