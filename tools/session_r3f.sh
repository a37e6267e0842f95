#!/usr/bin/env bash
# round-3 GPU session f: early record issued before round 2 + LDS tables in the
# reset path (knobs7) vs behind the compute phase (knobs5); tests; bench lines
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs5.so; B=build/ab/lib_knobs7.so
bash tools/ab_bench.sh r3f_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3f_sync 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3f_g21 2 $A $B -- --grid 21 --rays 10 --range 2 --plants 8 --obstacles 50 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
bash tools/gpu_session.sh r3f tests smoke benchx:drv:--steps_20_--warmup_5 bench
