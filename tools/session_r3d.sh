#!/usr/bin/env bash
# round-3 GPU session d: the early record restricted to one-word 64-env kernels
# (knobs5) vs before (knobs2); 25x25 with 16-B row loads; 8 waves x 16 envs at 4096;
# 32/16-env workgroups at 65536; tests of the product library
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs2.so; B=build/ab/lib_knobs5.so; C=build/ab/lib_knobs6.so
bash tools/ab_bench.sh r3d_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3d_sync 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3d_4096 3 $A $B "$C,PE_QUAD_WAVES=8 PE_QUAD_EPB=16" -- --envs 4096 --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3d_g25 3 $A $B -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3d_epb65536 2 $B $B,PE_QUAD_EPB=32 $B,PE_QUAD_EPB=16 -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
bash tools/gpu_session.sh r3d tests
