#!/usr/bin/env bash
# round-3 GPU session aa: the product library with the one-wave-per-env kernel's probe
# tables as byte offsets + shifts and 16-B long-row stores -- full GPU suite, then a
# same-box A/B against HEAD's library over the wave geometries and the headline
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_session.sh r3aa tests smoke
tail -n 3 $OUT/tests_r3aa.log
A=build/ab/lib_base.so; B=build/ab/lib_prod1.so
bash tools/ab_bench.sh r3aa_g64r32 2 $A $B -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3aa_g8r20 2 $A $B -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3aa_head 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 4096 --gather-steps 0 > /dev/null
echo ab done
