#!/usr/bin/env bash
# round-3 GPU session n: the single-done fast path (no barrier; the commit wave stores
# its env's chunks, the other waves the rest of the tile at once) -- tests first, then
# A/B vs knobs12
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs12.so; B=build/ab/lib_knobs14.so
bash tools/gpu_session.sh r3n tests
bash tools/ab_bench.sh r3n_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3n_sync 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
