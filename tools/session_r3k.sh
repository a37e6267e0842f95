#!/usr/bin/env bash
# round-3 GPU session k: the runtime-(C, R) sector kernel -- tests first (parity of
# the new kernel), then A/B vs the one-wave-per-env kernel (PE_STEP_KERNEL=wave) at
# 32x32/C24/R9 and 7x7/C12/R3, and the headline vs knobs9
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs9.so; B=build/ab/lib_knobs12.so
bash tools/gpu_session.sh r3k tests
bash tools/ab_bench.sh r3k_g32 2 "$B,PE_STEP_KERNEL=wave" $B -- --grid 32 --rays 24 --range 9 --plants 20 --obstacles 30 --steps 2000 --warmup 100 --desync-steps 4096 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3k_g7 2 "$B,PE_STEP_KERNEL=wave" $B -- --grid 7 --rays 12 --range 3 --plants 3 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 4096 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3k_head 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3k_g25 2 $A $B -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
