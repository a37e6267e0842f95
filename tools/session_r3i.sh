#!/usr/bin/env bash
# round-3 GPU session i: the early record's state writes at the start of the compute
# phase (knobs10) vs in the done path (knobs9); stamps; tests; driver-shaped benches
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs9.so; B=build/ab/lib_knobs10.so
bash tools/ab_bench.sh r3i_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3i_sync 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
timeout -k 10 180 python tools/stamps.py run --desync > $OUT/stampsd_r3i.json 2> $OUT/stampsd_r3i.err
echo stamps done
bash tools/gpu_session.sh r3i tests benchx:drv:--steps_20_--warmup_5 benchx:drv2:--steps_20_--warmup_5 benchx:drv3:--steps_20_--warmup_5
