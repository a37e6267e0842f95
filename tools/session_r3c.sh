#!/usr/bin/env bash
# round-3 GPU session c: early record A/B (knobs2 = before, knobs3 = after), window
# bracket variants, stamps at 25x25, tests + driver-shaped bench of the product lib
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs2.so; B=build/ab/lib_knobs3.so
timeout -k 10 120 python tools/diag/window_overhead2.py > $OUT/window2_r3c.json 2> $OUT/window2_r3c.err
echo window done
bash tools/ab_bench.sh early_desync_r3c 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh early_sync_r3c 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh early_4096_r3c 2 $A $B -- --envs 4096 --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
C=build/ab/lib_knobs4.so
bash tools/ab_bench.sh early_g25_r3c 2 $A $B $C -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh epb65536_r3c 2 $C $C,PE_QUAD_EPB=32 $C,PE_QUAD_EPB=16 -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
timeout -k 10 180 python tools/stamps.py run --grid 25 > $OUT/stamps25_r3c.json 2> $OUT/stamps25_r3c.err
echo stamps done
bash tools/gpu_session.sh r3c benchx:drv:--steps_20_--warmup_5 tests
