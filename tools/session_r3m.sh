#!/usr/bin/env bash
# round-3 GPU session m: the loader env's position by bpermute (knobs13) vs a second
# scalar load (knobs12), and both vs round-2-era knobs9 at 64x64 (regression check)
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs9.so; B=build/ab/lib_knobs12.so; C=build/ab/lib_knobs13.so
bash tools/ab_bench.sh r3m_head 3 $B $C -- --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3m_64 2 $A $B $C -- --grid 64 --rays 64 --range 6 --steps 2000 --warmup 100 --desync-steps 3000 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3m_4096 2 $B $C -- --envs 4096 --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3m_g25 2 $B $C -- --grid 25 --steps 4096 --warmup 200 --desync-steps 20480 --gather-steps 0 > /dev/null
echo ab done
