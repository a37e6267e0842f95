#!/usr/bin/env bash
# round-3 GPU session ad: probes of the multi-word sector kernel's round 2 at 25x25
# (timing only, wrong results): without its grid-row loads, without its visit-row loads
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_base.so; B=build/ab/lib_p_nogrid.so; C=build/ab/lib_p_novis.so
bash tools/ab_bench.sh r3ad_g25 2 $A $B $C -- --grid 25 --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
