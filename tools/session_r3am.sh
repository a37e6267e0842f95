#!/usr/bin/env bash
# round-3 GPU session am: the final library (w2's wave-kernel round trips + the re-staging
# slot skip; the 25x25 W2 variant measured slower in r3ak and removed): the GPU suite,
# smoke, the headline bench line, rocprof stats, FETCH / WRITE PMC, then the 25x25 and
# wave-kernel bench lines
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=r3am
bash tools/gpu_session.sh $T tests
tail -n 1 $OUT/tests_$T.log
bash tools/gpu_session.sh $T smoke bench stats pmcf pmcw \
  benchx:g25:--grid_25_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g40c48:--grid_40_--rays_48_--range_8_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5 \
  benchx:g64r32:--grid_64_--rays_64_--range_32_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5 \
  benchx:drv:--steps_20_--warmup_5 statsd pmcf64 pmcw64 bench64 \
  statsx:g25:--grid_25_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  pmcx:g25:FETCH_SIZE:--grid_25 pmcx:g25:WRITE_SIZE:--grid_25
echo pass done
