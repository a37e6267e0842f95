#!/usr/bin/env bash
# round-6 session v: the driver-shaped window's first-replay cost, bench.py's preamble piece by piece
# (tools/window_probe.py, one window per process, alternating variants)
set -euo pipefail
OUT=gpurun_out/window_probe_r6v.jsonl; : > $OUT
for r in 1 2 3 4 5; do
  for v in "upload=1 episodes=1" "upload=1 episodes=0" "upload=0 episodes=0" "upload=1 episodes=0 idle_ms=5"; do
    timeout -k 10 120 python tools/window_probe.py $v >> $OUT 2>> gpurun_out/window_probe_r6v.err
  done
done
cat $OUT
