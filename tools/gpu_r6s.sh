#!/usr/bin/env bash
# round-6 session s: graph replays against direct launches -- the long window (20000 steps) and the
# driver-shaped 20-step window -- alternating
set -euo pipefail
OUT=gpurun_out/launch_r6s.jsonl; : > $OUT
one() {
  local tag=$1; shift
  timeout -k 10 180 python bench.py --no-cpu-baseline --desync-steps 0 --gather-steps 0 "$@" > gpurun_out/s_one.json 2> gpurun_out/s_one.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/s_one.json')); r=d['roofline']; print(json.dumps({'tag': sys.argv[1], 'us': d['ms_per_step']*1e3, 'window_events_us': r.get('kernel_us_window'), 'events_us': r['kernel_us_events'], 'launch': d['config']['launch']}))" $tag >> $OUT
}
for r in 1 2; do
  one long_graph --steps 20000 --warmup 200
  one long_direct --steps 20000 --warmup 200 --graph 0
done
for r in 1 2 3 4; do
  one drv_graph --steps 20 --warmup 5
  one drv_direct --steps 20 --warmup 5 --short-window direct
done
cat $OUT
