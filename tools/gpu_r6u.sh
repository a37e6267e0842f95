#!/usr/bin/env bash
# round-6 session u: the driver-shaped bench window with the auto-reset counter read before the
# warm-up (PLANTOS_EP0=warmup, new default) against between warm-up and window (window), alternating
set -euo pipefail
OUT=gpurun_out/ep0_r6u.jsonl; : > $OUT
for r in 1 2 3 4 5 6; do
  for at in window warmup; do
    PLANTOS_EP0=$at timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --desync-steps 0 \
      --gather-steps 0 > gpurun_out/u_one.json 2> gpurun_out/u_one.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/u_one.json')); print(json.dumps({'ep0': sys.argv[1], 'round': int(sys.argv[2]), 'us': d['ms_per_step']*1e3, 'value': d['value'], 'window_events_us': d['roofline'].get('kernel_us_window'), 'resets': d.get('resets_in_window', d.get('resets_in_warmup_and_window'))}))" $at $r >> $OUT
  done
done
for r in 1 2 3; do
  timeout -k 10 120 python tools/window_probe.py episodes=0 episodes_before=1 >> gpurun_out/window_probe_r6u.jsonl 2>> gpurun_out/window_probe_r6u.err
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_r6u.json 2> gpurun_out/bench_drv_r6u.err
cat $OUT
