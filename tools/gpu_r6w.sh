#!/usr/bin/env bash
# round-6 session w: the driver-shaped window (--steps 20 --warmup 5) under each host wait policy
# (bench.py PLANTOS_WAIT), alternating, 5 rounds
set -euo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/wait_r6w.jsonl; : > $OUT
for r in 1 2 3 4 5; do
  for pol in auto spin yield blocking poll; do
    PLANTOS_WAIT=$pol timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --desync-steps 0 \
      --gather-steps 0 > gpurun_out/w_one.json 2> gpurun_out/w_one.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/w_one.json')); print(json.dumps({'pol': sys.argv[1], 'round': int(sys.argv[2]), 'us': d['ms_per_step']*1e3, 'value': d['value'], 'events_us': d['roofline']['kernel_us_events'], 'host_wait': d['config'].get('host_wait')}))" $pol $r >> $OUT
  done
done
cat $OUT
