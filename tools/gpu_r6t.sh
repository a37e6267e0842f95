#!/usr/bin/env bash
# round-6 session t: the driver-shaped window under a one-rank torchrun job (the N>1 code path:
# process group, barriers, max over ranks), the window's barriers through RCCL (nccl) or a host
# gloo group (gloo), alternating
set -euo pipefail
OUT=gpurun_out/barrier_r6t.jsonl; : > $OUT
P=29600
for r in 1 2 3 4 5; do
  for bk in nccl gloo; do
    P=$((P + 1))
    PLANTOS_BARRIER=$bk timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $P bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
      --desync-steps 0 --gather-steps 0 > gpurun_out/t_one.json 2> gpurun_out/t_one.err
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/t_one.json') if l.startswith('{')][-1]); print(json.dumps({'barrier': sys.argv[1], 'round': int(sys.argv[2]), 'us': d['ms_per_step']*1e3, 'value': d['value'], 'window_events_us': d['roofline'].get('kernel_us_window'), 'cfg_barrier': d['config'].get('barrier')}))" $bk $r >> $OUT
  done
done
cat $OUT
