#!/usr/bin/env bash
# round-3 GPU session p: the driver-shaped window (--steps 20 --warmup 5) with one
# captured graph vs direct launches, alternating, 4 rounds; the one-rank RCCL bench line
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/drv_ab_r3p.jsonl
for r in 1 2 3 4; do
  for gflag in 64 0; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph $gflag --no-cpu-baseline --desync-steps 0 --gather-steps 0 > $OUT/drv_one.json 2> $OUT/drv_one.err
    python3 -c "import json,sys; d=json.loads(open('$OUT/drv_one.json').read().splitlines()[-1]); print(json.dumps({'graph': int(sys.argv[1]), 'round': int(sys.argv[2]), 'wall_us': d['ms_per_step']*1e3, 'kernel_us': d['roofline']['kernel_ms']*1e3, 'value': d['value'], 'launch': d['config']['launch']}))" $gflag $r >> $OUT/drv_ab_r3p.jsonl
  done
done
cat $OUT/drv_ab_r3p.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 \
  bench.py --gpus 1 --steps 2000 --warmup 100 --desync-steps 2000 --gather-steps 500 --no-cpu-baseline > $OUT/rccl1_r3p.json 2> $OUT/rccl1_r3p.err
echo done
