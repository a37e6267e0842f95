set -e
mkdir -p gpurun_out; : > gpurun_out/drv_ab_${TAG:-r4l}.jsonl
for i in 1 2 3 4 5; do for m in graph direct; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --short-window $m --desync-steps 0 --gather-steps 0 --no-cpu-baseline > gpurun_out/one.json 2>gpurun_out/one.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/one.json')); print(json.dumps({'mode': sys.argv[1], 'round': int(sys.argv[2]), 'wall_us': d['ms_per_step']*1e3, 'events_us': d['roofline']['kernel_ms']*1e3, 'value': d['value'], 'launch': d['config']['launch']}))" $m $i >> gpurun_out/drv_ab_${TAG:-r4l}.jsonl
done; done
