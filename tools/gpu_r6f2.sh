#!/usr/bin/env bash
# round-6 closing check on the final tree: the GPU suite, smoke, and the driver-shaped bench line
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_r6f2.log 2>&1
tail -n 1 gpurun_out/tests_r6f2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6f2.log 2>&1
tail -n 1 gpurun_out/smoke_r6f2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_r6f2.json 2> gpurun_out/bench_drv_r6f2.err
cat gpurun_out/bench_drv_r6f2.json
