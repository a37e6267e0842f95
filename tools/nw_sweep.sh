set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests_nw.log 2>&1
for nw in 4 8; do
  PE_QUAD_WAVES=$nw timeout -k 10 200 python bench.py --no-cpu-baseline --graph 0 --steps 1000 > gpurun_out/nw_$nw.json
  PE_QUAD_WAVES=$nw timeout -k 10 200 python bench.py --no-cpu-baseline --graph 0 --steps 300 --grid 64 --rays 64 > gpurun_out/nw64_$nw.json
done
echo done
