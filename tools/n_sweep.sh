set -e
for n in 8192 16384 32768 49152 65536 98304 131072; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 --envs $n > gpurun_out/n_$n.json
done
echo done
