set -e
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d gpurun_out/pmc_l2 -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/pmc_l2.json 2>gpurun_out/pmc_l2.err
bash tools/gpu_profile.sh r1i stats pmc
