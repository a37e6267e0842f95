set -e
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 > gpurun_out/st_nt.json
for v in sc1 sc1_nt sc0_sc1_nt sc0_sc1 temporal; do
  PLANTOS_HIP_LIB=build/st_$v/libplantos_hip.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 > gpurun_out/st_$v.json
done
echo done
