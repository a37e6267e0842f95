set -e
for f in 0 54000 80000 160000; do
  PE_LDS_FLOOR=$f timeout -k 10 200 python bench.py --no-cpu-baseline --graph 0 --steps 1000 > gpurun_out/occ_$f.json
  PE_LDS_FLOOR=$f timeout -k 10 200 python bench.py --no-cpu-baseline --graph 0 --steps 300 --grid 64 --rays 64 > gpurun_out/occ64_$f.json
done
echo done
