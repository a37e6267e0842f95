set -e
for st in 0 1 2 3 4 6 8; do
  PE_STAGGER=$st timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1000 > gpurun_out/stag_$st.json
done
echo done
