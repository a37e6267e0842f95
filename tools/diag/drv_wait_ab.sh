set -e
mkdir -p gpurun_out/drvab
for i in 1 2 3; do
  for w in none 100 1000; do
    if [ $w = none ]; then
      timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > gpurun_out/drvab/$w.$i.json
    else
      ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > gpurun_out/drvab/$w.$i.json
    fi
    echo "$w $i $(tail -c 300 gpurun_out/drvab/$w.$i.json | head -c 80)"
  done
done
