# forward BN apply: rows in flight per thread 2 / 4 / 8 (kernel stats + whole step)
set -e
mkdir -p gpurun_out/s14
timeout -k 10 600 bash tools/ab_stats.sh gpurun_out/s14/stats ua2 ua8 > gpurun_out/s14/stats.log 2>&1
REPS=2 timeout -k 10 400 bash tools/ab_bench.sh ua2 ua8 > gpurun_out/s14/ab.txt 2>&1
