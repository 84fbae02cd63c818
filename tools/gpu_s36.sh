# deferred stem update A/B (--no-defer-stem = the joined order) and kernel stats of the new
# max-pool / SGDM kernels (single-stream backward), then a trace of the step's tail
set -e
mkdir -p gpurun_out/s36
export TMPDIR=/tmp
for r in 1 2; do
  for v in joined defer; do
    flag=""
    if [ $v = joined ]; then flag="--no-defer-stem"; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval $flag > gpurun_out/s36/ab_$v.json 2> gpurun_out/s36/ab.err
    echo "$v $(tail -n 1 gpurun_out/s36/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/s36/ab.txt
  done
done
SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s36/st -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-eval --no-profile > gpurun_out/s36/st.log 2>&1
python3 tools/rocpd_stats.py gpurun_out/s36/st/run_results.db gpurun_out/s36/kernel_stats.csv > gpurun_out/s36/kernel_classes.txt
rm -rf gpurun_out/s36/st
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s36/tr -o run -- python3 bench.py --steps 4 --warmup 2 --no-profile --no-cpu-baseline --no-eval > gpurun_out/s36/tr.log 2>&1
python3 tools/timeline.py gpurun_out/s36/tr/run_results.db 40 > gpurun_out/s36/timeline.txt 2>&1
rm -rf gpurun_out/s36/tr
grep -h 'sgdm\|maxpool' gpurun_out/s36/kernel_stats.csv | cut -c1-160
