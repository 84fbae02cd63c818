# round-end check of HEAD (after the dual BN backward and the dual data gradient): whole -m gpu suite, smoke, the driver's
# bench command, R101 lines, rocprofv3 kernel classes (single-stream backward)
set -e
mkdir -p gpurun_out/final3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/final3/tests.log 2>&1
tail -n 1 gpurun_out/final3/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1
tail -n 1 gpurun_out/final3/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final3/bench.json 2> gpurun_out/final3/bench.err
tail -n 1 gpurun_out/final3/bench.json | cut -c1-160
for cfg in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/final3/bench_$cfg.json 2>> gpurun_out/final3/bench.err
  tail -n 1 gpurun_out/final3/bench_$cfg.json | cut -c1-140
done
SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final3/st -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval > gpurun_out/final3/st.log 2>&1
python3 tools/rocpd_stats.py gpurun_out/final3/st/run_results.db gpurun_out/final3/kernel_stats.csv > gpurun_out/final3/kernel_classes.txt
rm -rf gpurun_out/final3/st
tail -n 3 gpurun_out/final3/kernel_classes.txt
