# two-stream step phases (rocprofv3 kernel trace of an unprofiled bench run)
set -e
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s18/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-eval --no-profile > gpurun_out/s18/bench.log 2>&1
python3 tools/phases.py gpurun_out/s18/prof/run_results.db > gpurun_out/s18/phases.txt 2>&1
python3 tools/timeline.py gpurun_out/s18/prof/run_results.db > gpurun_out/s18/timeline.txt 2>&1
rm -rf gpurun_out/s18/prof
