# kernel trace of unprofiled two-stream steps: per-stream busy/idle, phases and the step's tail
set -e
mkdir -p gpurun_out/s45
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s45/tr -o run -- python3 bench.py --steps 4 --warmup 2 --no-profile --no-cpu-baseline --no-eval > gpurun_out/s45/bench.log 2>&1
python3 tools/timeline.py gpurun_out/s45/tr/run_results.db 120 > gpurun_out/s45/timeline.txt 2>&1
python3 tools/phases.py gpurun_out/s45/tr/run_results.db > gpurun_out/s45/phases.txt 2>&1 || true
rm -rf gpurun_out/s45/tr
head -n 5 gpurun_out/s45/timeline.txt
