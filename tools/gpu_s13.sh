# R101 workloads (C3 bf16, C5 fp16 1:2:1) and the two-stream timeline of the C2 step
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s13
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline --no-eval > gpurun_out/s13/bench_C3.json 2> gpurun_out/s13/c3.err
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --no-eval > gpurun_out/s13/bench_C5.json 2> gpurun_out/s13/c5.err
timeout -k 10 300 python bench.py --config C4 --no-cpu-baseline --no-eval > gpurun_out/s13/bench_C4.json 2> gpurun_out/s13/c4.err
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s13/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile > gpurun_out/s13/prof.log 2>&1
python3 tools/timeline.py gpurun_out/s13/prof/run_results.db > gpurun_out/s13/timeline.txt 2>&1
rm -rf gpurun_out/s13/prof
