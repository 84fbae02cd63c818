# round-end check of HEAD: the whole -m gpu suite, smoke, the driver's bench command (CPU baseline
# and eval included), the R101 workload lines (C3 / C4 bf16, C5 fp16)
set -e
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/final/tests.log 2>&1
tail -n 1 gpurun_out/final/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
tail -n 1 gpurun_out/final/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
tail -n 1 gpurun_out/final/bench.json | cut -c1-200
for cfg in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/final/bench_$cfg.json 2>> gpurun_out/final/bench.err
  tail -n 1 gpurun_out/final/bench_$cfg.json | cut -c1-160
done
