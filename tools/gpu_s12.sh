# weight-gradient split sizing: single ops, parity, bench (profiled roofline) and step A/B vs build/prev
set -e
mkdir -p gpurun_out/s12
for l in b3c1 b3c3 b4c1 b4c3 b4c2 b3c2 head1 b1c2 b2c2 b1c3; do timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s12/ops.txt 2>&1; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py -k "wgrad or step" > gpurun_out/s12/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval > gpurun_out/s12/bench.json 2> gpurun_out/s12/bench.err
REPS=2 timeout -k 10 400 bash tools/ab_bench.sh prev > gpurun_out/s12/ab.txt 2>&1
