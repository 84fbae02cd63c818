# ping-pong weight-gradient split sweep (kernel alone) + default choices; bench with attainable fractions
set -e
mkdir -p gpurun_out/s11
for l in b3c1 b3c3 b4c1 b4c3 b4c2 b3c2 head1; do timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s11/default.txt 2>&1; done
PP_ONLY=1 timeout -k 10 500 python -u tools/wgrad_sweep.py b3c1 b3c3 b4c1 b4c3 b4c2 b3c2 head1 > gpurun_out/s11/sweep.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval > gpurun_out/s11/bench.json 2> gpurun_out/s11/bench.err
