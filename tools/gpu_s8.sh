# v2 weight-gradient tile / split sweep on the small-channel layers vs the default choice
set -e
mkdir -p gpurun_out/s8
for l in b1c2 b1c3 b2c2 b2c1 b3c2; do timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s8/default.txt 2>&1; done
timeout -k 10 400 python -u tools/wgrad_sweep.py b1c2 b2c2 b1c3 b1c1 b2c1 b2c3 > gpurun_out/s8/sweep.txt 2>&1
