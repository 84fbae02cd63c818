set -e
mkdir -p gpurun_out/s8
REPS=2 timeout -k 10 600 tools/ab_bench.sh r2 ntbal > gpurun_out/s8/ab_bench.txt 2>&1
OPS="fwd" LAYERS="b4c3 b3c3 b3c2 b4c2" timeout -k 10 300 tools/ab_ops.sh afold > gpurun_out/s8/ab_afold.txt 2>&1
