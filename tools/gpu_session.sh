set -e
mkdir -p gpurun_out/s9
OPS="fwd" LAYERS="b4c3 b3c3 b3c2 b4c2 b4c1" timeout -k 10 300 tools/ab_ops.sh afold > gpurun_out/s9/ab_afold.txt 2>&1
