set -e
out=gpurun_out/s13
mkdir -p $out
export TMPDIR=/tmp
echo parity; timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "wgrad" > $out/parity.txt 2>&1
echo ops; OPS="wgrad" LAYERS="b1c2 b2c2" timeout -k 10 300 tools/ab_ops.sh base > $out/ops.txt 2>&1
echo full; timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py > $out/full.txt 2>&1
echo ab; timeout -k 10 600 tools/ab_bench.sh base > $out/ab.txt 2>&1
echo done
