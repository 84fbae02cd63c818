# wgrad epilogue: LDS-staged coalesced slab stores vs the scattered stores vs none (timing only)
set -e
mkdir -p gpurun_out/s15
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py -k "wgrad or step" > gpurun_out/s15/tests.log 2>&1
B=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build
for l in b3c1 b3c3 b4c1 b4c2 b3c2 head1; do
  timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s15/ops.txt 2>&1
  SEG_HIP_LIB=$B/unstaged/libseg_hip.so timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s15/ops_unstaged.txt 2>&1
  SEG_HIP_LIB=$B/nostore/libseg_hip.so timeout -k 10 60 python tools/op_bench.py wgrad $l >> gpurun_out/s15/ops_nostore.txt 2>&1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-eval > gpurun_out/s15/bench.json 2> gpurun_out/s15/bench.err
REPS=2 timeout -k 10 400 bash tools/ab_bench.sh unstaged > gpurun_out/s15/ab.txt 2>&1
