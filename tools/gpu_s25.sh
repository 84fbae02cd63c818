# patch kernel: two workgroups per CU for the one-chunk 64-channel layers; op timings + parity
set -e
mkdir -p gpurun_out/s25
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "fwd or dgrad" > gpurun_out/s25/tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "block1_conv2_c64 or block2_conv2_c128" >> gpurun_out/s25/tests.log 2>&1
for v in 1 2; do
  for op in fwd dgrad; do
    for l in b1c2 b2c2; do
      SEG_PATCH=$v timeout -k 10 60 python tools/op_bench.py $op $l >> gpurun_out/s25/ops_$v.txt 2>&1
    done
  done
done
