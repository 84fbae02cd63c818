# parity of the conv kernel changes, single-op timings, whole-step A/B against build/prev
set -e
mkdir -p gpurun_out/s7
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py > gpurun_out/s7/tests.log 2>&1
for spec in "fwd b3c3" "fwd head1" "fwd b2c1" "fwd b1c2" "dgrad b2c1" "fwd b2c2"; do
  set -- $spec
  timeout -k 10 60 python tools/op_bench.py $1 $2 >> gpurun_out/s7/ops_new.txt 2>&1
  SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/prev/libseg_hip.so timeout -k 10 60 python tools/op_bench.py $1 $2 >> gpurun_out/s7/ops_prev.txt 2>&1
done
REPS=3 timeout -k 10 600 bash tools/ab_bench.sh prev > gpurun_out/s7/ab.txt 2>&1
