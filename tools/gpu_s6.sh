# parity of the NT kernel changes, per-tile timing, whole-step A/B against the HEAD build
set -e
mkdir -p gpurun_out/s6
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py > gpurun_out/s6/tests.log 2>&1
for spec in "fwd b3c3" "fwd b4c3" "dgrad b3c1" "fwd head1"; do
  set -- $spec
  echo "== $1 $2" >> gpurun_out/s6/timing.txt
  timeout -k 10 60 python tools/op_bench.py $1 $2 >> gpurun_out/s6/timing.txt 2>&1
  SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/tim/libseg_hip.so timeout -k 10 60 python tools/pp_timing.py $1 $2 >> gpurun_out/s6/timing.txt 2>&1
done
REPS=3 timeout -k 10 600 bash tools/ab_bench.sh base > gpurun_out/s6/ab.txt 2>&1
