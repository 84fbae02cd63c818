# round-4 session 12: NT epilogue merges its two wave rows' BN partials (256-row partials: half
# the bn_stats_final reads) vs the previous build: parity, op + finalize timing, step A/B
set -e
out=gpurun_out/r04_s12
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py tests/test_gpu_train.py > $out/tests.txt 2>&1
echo ops
for v in default prev default prev; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "fwd b4c3" "fwd b3c3" "fwd b4c2"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/ops.txt; done
done
unset SEG_HIP_LIB
echo layers; timeout -k 10 300 python3 tools/layer_report.py > $out/layers.txt 2>&1
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh prev > $out/ab_bench.txt 2>&1
echo done
