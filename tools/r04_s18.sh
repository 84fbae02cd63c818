# round-4 session 18: NT main loop with a static s_setprio 1 for the lagging wave row (default)
# vs per-MFMA-segment priority flips (flips, round 3): parity, single-op timing, step A/B
set -e
out=gpurun_out/r04_s18
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_step.py > $out/tests.txt 2>&1
echo ops
for v in default flips default flips; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "fwd b4c2" "dgrad b4c2" "fwd b4c3" "fwd b3c3" "dgrad b4c3" "fwd b4c1"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/ops.txt; done
done
unset SEG_HIP_LIB
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh flips > $out/ab_bench.txt 2>&1
echo done
