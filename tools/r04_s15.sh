# round-4 session 15: weight gradient with B1's fragment reads under the first quadrant's MFMAs
# and B1's DMA in M1 (default) vs round 3's schedule (b1l0): parity,
# segment stamps (WG_DBG_TIMING builds), single-op timing, step A/B
set -e
out=gpurun_out/r04_s15
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py > $out/tests.txt 2>&1
echo stamps
for v in wgtim wgtim0; do
  export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so
  for spec in "wgrad b4c2" "wgrad b4c1" "wgrad b3c1"; do echo "== $v $spec" >> $out/stamps.txt; timeout -k 10 120 python3 tools/wg_timing.py $spec >> $out/stamps.txt 2>&1; done
done
echo ops
for v in default b1l0 default b1l0; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "wgrad b4c2" "wgrad b4c1" "wgrad b4c3" "wgrad b3c1" "wgrad b3c3"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/ops.txt; done
  echo "$v SPLITS=4 $(SPLITS=4 timeout -k 10 120 python3 tools/op_bench.py wgrad b4c2)" >> $out/ops.txt
done
unset SEG_HIP_LIB
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh b1l0 > $out/ab_bench.txt 2>&1
echo done
