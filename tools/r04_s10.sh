# round-4 session 10: weight-gradient slab stores as buffer stores with SGPR row offsets (pp, v2,
# patch kernels) + the NT statistics butterfly over 8 values (no per-step s_nop) vs the
# previous build, + the loss head's fixed-bound x-reduction: parity, single-op timing, step A/B
set -e
out=gpurun_out/r04_s10
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py tests/test_gpu_vistas.py tests/test_gpu_eval.py > $out/tests.txt 2>&1
echo ops
for v in default prev default prev; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "wgrad b3c1" "wgrad b3c3" "wgrad b4c1" "wgrad b4c3" "wgrad b4c2" "wgrad b2c1" "wgrad b1c2" "fwd b4c3" "fwd b3c3"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/ops.txt; done
done
unset SEG_HIP_LIB
echo loss
for v in default prev default prev; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  echo "$v $(timeout -k 10 120 python3 tools/loss_bench.py 2>&1 | tail -n 1)" >> $out/loss.txt
done
unset SEG_HIP_LIB
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh prev > $out/ab_bench.txt 2>&1
echo done
