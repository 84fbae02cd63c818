# round-4 session 13: dense 1x1 residual data gradients on the persistent loop (PERSIST 2) with the
# consumer ReLU bits staged in LDS by DMA (res0 = the LDS bits, one tile per workgroup; prev =
# HEAD): parity, per-layer table (data-gradient class), step A/B
set -e
out=gpurun_out/r04_s13
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_vistas.py > $out/tests.txt 2>&1
echo layers
for v in default res0 prev; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  timeout -k 10 300 python3 tools/layer_report.py > $out/layers_$v.txt 2>&1; cp gpurun_out/layers.csv $out/layers_$v.csv
done
unset SEG_HIP_LIB
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh res0 prev > $out/ab_bench.txt 2>&1
echo done
