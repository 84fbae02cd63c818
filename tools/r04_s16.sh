# round-4 session 16: BN-backward row-block cap for the C <= 256 layers (1024 default vs 512 /
# 2048): per-layer BN classes, step A/B; parity on the variant with the most partials
set -e
out=gpurun_out/r04_s16
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; SEG_HIP_LIB=$PWD/ab/rb2048/libseg_hip.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_fullsize.py > $out/tests.txt 2>&1
echo layers
for v in default rb512 rb2048; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  timeout -k 10 300 python3 tools/layer_report.py > $out/layers_$v.txt 2>&1
done
unset SEG_HIP_LIB
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh rb512 rb2048 > $out/ab_bench.txt 2>&1
echo done
