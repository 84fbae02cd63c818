# round-4 session 17: BN-backward row-block caps: C <= 256 at 512 (new default) vs 256 (s256),
# vs 1024 (s1024, round 3), and every layer at 512 (all512): parity, step A/B
set -e
out=gpurun_out/r04_s17
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_train.py > $out/tests.txt 2>&1
echo abbench; REPS=3 timeout -k 10 1000 bash tools/ab_bench.sh s256 all512 s1024 > $out/ab_bench.txt 2>&1
echo done
