# BN-backward reduce with one accumulator set (131 instead of 191 VGPRs: 3 waves per SIMD) and
# row-block cap 1024 (in-tree) or 768 (build/rb768) vs HEAD (build/base4): parity, step A/B
set -e
mkdir -p gpurun_out/s41
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_dist.py > gpurun_out/s41/tests.log 2>&1
tail -n 2 gpurun_out/s41/tests.log
for r in 1 2; do
  for v in base4 new rb768; do
    unset SEG_HIP_LIB
    if [ $v != new ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/$v/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s41/ab_$v.json 2> gpurun_out/s41/ab.err
    echo "$v $(tail -n 1 gpurun_out/s41/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:21]: v["ms"] for k, v in d["roofline"]["classes"].items() if "bn" in k})')" | tee -a gpurun_out/s41/ab.txt
  done
done
