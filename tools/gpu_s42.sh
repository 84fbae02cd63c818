# dual BN backward for projection units (conv3 + shortcut BN share dz / bits: one reduce, one
# apply): parity (steps fp32/bf16/fp16, full-size chains incl. the shortcut dy checks, dist,
# train, GN), whole-step A/B against build/base5 (HEAD)
set -e
mkdir -p gpurun_out/s42
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_train.py tests/test_gpu_vistas.py > gpurun_out/s42/tests.log 2>&1
tail -n 2 gpurun_out/s42/tests.log
for r in 1 2; do
  for v in base new; do
    unset SEG_HIP_LIB
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base5/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s42/ab_$v.json 2> gpurun_out/s42/ab.err
    echo "$v $(tail -n 1 gpurun_out/s42/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:21]: v["ms"] for k, v in d["roofline"]["classes"].items() if "bn" in k})')" | tee -a gpurun_out/s42/ab.txt
  done
done
