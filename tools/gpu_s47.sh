# N-concatenated projection-unit forward (conv1 + shortcut in one ping-pong launch, ST == 5)
# one ping-pong GEMM): parity (conv ops, full-size chains that check the unit-input gradient,
# steps, train), op timings of the plain 1x1 launches (regression check), step A/B vs build/base7
set -e
mkdir -p gpurun_out/s47
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_eval.py > gpurun_out/s47/tests.log 2>&1
tail -n 2 gpurun_out/s47/tests.log
for v in base new; do
  for op in "fwd b4c3" "dgrad b3c1" "fwd b3c3"; do
    set -- $op
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base7/libseg_hip.so; else unset SEG_HIP_LIB; fi
    timeout -k 10 60 python tools/op_bench.py $1 $2 2>/dev/null | grep -v amdgpu >> gpurun_out/s47/ops_$v.txt
  done
done
unset SEG_HIP_LIB
cat gpurun_out/s47/ops_base.txt gpurun_out/s47/ops_new.txt
for r in 1 2; do
  for v in base new; do
    unset SEG_HIP_LIB
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base7/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s47/ab_$v.json 2> gpurun_out/s47/ab.err
    echo "$v $(tail -n 1 gpurun_out/s47/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items() if "conv" in k})')" | tee -a gpurun_out/s47/ab.txt
  done
done
