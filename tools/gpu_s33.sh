# residual-prefetch variant (build/respf, -DPP_RES_PF): parity of the residual dgrad launches,
# weight-gradient concurrency targets 96 / 192 workgroups (build/wg96, wg192);
# then an interleaved whole-step A/B against the in-tree library; then the whole -m gpu suite
set -e
mkdir -p gpurun_out/s33
VLIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/respf/libseg_hip.so
SEG_HIP_LIB=$VLIB timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py > gpurun_out/s33/tests_v.log 2>&1
tail -n 2 gpurun_out/s33/tests_v.log
unset SEG_HIP_LIB
for r in 1 2; do
  for v in base respf wg96 wg192; do
    unset SEG_HIP_LIB
    if [ $v != base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/$v/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s33/ab_$v.json 2> gpurun_out/s33/ab.err
    echo "$v $(tail -n 1 gpurun_out/s33/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items()})')" | tee -a gpurun_out/s33/ab.txt
  done
done
unset SEG_HIP_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s33/tests.log 2>&1
tail -n 2 gpurun_out/s33/tests.log
