# row-segment 3x3 mode (ST == 3) + residual prefetch variant: parity first (full-size C2 layers
# and step chain exercise the row-segment launches), then op timings and an interleaved A/B
set -e
mkdir -p gpurun_out/s32
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "conv_c2_layer" > gpurun_out/s32/tests_layers.log 2>&1
tail -2 gpurun_out/s32/tests_layers.log
for v in 0 1; do
  for op in fwd dgrad; do
    for l in b4c2 b3c2; do
      SEG_ROWSEG=$v timeout -k 10 60 python tools/op_bench.py $op $l >> gpurun_out/s32/ops_$v.txt 2>&1
    done
  done
done
tail -4 gpurun_out/s32/ops_0.txt gpurun_out/s32/ops_1.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s32/tests.log 2>&1
tail -2 gpurun_out/s32/tests.log
VLIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/respf/libseg_hip.so
SEG_HIP_LIB=$VLIB timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fullsize.py > gpurun_out/s32/tests_v.log 2>&1
tail -2 gpurun_out/s32/tests_v.log
for r in 1 2; do
  for v in base rowseg respf; do
    unset SEG_HIP_LIB SEG_ROWSEG
    if [ $v = base ]; then export SEG_ROWSEG=0; fi
    if [ $v = respf ]; then export SEG_HIP_LIB=$VLIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s32/ab_$v.json 2> gpurun_out/s32/ab.err
    echo "$v $(tail -1 gpurun_out/s32/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items()})')" | tee -a gpurun_out/s32/ab.txt
  done
done
