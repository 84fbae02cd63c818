# small-channel 3x3 patch kernel: op parity (small + C2 shapes), step layerwise, A/B
set -e
mkdir -p gpurun_out/s23
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "fwd or dgrad" > gpurun_out/s23/tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "block1_conv2_c64 or block2_conv2_c128" >> gpurun_out/s23/tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "bf16_layerwise or backward_layerwise or deterministic" >> gpurun_out/s23/tests.log 2>&1
for r in 1 2; do
  for v in 1 0; do
    SEG_PATCH=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/s23/ab_$v.json 2> gpurun_out/s23/ab.err
    echo "patch=$v $(tail -1 gpurun_out/s23/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items() if "conv" in k})')" >> gpurun_out/s23/ab.txt
  done
done
