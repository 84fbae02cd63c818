# stem patch kernel: step parity (layerwise incl. the stem forward), full-size C2 chain, A/B
set -e
mkdir -p gpurun_out/s28
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "layerwise or deterministic or fp32" > gpurun_out/s28/tests.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k "C2" >> gpurun_out/s28/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k "fwd" >> gpurun_out/s28/tests.log 2>&1
for r in 1 2; do
  for v in 1 0; do
    SEG_PATCH=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/s28/ab_$v.json 2> gpurun_out/s28/ab.err
    echo "patch=$v $(tail -1 gpurun_out/s28/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items() if "conv" in k})')" >> gpurun_out/s28/ab.txt
  done
done
SEG_PATCH=1 timeout -k 10 200 python tools/step_report.py C2 > gpurun_out/s28/rep.txt 2>&1
