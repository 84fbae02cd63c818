set -e
mkdir -p gpurun_out/s16
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "fused_bn or backward_layerwise" > gpurun_out/s16/tests2.log 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k "C2" >> gpurun_out/s16/tests2.log 2>&1
for r in 1 2; do
  for f in 3 0 1 2; do
    SEG_BWD_FUSE=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/s16/ab_$f.json 2> gpurun_out/s16/ab.err
    echo "fuse=$f $(tail -1 gpurun_out/s16/ab_$f.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v["ms"] for k, v in d["roofline"]["classes"].items()})')" >> gpurun_out/s16/ab.txt
  done
done
