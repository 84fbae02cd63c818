# ping-pong NT main loop: 2 phases per K-tile (4 barriers) vs 4 phases (8 barriers)
set -e
mkdir -p gpurun_out/s29
SEG_PP_PH2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "fwd or dgrad" > gpurun_out/s29/tests.log 2>&1
SEG_PP_PH2=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "block4 or block3 or aspp" >> gpurun_out/s29/tests.log 2>&1
for v in 0 1; do
  for op in fwd dgrad; do
    for l in b4c2 b4c3 b3c3 b3c2; do
      SEG_PP_PH2=$v timeout -k 10 60 python tools/op_bench.py $op $l >> gpurun_out/s29/ops_$v.txt 2>&1
    done
  done
done
for r in 1 2; do
  for v in 0 1; do
    SEG_PP_PH2=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval > gpurun_out/s29/ab_$v.json 2> gpurun_out/s29/ab.err
    echo "ph2=$v $(tail -1 gpurun_out/s29/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], {k[:24]: v["ms"] for k, v in d["roofline"]["classes"].items() if "conv" in k})')" >> gpurun_out/s29/ab.txt
  done
done
