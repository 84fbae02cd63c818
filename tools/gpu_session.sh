set -e
out=gpurun_out/s12
mkdir -p $out
export TMPDIR=/tmp
echo parity; SEG_WGRAD_LATE=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_train.py tests/test_gpu_buckets.py > $out/parity.txt 2>&1
echo ab
for r in 1 2 3; do for v in 0 1; do
  if [ $v = 0 ]; then unset SEG_WGRAD_LATE; else export SEG_WGRAD_LATE=1; fi
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval > $out/b.log 2>&1
  echo "late=$v $(tail -1 $out/b.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done; done > $out/ab.txt
echo done
