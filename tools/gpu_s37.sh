# max-pool backward fused into the stem's BN backward (pooled gather in the reduce / apply):
# parity (full-size C2 chain incl. the stem dy check, bf16/fp16 backward layerwise, steps,
# train, determinism), whole-step A/B against build/base1 (HEAD), kernel trace of the tail
set -e
mkdir -p gpurun_out/s37
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -k "defer or fullsize or train or two_step or deterministic or backward_layerwise" > gpurun_out/s37/tests.log 2>&1
tail -n 2 gpurun_out/s37/tests.log
for r in 1 2; do
  for v in base new; do
    unset SEG_HIP_LIB
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base1/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s37/ab_$v.json 2> gpurun_out/s37/ab.err
    echo "$v $(tail -n 1 gpurun_out/s37/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/s37/ab.txt
  done
done
unset SEG_HIP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s37/tr -o run -- python3 bench.py --steps 4 --warmup 2 --no-profile --no-cpu-baseline --no-eval > gpurun_out/s37/tr.log 2>&1
python3 tools/timeline.py gpurun_out/s37/tr/run_results.db 30 > gpurun_out/s37/timeline.txt 2>&1
rm -rf gpurun_out/s37/tr
