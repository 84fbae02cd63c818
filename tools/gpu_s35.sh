# max-pool backward with every window's argmax / gradient loaded up front: parity (full-size C2
# chain incl. the max-pool check, bf16 backward layerwise), step A/B against build/base0, and a
# kernel-stats pass for the max-pool backward time
set -e
mkdir -p gpurun_out/s35
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_step.py -k "fullsize or backward_layerwise or train_step_fp32" > gpurun_out/s35/tests.log 2>&1
tail -n 2 gpurun_out/s35/tests.log
for r in 1 2; do
  for v in base new; do
    unset SEG_HIP_LIB
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base0/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval > gpurun_out/s35/ab_$v.json 2> gpurun_out/s35/ab.err
    echo "$v $(tail -n 1 gpurun_out/s35/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/s35/ab.txt
  done
done
unset SEG_HIP_LIB
for v in base new; do
  if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base0/libseg_hip.so; else unset SEG_HIP_LIB; fi
  SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s35/st_$v -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-eval --no-profile > gpurun_out/s35/st_$v.log 2>&1
  python3 tools/rocpd_stats.py gpurun_out/s35/st_$v/run_results.db gpurun_out/s35/kernel_stats_$v.csv > gpurun_out/s35/kernel_classes_$v.txt
  rm -rf gpurun_out/s35/st_$v
done
grep -h maxpool gpurun_out/s35/kernel_classes_*.txt || true
