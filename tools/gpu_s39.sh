# stem BN + ReLU fused into the max-pool forward (z0 not stored): parity (steps fp32 / bf16 /
# fp16, eval, full-size chain with the stem dy and the materialised z0, train), smoke, whole-step
# A/B against build/base2 (HEAD) and kernel stats
set -e
mkdir -p gpurun_out/s39
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_eval.py tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_vistas.py > gpurun_out/s39/tests.log 2>&1
tail -n 2 gpurun_out/s39/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s39/smoke.log 2>&1
tail -n 1 gpurun_out/s39/smoke.log
for r in 1 2; do
  for v in base new; do
    unset SEG_HIP_LIB
    if [ $v = base ]; then export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/base2/libseg_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s39/ab_$v.json 2> gpurun_out/s39/ab.err
    echo "$v $(tail -n 1 gpurun_out/s39/ab_$v.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["eval"]["images_per_sec_per_gpu"], d["eval"]["miou_eval"])')" | tee -a gpurun_out/s39/ab.txt
  done
done
unset SEG_HIP_LIB
SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s39/st -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-eval --no-profile > gpurun_out/s39/st.log 2>&1
python3 tools/rocpd_stats.py gpurun_out/s39/st/run_results.db gpurun_out/s39/kernel_stats.csv > gpurun_out/s39/kernel_classes.txt
rm -rf gpurun_out/s39/st
grep -h 'maxpool\|bn_apply8_kernel<unsigned short, unsigned short, 0, 1>' gpurun_out/s39/kernel_stats.csv | cut -c1-120
