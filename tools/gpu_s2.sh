# round-2 check: FoV / slack / reverse-apply parity, then a whole-step A/B of the variants
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_conv.py tests/test_gpu_step.py > gpurun_out/s2/tests.log 2>&1
REPS=2 timeout -k 10 600 bash tools/ab_bench.sh noslack norev none > gpurun_out/s2/ab.txt 2>&1
