# round-4 session 1: the new parity tests, then the driver's bench and a two-stream trace
set -e
out=gpurun_out/r04_s1
mkdir -p $out
export TMPDIR=/tmp
echo tests; timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c_step.py tests/test_gpu_train.py tests/test_gpu_dist.py "tests/test_gpu_step.py::test_premask_matches" > $out/tests.txt 2>&1
echo bench; timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile --no-train-py > $out/tr.log 2>&1
python3 tools/timeline.py $out/tr/run_results.db > $out/timeline.txt
python3 tools/phases.py $out/tr/run_results.db > $out/phases.txt
echo done
