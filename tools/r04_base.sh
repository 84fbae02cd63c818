set -e
out=gpurun_out/r04_base
mkdir -p $out
export TMPDIR=/tmp
echo bench; timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile > $out/tr.log 2>&1
python3 tools/timeline.py $out/tr/run_results.db > $out/timeline.txt
python3 tools/phases.py $out/tr/run_results.db > $out/phases.txt
ls -la $out/tr
echo done
