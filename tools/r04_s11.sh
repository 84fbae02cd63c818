# round-4 session 11: final-record pass at HEAD (GPU suite, smoke, the driver's bench command) and
# the R101 bench lines (C3 / C4 bf16, C5 fp16)
set -e
out=gpurun_out/r04_s11
mkdir -p $out
export TMPDIR=/tmp
echo suite; timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $out/suite.txt 2>&1
echo smoke; timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo bench; timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
for c in C3 C4 C5; do echo "bench $c"; timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-train-py --no-eval > $out/bench_$c.json 2> $out/bench_$c.err; done
echo done
