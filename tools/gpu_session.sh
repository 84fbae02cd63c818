# One GPU-box pass for the round's final record: the driver's GPU suite, smoke and the
# driver's bench command (rocprofv3 / PMC passes: tools/measure_round.sh). Every step has its
# own time limit and the chain stops at the first failure.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_session.sh'
set -e
out=gpurun_out/final
mkdir -p $out
export TMPDIR=/tmp
echo suite; timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $out/suite.txt 2>&1
echo smoke; timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo bench; timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
echo done
