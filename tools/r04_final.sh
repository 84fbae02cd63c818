# round-4 final check (GPU box): the whole GPU suite and smoke() at HEAD, as the driver runs them
set -e
out=gpurun_out/${1:-r04_final}
mkdir -p $out
echo suite; timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/suite.txt 2>&1
echo smoke; timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
echo done
