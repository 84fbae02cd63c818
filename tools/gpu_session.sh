set -e
out=gpurun_out/s7
mkdir -p $out
export TMPDIR=/tmp
echo suite; timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $out/suite.txt 2>&1
echo done
