# the whole -m gpu suite (round-end check), one process, per-test timeouts
set -e
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/full/tests.log 2>&1
