#!/bin/bash
# A/B of whole-step throughput on one box: the working-tree library against each
# build/<variant>/libseg_hip.so given, interleaved, REPS rounds (bench.py --steps 10)
REPS=${REPS:-2}
for r in $(seq $REPS); do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train-py --no-eval > gpurun_out/ab.log 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
