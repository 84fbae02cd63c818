#!/bin/bash
# Interleaved whole-step A/B (bench.py, no CPU baseline / eval / train.py legs) of the working-tree
# library against ab/<variant>/libseg_hip.so: img/s and every profiled class's kernel-alone ms
# per step (the bench's own single-stream profiled step), REPS rounds.
#   bash tools/ab_classes.sh OUTFILE VARIANT...
out=$1; shift
for r in $(seq ${REPS:-3}); do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-train-py > gpurun_out/abc.log 2>&1 || exit 1
    tail -1 gpurun_out/abc.log | python3 tools/ab_line.py "$v" >> "$out"
  done
done
