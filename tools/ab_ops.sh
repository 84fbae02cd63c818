#!/bin/bash
# A/B single-op timings: default library vs build/<variant>/libseg_hip.so for each variant given
# OPS / LAYERS env override the op and layer lists
set -e
OPS=${OPS:-"fwd dgrad wgrad"}
LAYERS=${LAYERS:-"b4c2 b4c3 b4c1 b3c2"}
for v in default "$@"; do
  if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  echo "== $v"
  for op in $OPS; do
    for l in $LAYERS; do timeout -k 5 60 python tools/op_bench.py $op $l 2>&1 | grep -v amdgpu.ids; done
  done
done
