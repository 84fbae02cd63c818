#!/bin/bash
# Weight-gradient A/B on one box (usage: tools/gpu_wgrad_ab.sh TAG [ENVVAR]): parity of the
# C2 layers' weight gradients, op_bench timings default vs ENVVAR=1, and PMC passes of the block4
# 3x3 weight gradient in both arms. Every step has its own time limit; the chain stops at the
# first failure.
set -e
tag=$1; var=${2:-SEG_WGRAD_RASTER}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "c2_layer" > $out/parity.log 2>&1
for arm in default $var; do
  if [ $arm = default ]; then unset $var; else export $var=1; fi
  for l in ${LAYERS:-b4c2 b3c2 b4c1 b4c3 b3c1}; do timeout -k 5 60 python3 tools/op_bench.py wgrad $l 2>&1 | grep -v amdgpu.ids >> $out/ops_$arm.txt; done
  if [ -z "$NOPMC" ]; then
    tools/pmc_passes.sh $out/pmc_$arm wgrad b4c2 && python3 tools/rocpd_pmc.py $out/pmc_$arm conv > $out/pmc_wgrad_b4c2_$arm.txt && rm -rf $out/pmc_$arm
  fi
done
unset $var
echo done
