# round-4 session 6: XCD-aligned weight-gradient splits + channel-group tile order.
# parity (conv / full-size / step), single-op timing, PMC passes on block4 3x3 wgrad at the
# side-stream split counts; epilogue pack fix (v_cvt_pk both halves) vs alignonly; (HEAD order at 3 splits vs the new order at 4) and alone, step A/B.
set -e
out=gpurun_out/r04_s6
mkdir -p $out
export TMPDIR=/tmp
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py > $out/tests.txt 2>&1
echo ops
for cfg in "head 3" "head 4" "new 3" "new 4" "head 0" "new 0"; do
  set -- $cfg
  if [ $1 = head ]; then export SEG_HIP_LIB=$PWD/ab/head/libseg_hip.so; else unset SEG_HIP_LIB; fi
  if [ $2 = 0 ]; then unset SPLITS; else export SPLITS=$2; fi
  echo "$cfg $(timeout -k 10 120 python3 tools/op_bench.py wgrad b4c2)" >> $out/ops.txt
  echo "$cfg $(timeout -k 10 120 python3 tools/op_bench.py wgrad b3c2)" >> $out/ops.txt
done
for cfg in "head 3" "new 4" "new 0" "head 0"; do
  set -- $cfg
  if [ $1 = head ]; then export SEG_HIP_LIB=$PWD/ab/head/libseg_hip.so; else unset SEG_HIP_LIB; fi
  if [ $2 = 0 ]; then unset SPLITS; else export SPLITS=$2; fi
  d=$out/pmc_$1_s$2; mkdir -p $d
  echo "pmc $cfg"; tools/pmc_passes.sh $d/raw wgrad b4c2 && python3 tools/rocpd_pmc.py $d/raw conv > $d/pmc_wgrad_b4c2.txt && rm -rf $d/raw
  python3 tools/pmc_summary.py $d $d/summary.json > /dev/null || true
done
unset SEG_HIP_LIB SPLITS
echo packops
for v in default alignonly; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "fwd b4c3" "dgrad b4c1" "fwd b3c3" "fwd b4c1"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/packops.txt; done
done
unset SEG_HIP_LIB
echo abbench; REPS=2 timeout -k 10 900 bash tools/ab_bench.sh head noalign alignonly > $out/ab_bench.txt 2>&1
echo done
