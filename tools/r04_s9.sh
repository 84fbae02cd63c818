# round-4 session 9: NT staging writes as single ds_write_b64 (no write2st64 pairs on the same
# banks) vs the previous build: parity, counters on fwd b4c3, single-op timing, step A/B
set -e
out=gpurun_out/r04_s9
mkdir -p $out
export TMPDIR=/tmp
md5sum iv2019-boosting-semantic-segmentation-with-weak-labels_amd/libseg_hip.so ab/*/libseg_hip.so > $out/md5.txt
echo tests; timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_fullsize.py tests/test_gpu_step.py > $out/tests.txt 2>&1
echo ops
for v in default prev default prev; do
  if [ $v = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  for spec in "fwd b4c3" "fwd b3c3" "dgrad b4c3" "fwd b4c2"; do echo "$v $(timeout -k 10 120 python3 tools/op_bench.py $spec)" >> $out/ops.txt; done
done
unset SEG_HIP_LIB
echo pmc; tools/pmc_passes.sh $out/raw fwd b4c3 && python3 tools/rocpd_pmc.py $out/raw conv > $out/pmc_fwd_b4c3.txt && rm -rf $out/raw
python3 tools/pmc_summary.py $out $out/pmc_summary.json > /dev/null || true
echo abbench; REPS=3 timeout -k 10 900 bash tools/ab_bench.sh prev > $out/ab_bench.txt 2>&1
echo done
