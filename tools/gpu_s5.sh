# per-tile phase timing of the persistent NT kernel on short-K 1x1 layers vs the dilated 3x3
set -e
mkdir -p gpurun_out/s5
for spec in "fwd b3c3" "fwd b4c3" "fwd head1" "dgrad b3c1" "dgrad b4c1" "fwd b4c2" "fwd b3c2"; do
  set -- $spec
  echo "== $1 $2" >> gpurun_out/s5/timing.txt
  timeout -k 10 60 python tools/op_bench.py $1 $2 >> gpurun_out/s5/timing.txt 2>&1
  SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/tim/libseg_hip.so timeout -k 10 60 python tools/pp_timing.py $1 $2 >> gpurun_out/s5/timing.txt 2>&1
done
