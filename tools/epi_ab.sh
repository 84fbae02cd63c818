# epilogue cost of the NT kernel on short-K layers: default vs no global stores vs one staged
# pass (build/nostore, build/nostage), and without the fused BN statistics (NOSTATS=1)
set -e
for l in ${LAYERS:-b3c3 b4c3 head1 b3c1 b4c2}; do
 for v in default nostore nostage; do
  if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/$v/libseg_hip.so; fi
  echo -n "$v: "; timeout -k 5 60 python tools/op_bench.py ${OP:-fwd} $l 2>&1 | grep -v amdgpu.ids
 done
 unset SEG_HIP_LIB
 echo -n "nostats: "; NOSTATS=1 timeout -k 5 60 python tools/op_bench.py ${OP:-fwd} $l 2>&1 | grep -v amdgpu.ids
done
