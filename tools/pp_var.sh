# time fwd of a few layers under several library variants (build/<v>/libseg_hip.so)
set -e
for l in ${LAYERS:-b4c2 b4c3}; do
 for v in default "$@"; do
  if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/iv2019-boosting-semantic-segmentation-with-weak-labels_amd/build/$v/libseg_hip.so; fi
  echo -n "$v: "; timeout -k 5 60 python tools/op_bench.py ${OP:-fwd} $l 2>&1 | grep -v amdgpu.ids
 done
done
