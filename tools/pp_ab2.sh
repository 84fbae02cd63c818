# A/B of the NT conv main loops (SEG_NT_PP=0: v2, 1: ping-pong) on C2 layer shapes
for v in 0 1; do for op in ${OPS:-fwd dgrad}; do for l in ${LAYERS:-b4c2 b3c2 b4c3 b4c1}; do
  echo -n "pp=$v "; SEG_NT_PP=$v timeout -k 5 60 python tools/op_bench.py $op $l 2>&1 | grep -v amdgpu.ids
done; done; done
