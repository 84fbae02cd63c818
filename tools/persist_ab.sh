# A/B of the persistent NT tile loop: SEG_NT_PERSIST=0 (one tile per workgroup) vs 1
for v in 0 1; do for op in ${OPS:-fwd dgrad}; do for l in ${LAYERS:-b4c2 b3c2 b4c3 b4c1 b3c1 b3c3 head1}; do
  echo -n "persist=$v "; SEG_NT_PERSIST=$v timeout -k 5 60 python tools/op_bench.py $op $l 2>&1 | grep -v amdgpu.ids
done; done; done
