set -e
for l in b4c2 b4c3 b4c1 b3c2 b3c1 b3c3 head1; do
 for op in fwd dgrad; do
  for v in 0 1; do
   echo -n "pp=$v "; SEG_NT_PP=$v timeout -k 5 60 python tools/op_bench.py $op $l 2>&1 | grep -v amdgpu.ids
  done
 done
done
