# round-5 session 5 (temporary): the GPU suite at HEAD, smoke, PMC traffic of the bench step,
# PMC counters on the short-K layers
out=gpurun_out/r05_s5; mkdir -p $out
export TMPDIR=/tmp
bash tools/session.sh r05_s5 suite || echo "suite failed (continuing)"
bash tools/session.sh r05_s5 smoke traffic pmc=fwd:b4c3 pmc=dgrad:b4c1 pmc=wgrad:b4c2
echo done
