set -e
out=gpurun_out/r02v14
mkdir -p $out
export TMPDIR=/tmp
for spec in "wgrad b4c2" "fwd b4c2" "dgrad b4c2" "wgrad b4c1" "fwd b4c3" "wgrad b3c1"; do
  set -- $spec
  echo "pmc $1 $2" && tools/pmc_passes.sh $out/pmc_$1_$2 $1 $2 && python3 tools/rocpd_pmc.py $out/pmc_$1_$2 conv > $out/pmc_$1_$2.txt && rm -rf $out/pmc_$1_$2
done
