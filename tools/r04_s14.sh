# round-4 session 14: counter passes on the dilated 3x3 NT launches (block4 rate 4 forward /
# data gradient, block3 rate 2 forward) at HEAD, and per-segment s_memtime stamps of the NT main
# loop (NT_DBG_TIMING build): where the main loop loses its MFMA time
set -e
out=gpurun_out/r04_s14
mkdir -p $out
export TMPDIR=/tmp
for spec in "fwd b4c2" "dgrad b4c2" "fwd b3c2"; do
  set -- $spec
  echo "pmc $1 $2" && tools/pmc_passes.sh $out/pmc_$1_$2 $1 $2 && python3 tools/rocpd_pmc.py $out/pmc_$1_$2 conv > $out/pmc_$1_$2.txt && rm -rf $out/pmc_$1_$2
done
echo done1
echo stamps
export SEG_HIP_LIB=$PWD/ab/nttim/libseg_hip.so
for spec in "fwd b4c2" "dgrad b4c2" "fwd b4c3" "fwd b3c3" "dgrad b4c3"; do echo "== $spec" >> $out/nt_stamps.txt; timeout -k 10 120 python3 tools/nt_timing.py $spec >> $out/nt_stamps.txt 2>&1; done
unset SEG_HIP_LIB
echo done2
