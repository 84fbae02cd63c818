#!/bin/bash
# One GPU-box measurement pass for the round's profiles (usage: tools/measure_round.sh TAG):
# bench line, rocprofv3 kernel stats of the bench (single-stream backward so per-kernel times
# are kernel-alone, matching the bench's profiled step), PMC HBM traffic of the bench, and PMC
# MFMA / LDS / cache counter passes on the dominant layer classes. Every step has its own time
# limit and the chain stops at the first failure.
set -e
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
echo "bench" && timeout -k 10 400 python3 -u bench.py > $out/bench.json 2> $out/bench.err
echo "stats" && SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval > $out/stats.log 2>&1
python3 tools/rocpd_stats.py $out/stats/run_results.db $out/kernel_stats.csv > $out/kernel_classes.txt
rm -rf $out/stats   # rocpd databases: summarised above; gpurun copies back at most 64 MiB
echo "traffic" && tools/pmc_traffic.sh $out/traffic && python3 tools/pmc_traffic.py $out/traffic $out/pmc_traffic.json && rm -rf $out/traffic/fetch $out/traffic/write
for spec in "wgrad b4c2" "fwd b4c2" "dgrad b4c2" "wgrad b4c1" "fwd b4c3" "wgrad b3c1"; do
  set -- $spec
  echo "pmc $1 $2" && tools/pmc_passes.sh $out/pmc_$1_$2 $1 $2 && python3 tools/rocpd_pmc.py $out/pmc_$1_$2 conv > $out/pmc_$1_$2.txt && rm -rf $out/pmc_$1_$2
done
echo done
