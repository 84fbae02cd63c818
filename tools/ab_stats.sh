#!/bin/bash
# Kernel-time A/B: rocprofv3 --kernel-trace --stats of bench.py (two-stream step, as timed) for
# the working-tree library and each build/<variant>; per-kernel summaries kept, databases
# deleted (gpurun copies back <= 64 MiB). usage: tools/ab_stats.sh OUTDIR variant...
set -e
out=$1; shift
mkdir -p $out
export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile > $out/$v.log 2>&1
  python3 tools/rocpd_stats.py $out/$v/run_results.db $out/$v.csv > $out/$v.txt
  python3 tools/timeline.py $out/$v/run_results.db > $out/$v.timeline.txt || true
  rm -rf $out/$v
done
