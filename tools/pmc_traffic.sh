#!/bin/bash
# HBM traffic of the bench step from PMC counters (two separate kernel-trace passes, no
# sys/runtime trace; single-stream backward: the launch configuration of the bench's profiled
# step): FETCH_SIZE and WRITE_SIZE per dispatch -> profiles JSON via
# tools/pmc_traffic.py. usage (GPU box): tools/pmc_traffic.sh OUTDIR
set -e
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-eval --no-train-py > $out/fetch.log 2>&1
SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-eval --no-train-py > $out/write.log 2>&1
