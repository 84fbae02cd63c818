#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, kernel-trace only) for one single-op bench.
# usage: tools/pmc_passes.sh OUTDIR op layer
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  REPS=3 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d $out/p$i -o run -- python3 tools/op_bench.py "$@" > $out/p$i.log 2>&1
done
