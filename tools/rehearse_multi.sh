#!/bin/bash
# One-GPU rehearsal of bench.py's N > 1 path (barriers, max-over-ranks timing, bucketed
# all-reduce on the comm stream, the `comm` fields): N ranks share cuda:0 over gloo, since RCCL
# does not put two ranks on one device. The driver's SCALE run uses one GPU per rank over RCCL.
set -o pipefail
out=gpurun_out/rehearse_multi
mkdir -p $out
for n in 2 4; do
  echo "rehearsal n=$n" | tee -a $out/progress.txt
  SEG_BENCH_BACKEND=gloo timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29531 + n)) \
    bench.py --gpus $n --steps 4 --warmup 2 --no-eval > $out/n$n.log 2>&1 || { echo "n=$n failed rc=$?"; exit 1; }
  grep '^{"metric"' $out/n$n.log > $out/n$n.json
done
echo done
