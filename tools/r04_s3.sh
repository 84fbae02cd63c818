# round-4 session 3: Infinity-Cache streaming probe, per-layer kernel table, two-stream trace
# of the bench step (no train.py leg)
set -e
out=gpurun_out/r04_s3
mkdir -p $out
export TMPDIR=/tmp
echo mall; timeout -k 10 120 ./tools/mall_probe.bin > $out/mall.txt 2>&1
echo layers; timeout -k 10 300 python3 tools/layer_report.py > $out/layers.txt 2>&1; cp gpurun_out/layers.csv $out/ || true
echo trace2; timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile --no-train-py > $out/tr2.log 2>&1
echo done
