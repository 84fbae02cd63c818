# round-4 session 5: Infinity-Cache probe, per-layer kernel table, BN-backward channel-slab and
# co-residency A/B (gradient check + interleaved step throughput)
set -e
out=gpurun_out/r04_s5
mkdir -p $out
export TMPDIR=/tmp
echo mall; timeout -k 10 120 ./tools/mall_probe.bin > $out/mall.txt 2>&1
echo layers; timeout -k 10 300 python3 tools/layer_report.py > $out/layers.txt 2>&1; cp gpurun_out/layers.csv $out/ || true
echo abgrads; timeout -k 10 300 python3 tools/ab_grads.py ab/slab128/libseg_hip.so > $out/ab_grads.txt 2>&1
echo abbench; REPS=2 timeout -k 10 900 bash tools/ab_bench.sh slab64 slab128 slab192 bwdu1 > $out/ab_bench.txt 2>&1
echo done
