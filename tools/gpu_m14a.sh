set -e
tag=${TAG:-r02v14}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
echo "bench" && timeout -k 10 400 python3 -u bench.py > $out/bench.json 2> $out/bench.err
echo "stats" && SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval > $out/stats.log 2>&1
python3 tools/rocpd_stats.py $out/stats/run_results.db $out/kernel_stats.csv > $out/kernel_classes.txt
rm -rf $out/stats
echo "traffic" && tools/pmc_traffic.sh $out/traffic && python3 tools/pmc_traffic.py $out/traffic $out/pmc_traffic.json && rm -rf $out/traffic/fetch $out/traffic/write
