# round-4 session 2: single-stream trace (co-running analysis against r04_s1's two-stream
# trace) and the PMC step ledger
set -e
out=gpurun_out/r04_s2
mkdir -p $out
export TMPDIR=/tmp
echo trace1; SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile --no-train-py > $out/tr1.log 2>&1
echo traffic; tools/pmc_traffic.sh $out/traffic && python3 tools/pmc_traffic.py $out/traffic $out/pmc_traffic.json > /dev/null && rm -rf $out/traffic/fetch $out/traffic/write
echo done
