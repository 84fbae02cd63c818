# rocprofv3 kernel stats (single-stream backward), PMC HBM traffic of the bench step and counter passes on four C2 layers: tools/measure_final.sh TAG (GPU box)
set -e
out=gpurun_out/${1:-final_prof}
mkdir -p $out
export TMPDIR=/tmp
echo "stats" && SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval > $out/stats.log 2>&1
python3 tools/rocpd_stats.py $out/stats/run_results.db $out/kernel_stats.csv > $out/kernel_classes.txt
rm -rf $out/stats
echo "traffic" && tools/pmc_traffic.sh $out/traffic && python3 tools/pmc_traffic.py $out/traffic $out/pmc_traffic.json && rm -rf $out/traffic/fetch $out/traffic/write
for spec in "wgrad b4c2" "fwd b4c3" "dgrad b4c1" "wgrad b3c1"; do
  set -- $spec
  echo "pmc $1 $2" && tools/pmc_passes.sh $out/pmc_$1_$2 $1 $2 && python3 tools/rocpd_pmc.py $out/pmc_$1_$2 conv > $out/pmc_$1_$2.txt && rm -rf $out/pmc_$1_$2
done
echo timeline; bash tools/timeline_pass.sh $(basename $out)_tl
echo done
