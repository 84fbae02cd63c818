# Two-stream step timeline and phase split of the bench step (GPU box):
#   bash tools/timeline_pass.sh TAG  -> gpurun_out/TAG/{timeline,phases}.txt
set -e
out=gpurun_out/${1:-timeline}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile --no-train-py > $out/tr.log 2>&1
python3 tools/timeline.py $out/tr/run_results.db > $out/timeline.txt
python3 tools/phases.py $out/tr/run_results.db > $out/phases.txt
rm -rf $out/tr
echo done
