set -e
out=gpurun_out/s11
mkdir -p $out
export TMPDIR=/tmp
for v in default ru4 ru8 ru12; do
  if [ "$v" = default ]; then unset SEG_HIP_LIB; else export SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so; fi
  SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-profile > $out/$v.log 2>&1
  python3 tools/rocpd_stats.py $out/$v/run_results.db $out/$v.csv > $out/$v.txt
  rm -rf $out/$v
  echo "== $v"; grep -i "bn_bwd_reduce" $out/$v.txt
done > $out/summary.txt
unset SEG_HIP_LIB
timeout -k 10 600 tools/ab_bench.sh ru8 ru12 > $out/ab.txt 2>&1
SEG_HIP_LIB=$PWD/ab/ru8/libseg_hip.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step.py > $out/parity.txt 2>&1
echo done
