#!/bin/bash
# One GPU-box session, parametrised (replaces the per-session rNN_sMM.sh scripts):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/session.sh TAG STEP [STEP ...]'
# Output under gpurun_out/TAG/. Every step has its own time limit; the chain stops at the first
# failure (a GPU fault, abort or time limit ends the session there).
# Steps:
#   suite                 the driver's GPU suite (pytest -m gpu)
#   tests=A,B,...         pytest on the given test paths / node ids (comma-separated)
#   smoke                 __graft_entry__.smoke()
#   bench                 the driver's bench command (20 steps, 5 warm-up)
#   benchq                the bench without the CPU baseline / eval / train.py legs
#   multi=N               bench.py --gpus N self-launched, N ranks over gloo on this one GPU
#   stats                 rocprofv3 --kernel-trace --stats of the bench (single-stream backward)
#   timeline              two-stream trace -> timeline.txt / phases.txt
#   traffic               PMC HBM traffic of every kernel of the bench step
#   pmc=OP:LAYER          PMC counter passes of one single-op bench (OP fwd|dgrad|wgrad)
#   ab=V1,V2,...          interleaved whole-step A/B: the in-tree library vs ab/Vi/libseg_hip.so
#   ops=V1,V2,...         single-op A/B on the same variants (OPS / LAYERS env override)
#   envops=VAR[:A:B]      single-op A/B: VAR=A (default 0) vs VAR=B (default unset; OPS / LAYERS)
#   envab=VAR[:A:B]       interleaved whole-step A/B (benchq) of the same two arms, REPS rounds
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
  key=${step%%=*}; val=${step#*=}
  echo "== $step" | tee -a "$out/progress.txt"
  case $key in
    suite) timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$out/suite.txt" 2>&1 ;;
    tests) timeout -k 10 900 python3 -u -m pytest -x -v --timeout ${TT:-600} --timeout-method thread ${val//,/ } >> "$out/tests.txt" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 ;;
    bench) timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" ;;
    benchq) timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-train-py > "$out/benchq.json" 2> "$out/benchq.err" ;;
    multi) SEG_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus "$val" --steps 2 --warmup 1 --no-eval --no-train-py --no-cpu-baseline > "$out/multi$val.json" 2> "$out/multi$val.err" ;;
    stats)
      SEG_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-train-py > "$out/stats.log" 2>&1
      python3 tools/rocpd_stats.py "$out/stats/run_results.db" "$out/kernel_stats.csv" > "$out/kernel_classes.txt"
      rm -rf "$out/stats" ;;
    timeline) bash tools/timeline_pass.sh "$tag/tl" ;;
    traffic)
      tools/pmc_traffic.sh "$out/traffic" && python3 tools/pmc_traffic.py "$out/traffic" "$out/pmc_traffic.json"
      rm -rf "$out/traffic/fetch" "$out/traffic/write" ;;
    pmc)
      op=${val%%:*}; layer=${val#*:}
      tools/pmc_passes.sh "$out/pmc_${op}_$layer" "$op" "$layer"
      python3 tools/rocpd_pmc.py "$out/pmc_${op}_$layer" conv > "$out/pmc_${op}_$layer.txt"
      rm -rf "$out/pmc_${op}_$layer" ;;
    ab) REPS=${REPS:-3} bash tools/ab_bench.sh ${val//,/ } >> "$out/ab.txt" 2>&1 ;;
    ops) bash tools/ab_ops.sh ${val//,/ } >> "$out/ops.txt" 2>&1 ;;
    envops)
      [ "$val" = envops ] && { echo "envops needs =VAR"; exit 2; }
      IFS=: read -r var va vb <<< "$val"
      for v in "${va:-0}" "${vb:-default}"; do
        echo "== $var=$v" >> "$out/envops.txt"
        for op in ${OPS:-fwd dgrad}; do for l in ${LAYERS:-b4c3 b3c3 b2c3 b1c3 b4c1 b3c1}; do
          if [ "$v" = default ]; then timeout -k 5 60 python3 tools/op_bench.py $op $l >> "$out/envops.txt" 2>&1
          else env $var=$v timeout -k 5 60 python3 tools/op_bench.py $op $l >> "$out/envops.txt" 2>&1; fi
        done; done
      done ;;
    envab)
      [ "$val" = envab ] && { echo "envab needs =VAR"; exit 2; }
      IFS=: read -r var va vb <<< "$val"
      for r in $(seq ${REPS:-3}); do for v in "${va:-0}" "${vb:-default}"; do
        if [ "$v" = default ]; then timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-train-py > "$out/envab.tmp" 2>&1
        else env $var=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-eval --no-train-py > "$out/envab.tmp" 2>&1; fi
        echo "$var=$v $(tail -1 "$out/envab.tmp" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> "$out/envab.txt"
      done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done | tee -a "$out/progress.txt"
