# whole-step A/B of build/<variant> libraries against the working tree (usage: tools/gpu_ab.sh OUT variant...)
set -e
out=$1; shift
mkdir -p gpurun_out/$out
REPS=${REPS:-2} timeout -k 10 1000 bash tools/ab_bench.sh "$@" > gpurun_out/$out/ab.txt 2>&1
