# round-5 session 3 (temporary): new parity tests, the two A/B switches, the db kernel's timing
set -e
out=gpurun_out/r05_s3; mkdir -p $out
export TMPDIR=/tmp
TT=300 bash tools/session.sh r05_s3 tests=tests/test_gpu_step.py::test_bn_fold_matches,tests/test_gpu_step.py::test_defer_stem_update_matches,tests/test_gpu_eval.py::test_predict_order_resize_then_replace_voids,tests/test_gpu_eval.py::test_predict_spec_replace_voids_resized || echo "tests failed (continuing)"
REPS=2 bash tools/session.sh r05_s3 envab=SEG_DEFER_REDUCE:0:1
REPS=2 bash tools/session.sh r05_s3 envab=SEG_BN_FOLD:0:1
LAYERS="b4c3 b3c3 b1c3" OPS="fwd" bash tools/session.sh r05_s3 envops=SEG_NT_DB:0:1
for v in dbtim dbtimnost; do for t in "fwd b4c3" "dgrad b3c1"; do
  echo "== $v $t" >> $out/timing.txt
  SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so timeout -k 5 60 python3 tools/db_timing.py $t >> $out/timing.txt 2>&1
done; done
echo done
