set -e
out=gpurun_out/r05_s3; mkdir -p $out
export TMPDIR=/tmp
LAYERS="b4c3 b3c3 b1c3" OPS="fwd" bash tools/session.sh r05_s3 envops=SEG_NT_DB:0:1
LAYERS="b4c1 b3c1" OPS="dgrad" bash tools/session.sh r05_s3 envops=SEG_NT_DB:0:1
for v in dbtim dbtimnost; do for t in "fwd b4c3" "fwd b3c3" "dgrad b3c1"; do
  echo "== $v $t" >> $out/timing.txt
  SEG_HIP_LIB=$PWD/ab/$v/libseg_hip.so timeout -k 5 60 python3 tools/db_timing.py $t >> $out/timing.txt 2>&1
done; done
for t in "fwd b4c3" "fwd b3c3" "dgrad b4c1" "dgrad b3c1"; do
  echo "== nostore $t" >> $out/timing.txt
  SEG_HIP_LIB=$PWD/ab/dbnost/libseg_hip.so timeout -k 5 60 python3 tools/op_bench.py $t >> $out/timing.txt 2>&1
done
echo done
