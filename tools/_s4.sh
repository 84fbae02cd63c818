# round-5 session 4 (temporary): the driver's GPU suite at HEAD, smoke, the N=2 self-launch
# rehearsal, the driver's bench, rocprofv3 kernel stats and the two-stream timeline
out=gpurun_out/r05_s4; mkdir -p $out
export TMPDIR=/tmp
bash tools/session.sh r05_s4 suite || echo "suite failed (continuing)"
bash tools/session.sh r05_s4 smoke multi=2 bench stats timeline
echo done
