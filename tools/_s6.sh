# round-5 session 6 (temporary): the GPU suite at HEAD; per-class deltas of the two rejected
# A/B switches (rocprofv3 kernel classes, two-stream phases) against the default build
export TMPDIR=/tmp
bash tools/session.sh r05_s6 suite || echo "suite failed (continuing)"
SEG_BN_FOLD=1 bash tools/session.sh r05_s6_fold stats timeline
SEG_DEFER_REDUCE=1 bash tools/session.sh r05_s6_defer timeline
bash tools/session.sh r05_s6_base timeline
echo done
