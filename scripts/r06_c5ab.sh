#!/bin/bash
# Round 6: C5 step A/B of library builds (scripts/c5_lib_ab.py), into gpurun_out/$RECORD/c5_ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_c5ab}; mkdir -p $OUT
LIBS=$LIBS ROUNDS=${ROUNDS:-3} REPS=${REPS:-2} timeout -k 10 ${TLIM:-900} python scripts/c5_lib_ab.py > $OUT/c5_ab.jsonl 2> $OUT/c5_ab.err
r=$?; echo "c5 ab rc=$r"; cat $OUT/c5_ab.jsonl; tail -3 $OUT/c5_ab.err
exit $r
