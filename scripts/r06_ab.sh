#!/bin/bash
# Round 6: interleaved library A/B on one box (scripts/gemm_ab.py), into gpurun_out/$RECORD/ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_ab}; mkdir -p $OUT
LIBS=$LIBS SHAPES=${SHAPES:-2048:4096,4096:2048} ROUNDS=${ROUNDS:-2} \
  timeout -k 10 ${TLIM:-500} python scripts/gemm_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err
r=$?; echo "ab rc=$r"; cat $OUT/ab.jsonl; tail -3 $OUT/ab.err
exit $r
