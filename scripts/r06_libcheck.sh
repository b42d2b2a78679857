#!/bin/bash
# Round 6: correctness screen (scripts/lib_check.py) of each library in $LIBS, then the interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_libcheck}; mkdir -p $OUT
for L in ${LIBS//,/ }; do
  DLLM_LIB=$L timeout -k 10 120 python scripts/lib_check.py ${CHECK_SHAPES:-2048:4096,4096:2048,3000:4096,2048:4092} >> $OUT/check.jsonl 2>> $OUT/check.err
  r=$?; echo "check $L rc=$r"; tail -1 $OUT/check.jsonl
  case $r in 124|134|137|139) exit $r;; esac
done
LIBS=$LIBS SHAPES=${SHAPES:-2048:4096,4096:2048} ROUNDS=${ROUNDS:-3} \
  timeout -k 10 ${TLIM:-500} python scripts/gemm_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err
r=$?; echo "ab rc=$r"; cat $OUT/ab.jsonl
exit $r
