#!/bin/bash
# Round 6: the -m gpu suite, smoke() and the default bench line on one box, into gpurun_out/$RECORD/.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_check}; mkdir -p $OUT
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
rc=0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYK:+-k "$PYK"} \
  > $OUT/pytest_gpu.txt 2>&1
r=$?; rc=$((rc || r)); echo "pytest rc=$r"; tail -2 $OUT/pytest_gpu.txt
if hard $r; then exit $r; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
r=$?; rc=$((rc || r)); echo "smoke rc=$r"; tail -1 $OUT/smoke.txt
if hard $r; then exit $r; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.jsonl 2> $OUT/bench.err
r=$?; rc=$((rc || r)); echo "bench rc=$r"; head -c 700 $OUT/bench.jsonl; echo
exit $rc
