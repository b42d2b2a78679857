#!/bin/bash
# Round 6: the self-spawned 2-rank rehearsal of bench.py --gpus 2 (gloo, both ranks on one card:
# timings meaningless, the record shows which key `value` comes from), into gpurun_out/$RECORD/.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${RECORD:-r06_n2}; mkdir -p $OUT
DLLM_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --tp-steps 3 --dp-steps 3 \
  > $OUT/bench_n2_selfspawn_gloo.jsonl 2> $OUT/bench_n2_selfspawn_gloo.err
r=$?; echo "n2 rc=$r"; head -c 1500 $OUT/bench_n2_selfspawn_gloo.jsonl; echo
exit $r
