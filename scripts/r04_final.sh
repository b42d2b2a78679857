#!/bin/bash
# Round-4 record pass on one GPU box, into gpurun_out/r04_record/ (PART=1: the -m gpu suite, the
# default bench line, the 40-layer graph M-sweep, the bench GEMM's rocprofv3 kernel-trace stats;
# PART=2: every config under kernel-trace stats (bench_suite.py), the bench GEMM's PMC passes
# (r03_pmc.sh) and the 2-rank gloo rehearsal of the N > 1 bench path).  Each GPU step has its own
# limit; a hard failure (timeout / abort / segfault) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${RECORD:-r04_record}"
mkdir -p "$OUT"
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
rc=0
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.txt" 2>&1
  r=$?; rc=$((rc || r)); echo "pytest rc=$r"; tail -2 "$OUT/pytest_gpu.txt"
  if hard $r; then exit $r; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
  r=$?; rc=$((rc || r)); echo "bench rc=$r"; head -c 900 "$OUT/bench.jsonl"; echo
  if hard $r; then exit $r; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --sweep --no-cpu --no-denoise > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
  r=$?; rc=$((rc || r)); echo "sweep rc=$r"
  if hard $r; then exit $r; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --no-denoise \
    > "$OUT/kt.log" 2>&1
  r=$?; rc=$((rc || r)); echo "kernel-trace rc=$r"; tail -c 400 "$OUT/kt.log"; echo
  exit $rc
fi
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/suite" -o suite --output-format csv -- python3 scripts/bench_suite.py \
  > "$OUT/suite.jsonl" 2> "$OUT/suite.err"
r=$?; rc=$((rc || r)); echo "suite rc=$r"; cut -c1-200 "$OUT/suite.jsonl"
if hard $r; then exit $r; fi
bash scripts/r03_pmc.sh > "$OUT/pmc.log" 2>&1
r=$?; rc=$((rc || r)); echo "pmc rc=$r"; tail -3 "$OUT/pmc.log"
if hard $r; then exit $r; fi
DLLM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --tp-steps 3 \
  > "$OUT/bench_n2_rehearsal.jsonl" 2> "$OUT/bench_n2_rehearsal.err"
r=$?; rc=$((rc || r)); echo "rehearsal rc=$r"; head -c 400 "$OUT/bench_n2_rehearsal.jsonl"; echo
exit $rc
