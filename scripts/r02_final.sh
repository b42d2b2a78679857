#!/bin/bash
# Round-2 record pass on one GPU box, into gpurun_out/r02_final/: the -m gpu suite, the default
# bench line (+ M sweep), every config under rocprofv3 kernel-trace stats (bench_suite.py), the
# bench GEMM's PMC passes + FETCH calibration (r02_profile.sh) and the 2-rank gloo rehearsal of the
# N > 1 bench path.  Each GPU step has its own limit; the first hard failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${RECORD:-r02_final}"
mkdir -p "$OUT"
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.txt"
if hard $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sweep > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
rc2=$?; echo "bench rc=$rc2"; head -c 600 "$OUT/bench.jsonl"; echo
if hard $rc2; then exit $rc2; fi
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/suite" -o suite --output-format csv -- python3 scripts/bench_suite.py \
  > "$OUT/suite.jsonl" 2> "$OUT/suite.err"
rc3=$?; echo "suite rc=$rc3"; cat "$OUT/suite.jsonl" | cut -c1-220
if hard $rc3; then exit $rc3; fi
bash scripts/r02_profile.sh > "$OUT/profile.log" 2>&1
rc4=$?; echo "profile rc=$rc4"; tail -8 "$OUT/profile.log"
if hard $rc4; then exit $rc4; fi
DLLM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --tp-steps 2 \
  > "$OUT/bench_n2_rehearsal.jsonl" 2> "$OUT/bench_n2_rehearsal.err"
rc5=$?; echo "rehearsal rc=$rc5"; head -c 400 "$OUT/bench_n2_rehearsal.jsonl"; echo
exit $(( rc || rc2 || rc3 || rc4 ))
