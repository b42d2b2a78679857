#!/bin/bash
# One GPU-box pass (round 2): parity tests, the 1-GPU bench line, then a 2-rank rehearsal of the
# N > 1 bench path on the one GPU (gloo, both ranks on the same card: timings meaningless).
# Every GPU step has its own time limit; the script stops at the first hard failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 ${PT_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider ${PT_ARGS:-} > gpurun_out/pt.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pt.log | tail -60
if hard $rc; then echo "GPU step failed hard (rc=$rc); stopping"; exit $rc; fi
[ -n "${SKIP_BENCH:-}" ] && exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --sweep} > gpurun_out/bench.jsonl 2> gpurun_out/bench.err
rc2=$?
echo "bench rc=$rc2"; cat gpurun_out/bench.jsonl; tail -5 gpurun_out/bench.err
if hard $rc2; then exit $rc2; fi
[ -n "${SKIP_REHEARSAL:-}" ] && exit $(( rc || rc2 ))
DLLM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --tp-steps 2 \
  > gpurun_out/bench_n2_rehearsal.jsonl 2> gpurun_out/bench_n2_rehearsal.err
rc3=$?
echo "rehearsal rc=$rc3"; cat gpurun_out/bench_n2_rehearsal.jsonl; tail -5 gpurun_out/bench_n2_rehearsal.err
exit $(( rc || rc2 ))
