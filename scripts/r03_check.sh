#!/bin/bash
# Round-3 GPU pass: parity tests, the bench line, and a 2-rank rehearsal (gloo, both ranks on the
# one card) of the N > 1 path including the head-sharded C5 loop with its KV step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PT_ARGS:-} > gpurun_out/pt.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pt.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.log; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
DLLM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --tp-steps 4 --no-cpu > gpurun_out/bench_n2.log 2> gpurun_out/bench_n2.err
rc=$?
echo "bench n2 rc=$rc"; cat gpurun_out/bench_n2.log; tail -5 gpurun_out/bench_n2.err
exit $rc
