#!/bin/bash
# One GPU-box pass: parity tests, then (unless the GPU faulted/hung) a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== rocm-smi" && (rocm-smi --showproductname 2>/dev/null | head -20 || true)
timeout -k 10 ${PT_TIMEOUT:-600} python -m pytest tests -m gpu -q -p no:cacheprovider ${PT_ARGS:-} > gpurun_out/pt.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU step failed hard (rc=$rc); stopping"; exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --sweep} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc2=$?
echo "bench rc=$rc2"; cat gpurun_out/bench.log; tail -20 gpurun_out/bench.err
exit $rc2
