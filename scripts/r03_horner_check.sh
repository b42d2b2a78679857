#!/bin/bash
# New Horner kernel: linear parity tests, the K-slope timing, the bench line, the TP diagnostic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "linear" > gpurun_out/pt_linear.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pt_linear.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python scripts/gemm_kslope.py > gpurun_out/kslope.log 2>&1; rc=$?; cat gpurun_out/kslope.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-denoise --no-cpu > gpurun_out/bench.log 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.log; tail -3 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python scripts/diag_tp.py
