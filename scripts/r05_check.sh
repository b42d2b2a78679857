#!/bin/bash
# Round 5 check: the new GPU tests (token-parallel C5 emulation, workspace retire, bias_cast guard),
# the bench at N = 1, and the 2-rank gloo rehearsal of the N > 1 path (self-spawned ranks).
set -e
O=gpurun_out/r05_check; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parallel.py -k "token_parallel" > $O/pytest_token.txt 2>&1
cp gpurun_out/c5_token_parallel_G*.json $O/ 2>/dev/null || true
timeout -k 10 300 python -u bench.py > $O/bench.txt 2>&1
DLLM_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 10 --warmup 3 --tp-steps 2 --no-cpu > $O/bench_n2.txt 2>&1
