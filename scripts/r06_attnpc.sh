#!/bin/bash
# Round 6: producer/consumer attention (DLLM_ATTN_PC=1 build) -- parity with the attention tests,
# then an interleaved A/B against the product (v5) on config C4.  Measurement only.
set -o pipefail
OUT=gpurun_out/r06_attnpc
mkdir -p $OUT
DLLM_LIB=diffusion-llm-rs_amd/lib/libdllm_hip_attnpc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "attention" > $OUT/pytest_attnpc.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_attnpc.txt; exit 1; }
tail -3 $OUT/pytest_attnpc.txt
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_attnpc.so ROUNDS=3 \
  timeout -k 10 400 python scripts/attn_ab.py > $OUT/ab.jsonl 2> $OUT/ab.err
cat $OUT/ab.jsonl
