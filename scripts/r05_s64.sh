#!/bin/bash
# Round 5: A/B of 64 x 256 two-k-group tiles (libdllm_hip_s64.so, DLLM_EXACT_SHARD64=1) against the
# product's 128 x 128 two-k-group tiles on the 4-GPU column shard and the other grids they take.
set -e
O=gpurun_out/r05_s64; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_s64.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact or prefill or linear" > $O/parity_s64.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_s64.so SHAPES=4096:1024,2048:2048,2048:4096,3072:1024 ROUNDS=3 timeout -k 10 400 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
