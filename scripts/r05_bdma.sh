#!/bin/bash
# Round 5: attention K/V staging through a buffer descriptor with compile-time pieces
# (libdllm_hip_bdma.so, DLLM_ATTN_BDMA=1) against the product, at config C4.
set -e
O=gpurun_out/r05_bdma; mkdir -p $O
L=diffusion-llm-rs_amd/lib
DLLM_LIB=$PWD/$L/libdllm_hip_bdma2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "attention or kv" > $O/parity_bdma.txt 2>&1
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_bdma.so,$L/libdllm_hip_bdma2.so ROUNDS=4 timeout -k 10 600 python -u scripts/attn_ab.py > $O/ab.jsonl 2> $O/ab.err
