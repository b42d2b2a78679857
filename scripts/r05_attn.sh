#!/bin/bash
# Round 5: the 16x16x32 attention kernel (variant build attn16) -- parity on every attention test,
# then an interleaved A/B against the product (v5) at config C4.
set -e
O=gpurun_out/r05_attn; mkdir -p $O
L=diffusion-llm-rs_amd/lib
DLLM_LIB=$PWD/$L/libdllm_hip_attn16b.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "attention" > $O/parity_attn16.txt 2>&1
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_attn16.so,$L/libdllm_hip_attn16b.so ROUNDS=4 timeout -k 10 600 python -u scripts/attn_ab.py > $O/ab.jsonl 2> $O/ab.err
