#!/bin/bash
# Round 5: the staggered 128 x 256 exact tiles on 16x16x32 MFMAs (libdllm_hip_ss16.so) vs product.
set -e
O=gpurun_out/r05_ss16; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_ss16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact or prefill or linear" > $O/parity_ss16.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_ss16.so SHAPES=2048:4096,3072:4096,4096:2048 ROUNDS=4 timeout -k 10 400 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
