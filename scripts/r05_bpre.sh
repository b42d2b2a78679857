#!/bin/bash
# Round 5: exact kernels with the epilogue's bias loaded at kernel start (libdllm_hip_bpre.so) vs product.
set -e
O=gpurun_out/r05_bpre; mkdir -p $O
L=$PWD/diffusion-llm-rs_amd/lib
DLLM_LIB=$L/libdllm_hip_bpre.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact or prefill or linear or psample or staggered" > $O/parity.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_bpre.so SHAPES=2048:4096,4096:2048,4096:1024,4096:512,256:4096 ROUNDS=4 timeout -k 10 500 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
