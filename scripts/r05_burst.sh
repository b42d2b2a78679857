#!/bin/bash
# Round 5: exact kernels with compile-time slabs-per-group and burst X DMAs (libdllm_hip_burst.so)
# against the product build.
set -e
O=gpurun_out/r05_burst; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_burst.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity_burst.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_burst.so SHAPES=2048:4096,4096:2048,4096:1024,4096:512,256:4096,512:4096 ROUNDS=4 timeout -k 10 500 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
