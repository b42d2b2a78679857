#!/bin/bash
# Round 5: A/B of the staggered-halves 128 x 256 exact tiles (libdllm_hip_stag.so, DLLM_EXACT_STAG=1)
# against the product build on the shapes that route to them, plus the exact-GEMM parity tests on
# the variant build.
set -e
O=gpurun_out/r05_stag; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_stag.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact or prefill or linear" > $O/parity_stag.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_stag.so SHAPES=2048:4096,3072:4096,4096:1024,4096:2048,4096:512,2048:1024,256:4096,512:4096 ROUNDS=3 timeout -k 10 400 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
