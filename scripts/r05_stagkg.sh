#!/bin/bash
# Round 5: 128 x 128 two-k-group tiles with the k-group halves staggered and each stage's loads split
# over the two half steps (libdllm_hip_stagkg.so) against the product.
set -e
O=gpurun_out/r05_stagkg; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_stagkg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "exact or prefill or linear or shard" > $O/parity.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_stagkg.so SHAPES=4096:1024,2048:2048,3072:1024 ROUNDS=4 timeout -k 10 400 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
