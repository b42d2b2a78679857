#!/bin/bash
# Round 5: the fused p_sample epilogue with the tile's x_t / coefficient loads hoisted above its
# stores (libdllm_hip_epi.so) against the product: diffusion GPU tests on the build, then C5 A/B.
set -e
O=gpurun_out/r05_epi; mkdir -p $O
L=$PWD/diffusion-llm-rs_amd/lib
DLLM_LIB=$L/libdllm_hip_epi.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_diffusion.py tests/test_gpu_parity.py -k "psample or diffusion or denoise or p_sample or fused" > $O/parity.txt 2>&1
for r in 1 2 3; do
  DLLM_LIB=$L/libdllm_hip.so ROUNDS=1 timeout -k 10 200 python -u scripts/c5_breakdown.py 50 spread >> $O/c5_product.jsonl 2>> $O/err.txt
  DLLM_LIB=$L/libdllm_hip_epi.so ROUNDS=1 timeout -k 10 200 python -u scripts/c5_breakdown.py 50 spread >> $O/c5_epi.jsonl 2>> $O/err.txt
done
