#!/bin/bash
# Round 5: decode with LDS-staged X / scales (libdllm_hip_xl.so, DLLM_DECODE_XL=1) against the
# product build: decode parity tests on the variant, then the 40-layer chain A/B.
set -e
O=gpurun_out/r05_xl; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_xl.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity_xl.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_xl.so ROUNDS=3 timeout -k 10 500 python -u scripts/decode_chain_ab.py > $O/ab.jsonl 2> $O/ab.err
