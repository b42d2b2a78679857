#!/bin/bash
# Round 5: the lean Horner16 loop (libdllm_hip_lean.so, DLLM_H16_LEAN=1: opaque fragment bases,
# branch-free DMA pieces) against the product on the Horner shapes.
set -e
O=gpurun_out/r05_lean; mkdir -p $O
DLLM_LIB=$PWD/diffusion-llm-rs_amd/lib/libdllm_hip_lean.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "horner or exact or prefill or linear or psample" > $O/parity_lean.txt 2>&1
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_lean.so SHAPES=4096:4096,8192:4096,4096:8192 ROUNDS=4 timeout -k 10 400 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
