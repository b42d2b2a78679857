#!/bin/bash
# Round 5 shard study, part 3: the fold kept in its substep (variant 7) and with the coalesced KG2
# epilogue (8) against the product and variant 3: stamps, parity (shard + exact-integer policy
# tests), interleaved A/B on the shard shapes and the C5 layer shape.
set -e
O=gpurun_out/r05_shard3; mkdir -p $O
L=diffusion-llm-rs_amd/lib
for v in stamp7 stamp8; do
  timeout -k 10 240 python -u scripts/stamp_shard.py --lib $L/libdllm_hip_$v.so --shapes 4096x1024,2048x2048,2048x4096 --out $O/$v.jsonl > $O/$v.txt 2>&1
done
for v in shard7 shard8; do
  DLLM_LIB=$PWD/$L/libdllm_hip_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parallel.py tests/test_gpu_parity.py -k "column_shard or policy_exact or exact_weights_tight" > $O/parity_$v.txt 2>&1
done
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_shard3.so,$L/libdllm_hip_shard7.so,$L/libdllm_hip_shard8.so SHAPES=4096:1024,2048:2048,2048:4096,4096:512 ROUNDS=4 timeout -k 10 700 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
