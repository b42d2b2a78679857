#!/bin/bash
# Round 5 shard study (one box): stamped phase breakdowns of the product / variant 1 / variant 3,
# parity of each variant on the shard tests, then an interleaved A/B of the four builds.
set -e
O=gpurun_out/r05_shard; mkdir -p $O
L=diffusion-llm-rs_amd/lib
for v in stamp stamp1 stamp3; do
  timeout -k 10 240 python -u scripts/stamp_shard.py --lib $L/libdllm_hip_$v.so --shapes 4096x1024,4096x512,2048x2048 --out $O/$v.jsonl > $O/$v.txt 2>&1
done
for v in shard1 shard2 shard3; do
  DLLM_LIB=$PWD/$L/libdllm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parallel.py -k "column_shard" > $O/parity_$v.txt 2>&1
done
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_shard1.so,$L/libdllm_hip_shard2.so,$L/libdllm_hip_shard3.so SHAPES=4096:1024,4096:512,2048:2048,4096:4096 ROUNDS=3 timeout -k 10 600 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
