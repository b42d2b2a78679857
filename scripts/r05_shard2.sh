#!/bin/bash
# Round 5 shard study, part 2: the 64 x 256 one-k-group tiles (variants 4/5/6) against the product
# and variant 3 (KG2 + coalesced epilogue): stamps, parity on the shard tests, interleaved A/B.
set -e
O=gpurun_out/r05_shard2; mkdir -p $O
L=diffusion-llm-rs_amd/lib
for v in stamp4 stamp5; do
  timeout -k 10 240 python -u scripts/stamp_shard.py --lib $L/libdllm_hip_$v.so --shapes 4096x1024,2048x2048 --out $O/$v.jsonl > $O/$v.txt 2>&1
done
for v in shard4 shard5 shard6; do
  DLLM_LIB=$PWD/$L/libdllm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parallel.py -k "column_shard" > $O/parity_$v.txt 2>&1
done
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_shard3.so,$L/libdllm_hip_shard4.so,$L/libdllm_hip_shard5.so,$L/libdllm_hip_shard6.so SHAPES=4096:1024,2048:2048 ROUNDS=4 timeout -k 10 600 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
