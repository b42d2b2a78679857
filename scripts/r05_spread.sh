#!/bin/bash
# Round 5: the DMA-spread A/B of the fold kernels and the MFMA-only / load-only ablations (stamps
# with the DMA issue split out, parity of the spread build, interleaved timing).
set -e
O=gpurun_out/r05_spread; mkdir -p $O
L=diffusion-llm-rs_amd/lib
for v in stamp stampsp stampabl1 stampabl2; do
  timeout -k 10 240 python -u scripts/stamp_shard.py --lib $L/libdllm_hip_$v.so --shapes 4096x1024,2048x4096,2048x2048 --out $O/$v.jsonl > $O/$v.txt 2>&1
done
DLLM_LIB=$PWD/$L/libdllm_hip_spread.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parallel.py tests/test_gpu_parity.py -k "column_shard or policy_exact or exact_weights_tight or linear" > $O/parity_spread.txt 2>&1
LIBS=$L/libdllm_hip.so,$L/libdllm_hip_spread.so SHAPES=4096:1024,2048:4096,2048:2048,4096:512,4096:4096 ROUNDS=5 timeout -k 10 700 python -u scripts/gemm_ab.py > $O/ab.jsonl 2> $O/ab.err
timeout -k 10 100 python -u scripts/c5_shard_costs.py --out $O/c5_shard_costs.json > $O/c5_shard_costs.txt 2>&1
