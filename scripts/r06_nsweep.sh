#!/bin/bash
# Round 6: the 40-layer chain over M at the column-shard widths N 2048 / 1024 / 512 (policy survey).
set -o pipefail
OUT=gpurun_out/r06_nsweep; mkdir -p $OUT
for n in 2048 1024 512; do
  AB_N=$n LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so ROUNDS=1 MS=64,128,256,384,512,768,1024,1536,2048,3072,4096 \
    timeout -k 10 300 python scripts/decode_chain_ab.py > $OUT/chain_n$n.jsonl 2>> $OUT/err.txt || exit 1
done
