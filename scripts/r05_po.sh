#!/bin/bash
# Round 5: decode kernels vs the exact prefill kernels (prefill-only handles) at M 17..64.
set -e
O=gpurun_out/r05_po; mkdir -p $O
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so POS=0,1 MS=17,24,32,40,48,64 ROUNDS=3 timeout -k 10 500 python -u scripts/decode_chain_ab.py > $O/ab.jsonl 2> $O/ab.err
