#!/bin/bash
# Round 5 decode / mid-M study: stamps of the decode kernel (M 1 / 16 / 64, last layer of a warm
# 40-layer chain) and of the mid-M exact kernel (M 256, 512 at N 4096), plus the 40-layer graph sweep.
set -e
O=gpurun_out/r05_midm; mkdir -p $O
L=diffusion-llm-rs_amd/lib
timeout -k 10 300 python -u scripts/stamp_decode.py --lib $L/libdllm_hip_stamp.so --out $O/stamp_decode.jsonl > $O/stamp_decode.txt 2>&1
timeout -k 10 240 python -u scripts/stamp_shard.py --lib $L/libdllm_hip_stamp.so --shapes 256x4096,512x4096 --out $O/stamp_midm.jsonl > $O/stamp_midm.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --sweep --no-cpu --no-denoise > $O/sweep.jsonl 2> $O/sweep.err
