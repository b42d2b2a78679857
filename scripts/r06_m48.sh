#!/bin/bash
# Round 6: mid-M tiles from 48 tiles (narrow N) -- linear GPU tests on the m48 build, then the chain at
# N 2048 / 1024 / 512 against the product (96).
set -o pipefail
OUT=gpurun_out/r06_m48; mkdir -p $OUT
DLLM_LIB=diffusion-llm-rs_amd/lib/libdllm_hip_m48.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "linear" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for n in 2048 1024 512; do
  AB_N=$n LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_m48.so ROUNDS=2 MS=128,192,256,384,512 \
    timeout -k 10 300 python scripts/decode_chain_ab.py > $OUT/chain_n$n.jsonl 2>> $OUT/err.txt || exit 1
done
