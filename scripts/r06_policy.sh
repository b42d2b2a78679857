#!/bin/bash
# Round 6: the rounds-based choice between the 256 x 256 Horner, 128 x 256 PC and two-k-group PC grids
# (DLLM_POLICY_ROUNDS) -- the linear GPU tests on the product build, then the 40-layer chain against the
# full-round thresholds (pold build).
set -o pipefail
OUT=gpurun_out/r06_policy; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_diffusion.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "linear or mixed or denoise or psample" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_pold.so MS=1100,1280,1536,1800,1900,2048,2304,2560,3072,3584,4096 \
  timeout -k 10 600 python scripts/decode_chain_ab.py > $OUT/chain.jsonl 2> $OUT/chain.err || exit 1
