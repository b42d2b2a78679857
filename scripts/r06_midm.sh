#!/bin/bash
# Round 6: the mid-M 32 x 128 tiles on grids short of a round (DLLM_MIDM_MINFILL 96) -- linear GPU tests,
# then the 40-layer chain against the full-round threshold (mold build).
set -o pipefail
OUT=gpurun_out/r06_midm; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "linear" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_mold.so MS=65,96,128,160,192,224,256 \
  timeout -k 10 500 python scripts/decode_chain_ab.py > $OUT/chain.jsonl 2> $OUT/chain.err || exit 1
