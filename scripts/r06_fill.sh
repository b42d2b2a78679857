#!/bin/bash
# Round 6: the two-k-group PC tile choice (128- vs 64-row tiles by rounds, 64-row grids from 3/4 of a
# round) -- the linear GPU tests on the product build, then the 40-layer chain against the previous
# policy (fill256 build).
set -o pipefail
OUT=gpurun_out/r06_fill; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "linear" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_fill256.so MS=300,320,384,448,512,576,640,700,768,800,900,1024 \
  timeout -k 10 500 python scripts/decode_chain_ab.py > $OUT/chain3.jsonl 2> $OUT/chain3.err || exit 1
