#!/bin/bash
# Round 6: int2 g128 on the 256 x 256 Horner kernel -- the GEMM / C3 parity tests on the product build,
# then int2 4096^2 (and 8000 x 4096) against the round-5 product (fold-form int2 kernel), and the
# C3 suite line.
set -o pipefail
OUT=gpurun_out/r06_int2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "int2 or exact_integers or mixed or config3 or c3 or horner" > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
AB_BITS=2 LIBS=diffusion-llm-rs_amd/lib/libdllm_hip.so,diffusion-llm-rs_amd/lib/libdllm_hip_base.so ROUNDS=3 SHAPES=4096:4096,8000:4096 PREWARM_MS=300 \
  timeout -k 10 400 python scripts/gemm_ab.py > $OUT/ab_int2.jsonl 2> $OUT/ab.err || exit 1
cat $OUT/ab_int2.jsonl
