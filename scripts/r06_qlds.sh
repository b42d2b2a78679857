#!/bin/bash
# Round 6: the quantize map with LDS-assembled 16-B code stores (product, DLLM_QMAP_LDS=1) -- the GPU
# suite on the product build, then quant_kv_ab.py on it and on the per-lane-store build (qold).
set -o pipefail
OUT=gpurun_out/r06_qlds; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
for r in 0 1; do
  for L in libdllm_hip libdllm_hip_qold; do
    echo -n "{\"lib\": \"$L\", \"round\": $r, \"res\": " >> $OUT/ab.jsonl
    DLLM_LIB=diffusion-llm-rs_amd/lib/$L.so timeout -k 10 200 python3 scripts/quant_kv_ab.py 2>> $OUT/ab.err | tail -1 | tr -d '\n' >> $OUT/ab.jsonl || exit 1
    echo "}" >> $OUT/ab.jsonl
  done
done
cat $OUT/ab.jsonl
