#!/bin/bash
# Round 5, second decode study: the decode stamps with the 2-D grid fixed (M 64's K-split rows no
# longer fold onto each other) and the LDS-staged path (M 16), plus the new product decode test.
set -e
O=gpurun_out/r05_midm2; mkdir -p $O
L=diffusion-llm-rs_amd/lib
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lds_staged" > $O/pytest_lds_staged.txt 2>&1
timeout -k 10 300 python -u scripts/stamp_decode.py --lib $L/libdllm_hip_stamp.so --ms 1,16,33,64 --out $O/stamp_decode.jsonl > $O/stamp_decode.txt 2>&1
