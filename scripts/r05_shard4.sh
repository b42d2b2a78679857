#!/bin/bash
# Round 5 shard study, part 4: per-kernel rocprof times of the decoupled k-half variants (9: 128-deep
# stages, 10: 64-deep in a 3-ring; f32 slabs + combine launch) against the product and variant 3.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_shard4; mkdir -p $O
L=diffusion-llm-rs_amd/lib
for v in "" _shard3 _shard9 _shard10; do
  for s in 4096:1024 2048:2048; do
    n=lib${v:-_prod}_${s/:/x}
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o $n -- python3 scripts/kernel_times.py $L/libdllm_hip$v.so $s > $O/$n.log 2>&1 && find /tmp/prof -name "${n}_kernel_stats.csv" -exec cp {} $O/ \;
  done
done
