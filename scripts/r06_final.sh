#!/bin/bash
# Round-6 record pass on one GPU box, into gpurun_out/${RECORD:-r06_final}/.
# PART=1: the -m gpu suite, smoke(), the default bench line, the 40-layer graph M-sweep, the bench's
#         rocprofv3 kernel-trace stats.
# PART=2: rocprofv3 kernel-trace means of the column-shard / C5 GEMM shapes (kernel_times.py), every
#         config under kernel-trace (bench_suite.py), the self-spawned 2-rank gloo rehearsal of
#         bench.py --gpus 2.
# rocprofv3 output goes to /tmp; only the stats CSVs are copied.  Each GPU step has its own limit; a
# hard failure (timeout / abort / segfault) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${RECORD:-r06_final}"
mkdir -p "$OUT"
hard() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
rc=0
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.txt" 2>&1
  r=$?; rc=$((rc || r)); echo "pytest rc=$r"; tail -2 "$OUT/pytest_gpu.txt"
  if hard $r; then exit $r; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
  r=$?; rc=$((rc || r)); echo "smoke rc=$r"; tail -1 "$OUT/smoke.txt"
  if hard $r; then exit $r; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
  r=$?; rc=$((rc || r)); echo "bench rc=$r"; head -c 900 "$OUT/bench.jsonl"; echo
  if hard $r; then exit $r; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --sweep --no-cpu --no-denoise > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
  r=$?; rc=$((rc || r)); echo "sweep rc=$r"
  if hard $r; then exit $r; fi
  rm -rf /tmp/prof_kt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --no-denoise \
    > "$OUT/kt.log" 2>&1
  r=$?; rc=$((rc || r)); echo "kernel-trace rc=$r"; tail -c 300 "$OUT/kt.log"; echo
  find /tmp/prof_kt -name "*kernel_stats.csv" -exec cp {} "$OUT/bench_kernel_stats.csv" \;
  exit $rc
fi
mkdir -p "$OUT/shapes"
for sh in 4096:4096 4096:2048 4096:1024 4096:512 2048:4096 2048:2048 2048:1024 1024:4096 512:4096; do
  tag=$(echo $sh | tr ':' 'x'); rm -rf /tmp/prof_$tag
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o $tag --output-format csv -- python3 scripts/kernel_times.py \
    diffusion-llm-rs_amd/lib/libdllm_hip.so $sh > "$OUT/shapes/$tag.log" 2>&1
  r=$?; rc=$((rc || r)); echo "shape $sh rc=$r"
  find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} "$OUT/shapes/${tag}_kernel_stats.csv" \;
  if hard $r; then exit $r; fi
done
rm -rf /tmp/prof_suite
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d /tmp/prof_suite -o suite --output-format csv -- python3 scripts/bench_suite.py \
  > "$OUT/suite.jsonl" 2> "$OUT/suite.err"
r=$?; rc=$((rc || r)); echo "suite rc=$r"; cut -c1-200 "$OUT/suite.jsonl"
find /tmp/prof_suite -name "*kernel_stats.csv" -exec cp {} "$OUT/suite_kernel_stats.csv" \;
if hard $r; then exit $r; fi
# PMC of the producer/consumer kernels (FETCH / WRITE in their own passes): C5 layer and 4-GPU shard
for spec in "wq_horner_pc_kernel 2048:4096" "wq_horner_pc_kg2_kernel 4096:1024"; do
  set -- $spec; KRE=$1; SH=$2; tag=$(echo $SH | tr ':' 'x'); j=0
  for C in "FETCH_SIZE" "WRITE_SIZE"; do
    j=$((j+1)); rm -rf /tmp/pmcpc_$j
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d /tmp/pmcpc_$j -o pmc --output-format csv -- python3 scripts/kernel_times.py diffusion-llm-rs_amd/lib/libdllm_hip.so $SH > "$OUT/pmc_${tag}_$j.log" 2>&1
    r=$?; echo "pmc $KRE $C rc=$r"; rc=$((rc || r))
    [ $r -eq 0 ] || exit $r
    mkdir -p "$OUT/pmc_$tag/p$j"; find /tmp/pmcpc_$j -name "*counter_collection.csv" -exec cp {} "$OUT/pmc_$tag/p$j/" \;
  done
  python3 scripts/pmc_to_json.py "$OUT/pmc_$tag" "$OUT/pmc_$tag.json" "$KRE" ${SH%%:*} 4096 ${SH##*:} 4 128 r06-pc
done
DLLM_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --tp-steps 3 --dp-steps 3 \
  > "$OUT/bench_n2_selfspawn_gloo.jsonl" 2> "$OUT/bench_n2_selfspawn_gloo.err"
r=$?; rc=$((rc || r)); echo "rehearsal rc=$r"; head -c 400 "$OUT/bench_n2_selfspawn_gloo.jsonl"; echo
exit $rc
