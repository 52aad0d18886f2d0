#!/bin/bash
# Dev A/B (GPU box): bench.py with the streaming legs before the GEMM leg
# (default) and after it (SPARTAN_BENCH_DOT_FIRST=1), alternating, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ao; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --cpu-baseline 0 > $O/new_$i.json 2> $O/new_$i.err || exit 1
  SPARTAN_BENCH_DOT_FIRST=1 timeout -k 10 400 python3 bench.py --cpu-baseline 0 > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
