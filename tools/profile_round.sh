#!/bin/bash
# Round-end profiles (GPU box): kernel trace + stats of the bench, separate
# FETCH_SIZE / WRITE_SIZE passes over cfg2 and over k-means iterations.
#   bash tools/profile_round.sh TAG   -> gpurun_out/prof_TAG/...
set -e
R=$GRAFT_REPO_ROOT
T=${1:-r02}
O=$R/gpurun_out/prof_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace -o p --output-format csv -- python3 $R/bench.py --cpu-baseline 0 > $O/bench_under_rocprof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/c2f -o p --output-format csv -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 3 --warmup 1 > $O/c2f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/c2w -o p --output-format csv -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 3 --warmup 1 > $O/c2w.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/kmf -o p --output-format csv -- python3 $R/tools/km_iter.py 100000000 2 > $O/kmf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/kmw -o p --output-format csv -- python3 $R/tools/km_iter.py 100000000 2 > $O/kmw.log 2>&1
echo done
