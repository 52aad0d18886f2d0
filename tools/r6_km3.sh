# round-6 GPU session: k-means tests, then the k-means legs of the bench (no trace, then traced)
set -o pipefail
d=gpurun_out/$1; mkdir -p $d
timeout -k 10 500 python -u -m pytest tests/ -q -x -m gpu --timeout 300 --timeout-method thread -k "kmeans or join or cdist" > $d/km_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dot 0 --workloads kmeans,kmeans_api --cpu-baseline 0 > $d/bench_plain.json 2> $d/bench_plain.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$d/trace -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --dot 0 --workloads kmeans,kmeans_api --cpu-baseline 0 > $GRAFT_REPO_ROOT/$d/bench.json 2> $GRAFT_REPO_ROOT/$d/bench.err || exit 1
