set -o pipefail
d=gpurun_out/$1; mkdir -p $d
timeout -k 10 500 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread -k "kmeans or join or cdist" > $d/km_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/km_api_timeline.py 100000000 5 > $d/timeline.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --dot 0 --workloads kmeans,kmeans_api --cpu-baseline 0 > $d/bench.json 2> $d/bench.err || exit 1
