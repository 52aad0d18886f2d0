# round-6 GPU session: GEMM sweeps (optional) then the default bench line
set -o pipefail
d=gpurun_out/$1; mkdir -p $d
if [ -n "$2" ]; then
  for m in $2; do timeout -k 10 200 ./tools/devbin/gemm_tune 16384 3 $m > $d/gemm_$m.txt 2>&1 || exit 1; done
fi
timeout -k 10 500 python -u bench.py > $d/bench.json 2> $d/bench.err || exit 1
