set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kmt -o p --output-format csv -- python3 $R/bench.py --dot 0 --cpu-baseline 0 --steps 2 > $R/gpurun_out/kmt.log 2>&1
