# round-6 GPU session: the default bench (minus the CPU legs) under a kernel trace
set -o pipefail
d=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $d
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d/benchtrace -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 > $d/benchtrace.json 2> $d/benchtrace.err
