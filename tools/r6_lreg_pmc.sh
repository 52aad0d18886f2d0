# round-6 GPU session: cfg2 and lreg kernels side by side, FETCH_SIZE and wait counters (separate passes)
set -o pipefail
d=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $d
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --dot 0 --workloads lreg --cpu-baseline 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o p --output-format csv -- $B > $d/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM -d $d/wait -o p --output-format csv -- $B > $d/wait.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $d/trace -o p --output-format csv -- $B > $d/trace.log 2>&1 || exit 1
