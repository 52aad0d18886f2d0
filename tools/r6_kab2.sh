# round-6 GPU session: fused k-means step A/B (product libspx.so vs a variant .so): time, result checksums, kernel trace
set -o pipefail
d=$GRAFT_REPO_ROOT/gpurun_out/$1; v=$2; mkdir -p $d
cd $GRAFT_REPO_ROOT
for k in 1 2; do
  timeout -k 10 120 python tools/km_step_once.py 100000000 5 step >> $d/base.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/km_step_once.py 100000000 5 step $v >> $d/var.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d/trace_var -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_step_once.py 100000000 3 step $GRAFT_REPO_ROOT/$v > $d/trace_var.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d/trace_base -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_step_once.py 100000000 3 step > $d/trace_base.log 2>&1 || exit 1
