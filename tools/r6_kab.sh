# round-6 GPU session: k_kmeans_pp A/B (product libspx.so vs a variant .so), time and SALU / VALU counters
set -o pipefail
d=$GRAFT_REPO_ROOT/gpurun_out/$1; v=$2; mkdir -p $d
cd $GRAFT_REPO_ROOT
for k in 1 2; do
  timeout -k 10 120 python tools/km_step_once.py 100000000 5 step >> $d/time_base.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/km_step_once.py 100000000 5 step $v >> $d/time_var.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $d/pmc_base -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_step_once.py 100000000 2 step > $d/pmc_base.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $d/pmc_var -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_step_once.py 100000000 2 step $GRAFT_REPO_ROOT/$v > $d/pmc_var.log 2>&1 || exit 1
