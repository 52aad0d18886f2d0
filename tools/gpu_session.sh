#!/bin/bash
# One GPU-box session: GPU tests, the default bench line, a cfg2-only kernel
# trace, and the cfg5 (lreg) FETCH_SIZE / WRITE_SIZE passes.
#   bash tools/gpu_session.sh TAG [steps...]   -> gpurun_out/TAG/...
# steps: tests bench trace2 lregpmc (default: all, in that order).  A step
# that ends in a fault, abort, signal or time limit stops the session (no
# further GPU work in this call); an ordinary test failure (pytest exit 1)
# does not.
R=$GRAFT_REPO_ROOT
T=${1:-sess}
shift
STEPS=${*:-tests bench trace2 lregpmc}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with $rc" | tee -a $O/steps.log
    exit $rc
  fi
}
for s in $STEPS; do
  case $s in
    tests)
      cd $R && step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $O/pytest.log 2>&1 ;;
    bench)
      cd $R && step bench 600 python3 bench.py > $O/bench.json 2> $O/bench.err ;;
    trace2)
      cd /tmp && step trace2 300 rocprofv3 --kernel-trace --stats -d $O/trace2 -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 20 --warmup 5 > $O/trace2.log 2>&1 ;;
    trace5)
      cd /tmp && step trace5 300 rocprofv3 --kernel-trace --stats -d $O/trace5 -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/trace5.log 2>&1 ;;
    lregpmc)
      cd /tmp && step lregf 300 rocprofv3 --pmc FETCH_SIZE -d $O/lregf -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/lregf.log 2>&1
      cd /tmp && step lregw 300 rocprofv3 --pmc WRITE_SIZE -d $O/lregw -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/lregw.log 2>&1 ;;
    kmpmc)
      cd /tmp && step kmf 300 rocprofv3 --pmc FETCH_SIZE -d $O/kmf -o p --output-format csv \
        -- python3 $R/tools/km_iter.py 100000000 2 > $O/kmf.log 2>&1
      cd /tmp && step kmw 300 rocprofv3 --pmc WRITE_SIZE -d $O/kmw -o p --output-format csv \
        -- python3 $R/tools/km_iter.py 100000000 2 > $O/kmw.log 2>&1 ;;
    *)
      # anything else: a python script under tools/ with its arguments joined by ':'
      cd $R && step "$s" 600 python3 ${s//:/ } > $O/$(basename ${s%%:*}).log 2>&1 ;;
  esac
done
echo "[$(date +%T)] session done" | tee -a $O/steps.log
