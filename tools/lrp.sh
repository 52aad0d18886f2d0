set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lrp0 -o p --output-format csv -- python3 $R/tools/lreg_prof.py 100000000 10 > $R/gpurun_out/lrp0.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/lrp1 -o p --output-format csv -- python3 $R/tools/lreg_prof.py 100000000 4 > $R/gpurun_out/lrp1.log 2>&1
