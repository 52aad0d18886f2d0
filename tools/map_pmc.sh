set -e
R=$GRAFT_REPO_ROOT
SPX_MAP_GRID=1048576 timeout -k 10 100 python3 -u $R/tools/map_check.py > $R/gpurun_out/mc2.log 2>&1
cd /tmp && export TMPDIR=/tmp
SPX_MAP_GRID=1048576 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/mcf -o p --output-format csv -- python3 $R/tools/map_check.py > $R/gpurun_out/mcf.log 2>&1
SPX_MAP_GRID=1048576 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/mcw -o p --output-format csv -- python3 $R/tools/map_check.py > $R/gpurun_out/mcw.log 2>&1
