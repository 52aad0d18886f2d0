set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/gpurun_out/kmpmc1 -o p --output-format csv -- python3 $R/tools/km_once.py 100000000 2 > $R/gpurun_out/kmpmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kmpmc0 -o p --output-format csv -- python3 $R/tools/km_once.py 100000000 2 > $R/gpurun_out/kmpmc0.log 2>&1
