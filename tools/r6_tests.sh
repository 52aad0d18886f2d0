# round-6 GPU session: the whole GPU test suite in one process
set -o pipefail
mkdir -p gpurun_out/$1
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$1/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/$1/pytest_gpu.log
