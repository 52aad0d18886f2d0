set -o pipefail
mkdir -p gpurun_out/r6l
timeout -k 10 200 ./tools/devbin/gemm_tune 16384 3 p3 > gpurun_out/r6l/p3.txt 2>&1 || exit 1
timeout -k 10 300 ./tools/devbin/gemm_tune 32768 2 p3 > gpurun_out/r6l/p3_32k.txt 2>&1 || exit 1
SPX_GEMM_P3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -m gpu -k "dot" > gpurun_out/r6l/dot_tests_p3.log 2>&1 || exit 1
SPX_GEMM_P3=1 timeout -k 10 300 python -u bench.py --workloads 0 --cpu-baseline 0 > gpurun_out/r6l/bench_p3.json 2> gpurun_out/r6l/bench_p3.err || exit 1
