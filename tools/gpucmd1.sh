set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu1.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu1.txt
timeout -k 10 300 python tools/quick_bench.py > gpurun_out/quick_bench1.txt 2>&1
echo "bench rc=$?" >> gpurun_out/quick_bench1.txt
