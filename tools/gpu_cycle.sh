set -e
mkdir -p gpurun_out/cyc
timeout -k 10 400 python -u -m pytest tests/test_gpu_cycle.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/cyc/tests.log 2>&1
