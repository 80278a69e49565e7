set -e
mkdir -p gpurun_out/obs
timeout -k 10 500 python -u -m pytest tests/test_gpu_obs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/obs/tests.log 2>&1
