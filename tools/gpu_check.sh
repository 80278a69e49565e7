# GPU tests + one bench line (no CPU baseline); usage: bash tools/gpu_check.sh TAG
set -e
T=${1:-chk}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
