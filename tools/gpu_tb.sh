set -e
T=${1:-tb}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
