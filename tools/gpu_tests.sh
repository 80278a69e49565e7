# GPU test suite (verbose, per-test timeout) + smoke; usage: bash tools/gpu_tests.sh TAG [pytest -k expr]
set -e
T=${1:-chk}
K=${2:-}
mkdir -p gpurun_out/$T
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$T/gpu_tests.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
