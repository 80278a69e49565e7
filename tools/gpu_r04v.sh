# r04: reduce_batch test + L-BFGS paths
set -e
mkdir -p gpurun_out/r04v
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "reduce_batch or lbfgs or vector or two_loop or one_step" > gpurun_out/r04v/focus.log 2>&1
