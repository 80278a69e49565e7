# r04: speculative line-search start (deferred gtd / d_norm): L-BFGS tests, then config-2 bench A/B
set -e
mkdir -p gpurun_out/r04w
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "trajectory or lbfgs or one_step or sc4dvar or batch or reduce_batch" > gpurun_out/r04w/focus.log 2>&1
B="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar"
for i in 1 2; do for v in 0 1; do
  VAEVAR_LBFGS_SPECULATE=$v timeout -k 10 300 python3 bench.py $B > gpurun_out/r04w/c2_s${v}_$i.json 2> gpurun_out/r04w/c2_s${v}_$i.err
done; done
