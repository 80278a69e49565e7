# same-box A/B (dev): VAEVAR_H3_NOA2=0 (concat-capable h3 everywhere) vs default (A2-free h3 where possible)
set -e
mkdir -p gpurun_out/ab8
VAEVAR_H3_NOA2=0 ERR=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab8/h3_ref.log 2>&1
ERR=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab8/h3_new.log 2>&1
for i in 1 2; do
VAEVAR_H3_NOA2=0 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab8/ref_$i.json 2>/dev/null
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab8/new_$i.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -k "not g6" --timeout 250 --timeout-method thread > gpurun_out/ab8/tests.log 2>&1
