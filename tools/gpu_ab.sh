# same-box A/B (dev): k_gemm_h3 with B staged by global_load_lds (VAEVAR_H3_GLDS=1) vs default
set -e
mkdir -p gpurun_out/ab9; rm -f gpurun_out/ab9/*
ERR=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab9/h3_ref.log 2>&1
VAEVAR_H3_GLDS=1 ERR=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab9/h3_gl.log 2>&1
for i in 1 2; do
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab9/ref_$i.json 2>/dev/null
VAEVAR_H3_GLDS=1 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab9/gl_$i.json 2>/dev/null
done
VAEVAR_H3_GLDS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -k "not g6" --timeout 250 --timeout-method thread > gpurun_out/ab9/tests.log 2>&1
