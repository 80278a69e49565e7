set -e
mkdir -p gpurun_out/ss
VAEVAR_SMALL_SPLIT=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ss/h3_off.log 2>&1
TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ss/h3_on.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ss/b_on.json 2> gpurun_out/ss/b_on.err
VAEVAR_SMALL_SPLIT=0 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ss/b_off.json 2> gpurun_out/ss/b_off.err
timeout -k 10 500 python -u -m pytest tests/test_gpu_obs.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > gpurun_out/ss/tests.log 2>&1 || true
