set -e
mkdir -p gpurun_out/ks
VAEVAR_H3_KS=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ks/h3_off.log 2>&1
TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ks/h3_on.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ks/b_on.json 2> gpurun_out/ks/b_on.err
VAEVAR_H3_KS=1 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ks/b_off.json 2> gpurun_out/ks/b_off.err
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ks/tests.log 2>&1
