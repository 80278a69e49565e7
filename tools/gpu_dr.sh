set -e
mkdir -p gpurun_out/dr
TILES=36,40 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/dr/h3.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/dr/b36.json 2> gpurun_out/dr/b36.err
VAEVAR_F16_KERNEL=40 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/dr/b40.json 2> gpurun_out/dr/b40.err
VAEVAR_F16_KERNEL=40 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "g3 or g6" --timeout 250 --timeout-method thread > gpurun_out/dr/par40.log 2>&1
