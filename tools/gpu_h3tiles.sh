# fp16x3 tile variants on the LG shapes (dev); usage: bash tools/gpu_h3tiles.sh TAG
set -e
T=${1:-h3t}
mkdir -p gpurun_out/$T
TILES=-1,36,40,41,42 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/split_on.jsonl 2>&1
VAEVAR_SMALL_SPLIT=0 TILES=36,40,41,42 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/split_off.jsonl 2>&1
MROWS=4 TILES=36,40,41,42 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m4.jsonl 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
