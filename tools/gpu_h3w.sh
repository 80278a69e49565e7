# the 128x64-per-wave fp16x3 kernel (tile 45) vs 36 / 44: kernel tests, then per-shape times at 2048 / 8192 / 16384 rows
set -e
T=${1:-h3w}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 250 --timeout-method thread -k "split16 or splitk or rejects or resample" > gpurun_out/$T/tests.log 2>&1
TILES=36,44,45 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m1.jsonl 2>&1
MROWS=4 TILES=36,44,45 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m4.jsonl 2>&1
MROWS=8 TILES=36,44,45 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m8.jsonl 2>&1
