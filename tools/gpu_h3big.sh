# 256x128 fp16x3 tile (44) vs 128x128 (36): kernel tests, per-shape times at 2048 / 8192 / 16384 rows, and
# config-2 / batch-8 bench lines per VAEVAR_H3_BIG routing threshold; usage: bash tools/gpu_h3big.sh TAG
set -e
T=${1:-h3big}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
TILES=36,44 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m1.jsonl 2>&1
MROWS=4 TILES=36,44 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m4.jsonl 2>&1
MROWS=8 TILES=36,44 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m8.jsonl 2>&1
for B in 0 200 100; do
  VAEVAR_H3_BIG=$B timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 > gpurun_out/$T/c2_big$B.json 2> gpurun_out/$T/c2_big$B.err
  VAEVAR_H3_BIG=$B timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 > gpurun_out/$T/c2b8_big$B.json 2> gpurun_out/$T/c2b8_big$B.err
done
