# same-box A/B: ping-pong kernel for sub-chip fp16x3 GEMMs (dev)
set -e
mkdir -p gpurun_out/ab7
TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab7/h3_base.log 2>&1
VAEVAR_PINGPONG=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab7/h3_pp.log 2>&1
VAEVAR_PINGPONG=1 VAEVAR_SMALL_SPLIT=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab7/h3_pp_nosplit.log 2>&1
for i in 1 2; do
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab7/base_$i.json 2>/dev/null
VAEVAR_PINGPONG=1 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab7/pp_$i.json 2>/dev/null
VAEVAR_PINGPONG=1 VAEVAR_SMALL_SPLIT=0 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab7/ppns_$i.json 2>/dev/null
done
