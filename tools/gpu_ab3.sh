set -e
mkdir -p gpurun_out/ab3
VAEVAR_SMALL_SPLIT_MINKT=18 ERR=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab3/h3_18.log 2>&1
ERR=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab3/h3_24.log 2>&1
for i in 1 2; do
VAEVAR_SMALL_SPLIT_MINKT=18 timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab3/m18_$i.json 2>/dev/null
timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab3/m24_$i.json 2>/dev/null
done
