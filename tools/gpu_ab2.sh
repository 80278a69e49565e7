set -e
mkdir -p gpurun_out/ab2
for i in 1 2; do
VAEVAR_SMALL_SPLIT_MINKT=12 timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab2/m12_$i.json 2>/dev/null
VAEVAR_SMALL_SPLIT_MINKT=24 timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab2/m24_$i.json 2>/dev/null
VAEVAR_SMALL_SPLIT=0 timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab2/off_$i.json 2>/dev/null
done
