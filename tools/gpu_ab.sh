# same-box A/B of GEMM routing thresholds (dev)
set -e
mkdir -p gpurun_out/ab6
for i in 1 2; do
for k in 768 384 192; do
VAEVAR_H3_MINK=$k timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab6/k${k}_$i.json 2>/dev/null
done
done
VAEVAR_H3_MINK=96 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab6/k96_1.json 2>/dev/null
