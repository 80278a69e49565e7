# whole-grid split-K floor for the sub-chip fp16x3 GEMMs (VAEVAR_SMALL_SPLIT_MINKT 24 / 18 / 12: K = 1152 shapes
# unsplit / S = 2 / S = 3), config-2 lines interleaved twice
set -e
T=${1:-smallk}
mkdir -p gpurun_out/$T
for R in 1 2; do
  for K in 24 18 12; do
    VAEVAR_SMALL_SPLIT_MINKT=$K timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-sc4dvar >> gpurun_out/$T/c2_s$K.json 2>/dev/null
  done
done
