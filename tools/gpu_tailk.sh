# tail split-K chunk threshold A/B (VAEVAR_TAIL_MINKT 12 / 9: S = 3 / 4 at K = 1152; 18 / 40 measured too), config-2 lines
# interleaved twice, plus the per-shape GEMM times at 2048 rows
set -e
T=${1:-tailk}
mkdir -p gpurun_out/$T
for R in 1 2; do
  for K in 12 9; do
    VAEVAR_TAIL_MINKT=$K timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-sc4dvar >> gpurun_out/$T/c2_t$K.json 2>/dev/null
  done
done
for K in 12 9; do
  VAEVAR_TAIL_MINKT=$K TILES=-1 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m1_t$K.jsonl 2>&1
done
