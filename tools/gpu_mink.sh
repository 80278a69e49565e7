# fp16x3 routing threshold A/B now that LayerNorm supplies the qkv / fc1 row scales in every stage:
# config-2 bench lines per VAEVAR_H3_MINK (smallest K sent to the fp16x3 kernel), interleaved twice
set -e
T=${1:-mink}
mkdir -p gpurun_out/$T
for R in 1 2; do
  for K in 768 384 192 96; do
    VAEVAR_H3_MINK=$K timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-sc4dvar >> gpurun_out/$T/c2_k$K.json 2>> gpurun_out/$T/c2_k$K.err
  done
done
