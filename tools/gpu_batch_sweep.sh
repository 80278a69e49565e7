# analyses per GPU B = 1, 2, 4, 8 for config 2 and config 4 (one GPU); usage: bash tools/gpu_batch_sweep.sh TAG
set -e
T=${1:-bsw}
mkdir -p gpurun_out/$T
for B in 1 2 4 8; do
  timeout -k 10 300 python bench.py --batch $B --steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-config5 > gpurun_out/$T/c2_b$B.json 2> gpurun_out/$T/c2_b$B.err
done
for B in 1 2 4 8; do
  timeout -k 10 400 python bench.py --config 4 --batch $B --steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile > gpurun_out/$T/c4_b$B.json 2> gpurun_out/$T/c4_b$B.err
done
