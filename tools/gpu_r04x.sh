# r04: analyses per GPU (--batch B) at HEAD: config 2 B = 1, 2, 4, 8; config 4 B = 1, 4, 8
set -e
mkdir -p gpurun_out/r04x
X="--steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config3 --no-config4 --no-config5 --no-sc4dvar"
for B in 1 2 4 8; do
  timeout -k 10 300 python bench.py --batch $B $X > gpurun_out/r04x/c2_b$B.json 2> gpurun_out/r04x/c2_b$B.err
done
for B in 1 4 8; do
  timeout -k 10 400 python bench.py --config 4 --batch $B $X > gpurun_out/r04x/c4_b$B.json 2> gpurun_out/r04x/c4_b$B.err
done
