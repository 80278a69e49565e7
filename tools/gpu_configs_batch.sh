# bench lines for configs 3 / 4 / 5 and the batched config-2 / config-4 lines (1 GPU) on the current tree
set -e
bash tools/gpu_configs.sh
timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-config5 --no-sc4dvar > gpurun_out/cfg/c2_b8.json 2> gpurun_out/cfg/c2_b8.err
echo c2b8
timeout -k 10 400 python bench.py --config 4 --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-sc4dvar > gpurun_out/cfg/c4_b8.json 2> gpurun_out/cfg/c4_b8.err
echo c4b8
