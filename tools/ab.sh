set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/gpu_tests.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab/cur44.json 2> gpurun_out/ab/cur44.err
(cd ab_head && timeout -k 10 240 python bench.py --no-cpu-baseline > ../gpurun_out/ab/head.json 2> ../gpurun_out/ab/head.err)
VAEVAR_F16_KERNEL=36 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab/cur36.json 2> gpurun_out/ab/cur36.err
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab/cur44b.json 2> gpurun_out/ab/cur44b.err
