set -e
mkdir -p gpurun_out/ab4
R=$PWD/vae-var_amd/vaevar/libvaevar_ref.so
VAEVAR_LIB=$R ERR=0 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab4/h3_ref.log 2>&1
ERR=1 TILES=36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/ab4/h3_new.log 2>&1
for i in 1 2; do
VAEVAR_LIB=$R timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab4/ref_$i.json 2>/dev/null
timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab4/new_$i.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab4/kt.log 2>&1
