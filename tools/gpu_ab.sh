# same-box A/B (dev): current build vs the reference .so in vae-var_amd/vaevar/libvaevar_ref.so
set -e
mkdir -p gpurun_out/ab10; rm -f gpurun_out/ab10/*
R=$PWD/vae-var_amd/vaevar/libvaevar_ref.so
for i in 1 2 3; do
VAEVAR_LIB=$R timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab10/ref_$i.json 2>/dev/null
timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab10/new_$i.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_obs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab10/tests.log 2>&1
