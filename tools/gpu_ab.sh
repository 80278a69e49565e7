set -e
mkdir -p gpurun_out/ab5
R=$PWD/vae-var_amd/vaevar/libvaevar_ref.so
for i in 1 2; do
VAEVAR_LIB=$R timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab5/ref_$i.json 2>/dev/null
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/ab5/new_$i.json 2>/dev/null
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "g1 or g3 or batch2 or edge" --timeout 200 --timeout-method thread > gpurun_out/ab5/par.log 2>&1
