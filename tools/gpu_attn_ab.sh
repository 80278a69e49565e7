# attention workgroup size A/B (dev): libvaevar.so (256 threads) vs libvaevar_a512.so (VV_ATTN_THREADS=512):
# per-shape kernel trace of the closure, config-2 bench lines interleaved, parity tests on the variant
set -e
T=${1:-attn}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
V=$PWD/vae-var_amd/vaevar/libvaevar_a512.so
VAEVAR_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt512 -o run -- python tools/quick_time.py > gpurun_out/$T/qt512.log 2>&1
python tools/trace_shapes.py $(find /tmp/kt512 -name "*kernel_trace.csv" | head -1) > gpurun_out/$T/shapes512.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-sc4dvar >> gpurun_out/$T/c2_256.json 2>/dev/null
  VAEVAR_LIB=$V timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile --no-config4 --no-sc4dvar >> gpurun_out/$T/c2_512.json 2>/dev/null
done
VAEVAR_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fcst.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests512.log 2>&1
