# tile 25 (register-blocked short K): kernel tests, tower-shape timings, G1/G3 parity, same-box bench A/B vs REF
set -e
T=${1:-rb}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -s --timeout 250 --timeout-method thread -k "short_k or rejects" > gpurun_out/$T/tests.log 2>&1
TILES=24,25 timeout -k 10 200 python tools/tower_gemm_bench.py > gpurun_out/$T/tow.jsonl 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "g1 or g3 or ln_row" > gpurun_out/$T/parity.log 2>&1
REF=$PWD/vae-var_amd/vaevar/libvaevar_ref.so bash tools/gpu_ab2.sh ${T}_ab
