# A/B of the fp16x3 GEMM variants on the LG shapes (same box); usage: bash tools/gpu_h3ab.sh TAG
set -e
T=${1:-h3ab}
mkdir -p gpurun_out/$T
for i in 1 2; do
VAEVAR_H3_APRE=0 timeout -k 10 120 python tools/h3_bench.py > gpurun_out/$T/split_$i.jsonl 2>&1
VAEVAR_H3_APRE=1 timeout -k 10 120 python tools/h3_bench.py > gpurun_out/$T/apre_$i.jsonl 2>&1
done
MROWS=4 VAEVAR_H3_APRE=1 timeout -k 10 120 python tools/h3_bench.py > gpurun_out/$T/apre_m4.jsonl 2>&1
VAEVAR_H3_APRE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-config4 --no-exact-f32 > gpurun_out/$T/bench_split.json 2>/dev/null
VAEVAR_H3_APRE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-config4 --no-exact-f32 > gpurun_out/$T/bench_apre.json 2>/dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "gemm or g3 or g5 or graph" > gpurun_out/$T/tests.log 2>&1
