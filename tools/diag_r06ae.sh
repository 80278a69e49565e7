# r06ae: tile 49 reading gathered producer row scales itself as a compile-time kernel form (k_gemm_h5<EPI, true>):
# GEMM + bitwise tests, same-box bench A/B against the previous library, the eager closure's kernel list.
set -e
TAG=${1:-r06ae}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "gemm or bitwise or h5 or fixup or gather" > $OUT/tests.log 2>&1
echo "tests done"; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -3
bash tools/gpu_ab_libs.sh ${TAG}_ab ab_head/lib_base.so head ab_head/lib_base.so head
VAEVAR_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ct -o run -- python tools/closure_ktrace.py > $OUT/ct.log 2>&1
python tools/closure_ktrace.py --analyse $(find $OUT/ct -name "*kernel_trace.csv" | head -1) > $OUT/closure_kernels.txt
rm -rf $OUT/ct
grep -E "one closure|gather|k_gemm_h5" $OUT/closure_kernels.txt | head -12
echo ok
