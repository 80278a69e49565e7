# r06ah: k_gemm_fixup49 on 4-wave workgroups (64 tiles x 2 x 2 = 256, was 128 of 8 waves): GEMM / bitwise tests,
# same-box closure A/B against the previous library.
set -e
TAG=${1:-r06ah}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "gemm or bitwise or h5 or fixup or split" > $OUT/tests.log 2>&1
echo "tests done"; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -3
bash tools/gpu_ab_closure.sh $OUT/closure_ab.jsonl ab_head/lib_base.so head
echo ok
