# r06v: tile 49 gathers the producer's row scales itself (h4_gather): GEMM + bitwise-knob tests, a same-process
# A/B against h4_gather=0 (the separate gather-scales launch) and the eager closure's kernel list.
set -e
TAG=${1:-r06v}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "gemm or bitwise or h5 or fixup or gather" > $OUT/tests.log 2>&1
echo "tests done"; grep -cE "PASSED" $OUT/tests.log; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -3
timeout -k 10 400 python tools/knob_ab.py --reps 3 default h4_gather=0 > $OUT/knob_ab_h4_gather.jsonl 2> $OUT/knob_ab.err
echo "knob ab done"; cut -c1-300 $OUT/knob_ab_h4_gather.jsonl
VAEVAR_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ct -o run -- python tools/closure_ktrace.py > $OUT/ct.log 2>&1
python tools/closure_ktrace.py --analyse $(find $OUT/ct -name "*kernel_trace.csv" | head -1) > $OUT/closure_kernels.txt
rm -rf $OUT/ct
grep -iE "gather|closure|total" $OUT/closure_kernels.txt | head -20
echo ok
