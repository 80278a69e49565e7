# r06g: the persistent patch kernels (patch_pers): bitwise tests at the decoder's and the flow's shapes, the config-4
# T=6 closure vs the oracle (the r06e failure: the 112-tap weight staging ran past its rows), a same-process knob A/B
# of the closure and a kernel trace. Each GPU step under its own time limit, stopping at the first failure.
set -e
TAG=${1:-r06g}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -v -s --timeout 300 \
    --timeout-method thread -k "patch_pers or test_full_t6_closure_vs_oracle" > $OUT/tests.log 2>&1
echo "tests done"; grep -E "PASSED|FAILED|config-4 T=6 closure:" $OUT/tests.log | cut -c1-220
timeout -k 10 400 python tools/knob_ab.py --reps 3 default patch_pers=0 patch_pers=2 > $OUT/knob_ab_patch_pers.jsonl 2> $OUT/knob_ab.err
echo "knob ab done"; cut -c1-300 $OUT/knob_ab_patch_pers.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp -o run -- python bench.py --steps 5 --no-cpu-baseline --no-config5 > $OUT/rp.log 2>&1
find $OUT/rp -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/rp
grep -E "p2t|t2p" $OUT/kernel_stats.csv | cut -c1-160
echo ok
