# r06ad: the persistent patch kernels on 2- or 4-wave workgroups where 8-wave ones leave CUs idle (patch_pers 2 / 4;
# a batch-1 128 x 256 image: 64 workgroups of 8 waves): bitwise tests, then a same-process closure A/B.
set -e
TAG=${1:-r06ad}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -v --timeout 300 \
    --timeout-method thread -k "patch_pers or tuning" > $OUT/tests.log 2>&1
echo "tests done"; grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -8
timeout -k 10 400 python tools/knob_ab.py --reps 3 default patch_pers=2 patch_pers=4 default patch_pers=2 patch_pers=4 > $OUT/knob_ab_patch_waves.jsonl 2> $OUT/knob_ab.err
python - $OUT/knob_ab_patch_waves.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print(r["setting"], round(r["ms_min"],3), round(r["ms_median"],3), r["class_ms_per_eval"].get("patch"))
PY
VAEVAR_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ct -o run -- python tools/closure_ktrace.py > $OUT/ct.log 2>&1
python tools/closure_ktrace.py --analyse $(find $OUT/ct -name "*kernel_trace.csv" | head -1) > $OUT/closure_kernels.txt
rm -rf $OUT/ct
grep -E "p2t|t2p|one closure" $OUT/closure_kernels.txt | head -12
echo ok
