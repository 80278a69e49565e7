# r06w: persistent patch kernels at up to 2 / 3 workgroups per CU (patch_pers as the cap, the kernel's residency the
# limit): bitwise tests, then a same-process A/B of the closure's patch class.
set -e
TAG=${1:-r06w}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -v --timeout 300 \
    --timeout-method thread -k "patch_pers or tuning" > $OUT/tests.log 2>&1
echo "tests done"; grep -cE "PASSED" $OUT/tests.log; grep -E "FAILED|passed|failed" $OUT/tests.log | tail -3
timeout -k 10 400 python tools/knob_ab.py --reps 3 default patch_pers=2 patch_pers=3 > $OUT/knob_ab_patch_pers.jsonl 2> $OUT/knob_ab.err
echo "knob ab done"; python - $OUT/knob_ab_patch_pers.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print(r["setting"], round(r["ms_min"],3), round(r["ms_median"],3), r["class_ms_per_eval"]["patch"])
PY
echo ok
