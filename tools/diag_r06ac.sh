# r06ac: fused fixup + LayerNorm with the row's own loads issued before the partial staging (fixup_stage 2, tile 49):
# bitwise against fixup_stage 1, then a same-process closure A/B.
set -e
TAG=${1:-r06ac}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "bitwise_knobs and fixup_stage" > $OUT/tests.log 2>&1
echo "tests done"; grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -4
timeout -k 10 400 python tools/knob_ab.py --reps 3 default fixup_stage=2 default fixup_stage=2 > $OUT/knob_ab_fixup_stage.jsonl 2> $OUT/knob_ab.err
python - $OUT/knob_ab_fixup_stage.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print(r["setting"], round(r["ms_min"],3), round(r["ms_median"],3), r["class_ms_per_eval"].get("layernorm"), r["class_ms_per_eval"].get("gemm16"))
PY
echo ok
