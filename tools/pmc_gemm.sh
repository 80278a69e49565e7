# PMC passes over one fp16x3 GEMM shape for several tiles: bash tools/pmc_gemm.sh M N K TAG TILES...
set -e
M=$1; N=$2; K=$3; TAG=$4
shift 4
for T in "$@"; do
OUT=$PWD/gpurun_out/pmc_h3/${TAG}_t$T
mkdir -p $OUT
export TMPDIR=/tmp PRE=1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p1 -o run -- python tools/gemm_one.py $M $N $K $T 40 > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/gemm_one.py $M $N $K $T 40 > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- python tools/gemm_one.py $M $N $K $T 40 > $OUT/p3.log 2>&1 || true
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python tools/gemm_one.py $M $N $K $T 40 > $OUT/kt.log 2>&1
python tools/pmc_summary_h3.py $OUT > $OUT/summary.txt
python - "$OUT" <<'PY'
import glob, sys, csv, collections
out = sys.argv[1]
f = glob.glob(f"{out}/p3/**/*counter_collection.csv", recursive=True)
if f:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    with open(f"{out}/summary.txt", "a") as fh:
        for k, d in agg.items():
            fh.write(f"p3 {k} " + str({c: f"{sum(v)/len(v):.4g}" for c, v in d.items()}) + "\n")
PY
rm -rf $OUT/p1 $OUT/p2 $OUT/p3 $OUT/kt
done
