# PMC passes over the kernels matching REGEX in one program: bash tools/pmc_kernel.sh REGEX TAG python3 prog.py ...
# Writes gpurun_out/pmc_k/TAG/summary.txt (per-kernel means of each counter).
set -e
RE=$1; TAG=$2
shift 2
OUT=$PWD/gpurun_out/pmc_k/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$RE" --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
done
python3 - "$OUT" <<'PY'
import glob, sys, csv, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        key = n.split("(")[0][-60:] + " grid " + r.get("Grid_Size", "")
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{out}/summary.txt", "w") as fh:
    for k, d in agg.items():
        fh.write(k + " " + str({c: f"{sum(v)/len(v):.4g}" for c, v in d.items()}) + "\n")
PY
rm -rf $OUT/p1 $OUT/p2 $OUT/p3
