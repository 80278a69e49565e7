# PMC passes over one GEMM shape / tile (dev tool): bash tools/pmc_gemm.sh M N K TILE
export TMPDIR=/tmp
M=${1:-2048}; N=${2:-3456}; K=${3:-1152}; T=${4:-21}
out=gpurun_out/pmc_${M}_${N}_${K}_t$T
mkdir -p $out
export PRE=1
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $out/p$i -o run -- python tools/gemm_one.py $M $N $K $T 20 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python tools/pmc_summary.py gemm $(find $out -name "*counter_collection.csv")
