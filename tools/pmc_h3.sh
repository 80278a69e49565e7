# PMC passes over one fp16x3 GEMM shape (dev tool): bash tools/pmc_h3.sh M N K TAG  (env VAEVAR_SK etc. pass through)
set -e
M=$1; N=$2; K=$3; TAG=$4
OUT=$PWD/gpurun_out/pmc_h3/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PRE=1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p1 -o run -- python tools/gemm_one.py $M $N $K ${TILE:-36} 40 > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/gemm_one.py $M $N $K ${TILE:-36} 40 > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python tools/gemm_one.py $M $N $K ${TILE:-36} 40 > $OUT/kt.log 2>&1
python tools/pmc_summary_h3.py $OUT > $OUT/summary.txt
rm -rf $OUT/p1 $OUT/p2 $OUT/kt
