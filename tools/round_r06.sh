# The round-end evidence of r06 on the GPU box (run via gpurun from the repo root), each GPU step under its own time
# limit, stopping at the first failure (set -e):
#   GPU suite with the parity-margin records, smoke(), the default bench line, rocprofv3 --kernel-trace --stats of the
#   bench (kernel_stats + the fp16x3 per-call summary), FETCH_SIZE / WRITE_SIZE passes (GEMM traffic), the MFMA-busy /
#   held-clock passes (tools/pmc_mfma.py) and the kernel-outlier trace (tools/ktrace_outliers.py).
# Usage: VV_HEAD=<commit> bash tools/round_r06.sh TAG   -> gpurun_out/TAG/...
set -e
TAG=${1:-r06q}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export VV_MARGINS=$OUT/parity_margins.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
echo "tests done"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke done"
timeout -k 10 420 python bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench done"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp -o run -- python bench.py --no-cpu-baseline > $OUT/rp.log 2>&1
echo "rocprof done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python bench.py --steps 2 --no-cpu-baseline --no-profile --no-config5 > $OUT/pf.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python bench.py --steps 2 --no-cpu-baseline --no-profile --no-config5 > $OUT/pw.log 2>&1
echo "pmc traffic done"
python tools/pmc_traffic.py $(find $OUT/pf -name "*counter_collection.csv") $(find $OUT/pw -name "*counter_collection.csv") $OUT/gemm_traffic.json > /dev/null
python tools/rocprof_gemm_summary.py $(find $OUT/rp -name "*kernel_stats.csv") $OUT/gemm_rocprof_summary.json > /dev/null
find $OUT/rp -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python tools/ktrace_outliers.py $(find $OUT/rp -name "*kernel_trace.csv") > $OUT/outliers.txt
rm -rf $OUT/rp $OUT/pf $OUT/pw
timeout -k 10 700 python tools/pmc_mfma.py $OUT/pmc > $OUT/pmc_mfma.log 2>&1
echo "pmc mfma done"
echo "ok"
