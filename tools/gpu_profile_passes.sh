# rocprofv3 --kernel-trace --stats of bench.py and separate --pmc FETCH_SIZE / WRITE_SIZE passes (the second half of
# round_profile.sh, for when the bench line was taken in its own call); usage: bash tools/gpu_profile_passes.sh TAG
set -e
TAG=${1:-run}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp -o run -- python bench.py --no-cpu-baseline > $OUT/rp.log 2>&1
echo "rocprof done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o run -- python bench.py --steps 2 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar > $OUT/pf.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o run -- python bench.py --steps 2 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar > $OUT/pw.log 2>&1
echo "pmc done"
python tools/pmc_traffic.py $(find $OUT/pf -name "*counter_collection.csv") $(find $OUT/pw -name "*counter_collection.csv") $OUT/gemm_traffic.json > /dev/null
python tools/rocprof_gemm_summary.py $(find $OUT/rp -name "*kernel_stats.csv") $OUT/gemm_rocprof_summary.json > /dev/null
find $OUT/rp -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/rp $OUT/pf $OUT/pw
echo "ok"
