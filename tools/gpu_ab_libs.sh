# same-box A/B of several library builds (bisecting a regression): bash tools/gpu_ab_libs.sh TAG lib1.so lib2.so ...
# ("head" = the in-tree build); each library's short bench twice, interleaved
set -e
T=$1
shift
mkdir -p gpurun_out/$T
for i in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    if [ "$L" = head ]; then unset VAEVAR_LIB; else export VAEVAR_LIB=$PWD/$L; fi
    timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --no-exact-f32 --no-config4 --no-config5 --steps 2 > gpurun_out/$T/${n}_$i.json 2>/dev/null
    python -c "import json,sys;b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], round(b['value'],2), round(b['ms_per_eval'],3))" gpurun_out/$T/${n}_$i.json
  done
done
