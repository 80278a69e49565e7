# same-box A/B of two library builds: REF=<path to the other .so> bash tools/gpu_ab_lib.sh TAG [bench args]
set -e
T=${1:-ab}
shift || true
mkdir -p gpurun_out/$T
for i in 1 2; do
  VAEVAR_LIB=$REF timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --no-exact-f32 --no-config4 --no-config5 --steps 2 "$@" > gpurun_out/$T/ref_$i.json 2>/dev/null
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --no-exact-f32 --no-config4 --no-config5 --steps 2 "$@" > gpurun_out/$T/new_$i.json 2>/dev/null
done
