# same-box A/B of one build under two environments: A="VAR=x" B="VAR=y" bash tools/gpu_abenv.sh TAG [bench args]
set -e
T=${1:-abenv}
shift || true
mkdir -p gpurun_out/$T
for i in 1 2; do
  env $A timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --no-exact-f32 --no-config4 --no-sc4dvar --steps 2 "$@" > gpurun_out/$T/a_$i.json 2>/dev/null
  env $B timeout -k 10 240 python bench.py --no-cpu-baseline --no-profile --no-exact-f32 --no-config4 --no-sc4dvar --steps 2 "$@" > gpurun_out/$T/b_$i.json 2>/dev/null
done
