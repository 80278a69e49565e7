# Same-box sweep of one per-context tuning knob (vaevar.engine.Context.TUNING_KEYS, applied from VAEVAR_<KEY>):
# config-2 bench lines for every value, interleaved twice.  usage: bash tools/gpu_sweep.sh TAG KEY V1 V2 ... [-- bench args]
# (regenerates profiles/r02/mink: KEY h3_mink 768 384 192 96; smallk: small_split_minkt 24 18 12;
#  tailk: tail_minkt 12 9 18 40; h3big: h3_big 1 0)
set -e
T=$1; KEY=$2; shift 2
VALS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VALS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
ENVK=VAEVAR_$(echo $KEY | tr a-z A-Z)
mkdir -p gpurun_out/$T
for R in 1 2; do
  for V in "${VALS[@]}"; do
    env $ENVK=$V timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact-f32 --no-profile \
      --no-config3 --no-config4 --no-config5 --no-sc4dvar "$@" >> gpurun_out/$T/c2_${KEY}_$V.json 2>> gpurun_out/$T/c2_${KEY}_$V.err
  done
done
