# one bench line (+ optional extra args) and a rocprofv3 --stats profile of the same command; usage:
#   bash tools/gpu_bench.sh TAG [bench args...]
set -e
T=${1:-b}
shift || true
mkdir -p gpurun_out/$T
timeout -k 10 600 python bench.py "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-config4 --no-config5 --no-exact-f32 --no-profile --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/$T/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$T/prof.err
