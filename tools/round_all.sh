# full GPU test suite, then bench + rocprof stats + PMC traffic (tools/round_profile.sh)
set -e
TAG=${1:-run}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/prof_$TAG/gpu_tests.log 2>&1
echo "tests done"
bash tools/round_profile.sh $TAG
