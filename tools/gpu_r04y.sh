# r04 final records at HEAD: full GPU suite + smoke, then bench + rocprof stats + PMC traffic
set -e
bash tools/gpu_tests.sh r04y
bash tools/round_profile.sh r04y
