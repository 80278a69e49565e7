# r04 records: full GPU suite + smoke, then bench + rocprof stats + PMC traffic (tools/round_profile.sh)
set -e
bash tools/gpu_tests.sh r04n
bash tools/round_profile.sh r04n
