# r04: the full GPU suite + smoke at the final HEAD
set -e
bash tools/gpu_tests.sh r04ac
