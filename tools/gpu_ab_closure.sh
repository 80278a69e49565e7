# same-box closure A/B of library builds, interleaved 3 times: bash tools/gpu_ab_closure.sh OUT lib1.so ... head
set -e
O=$1
shift
mkdir -p $(dirname $O)
: > $O
for i in 1 2 3; do
  for L in "$@"; do
    if [ "$L" = head ]; then unset VAEVAR_LIB; else export VAEVAR_LIB=$PWD/$L; fi
    timeout -k 10 180 python tools/closure_time.py >> $O
  done
done
cat $O
