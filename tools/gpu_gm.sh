# tile-grouping check (dev): h3_bench + a FETCH_SIZE pass per LG shape class with the current build
set -e
O=gpurun_out/tile_group; mkdir -p $O
export TMPDIR=/tmp
TILES=-1 timeout -k 10 120 python -u tools/h3_bench.py > $O/h3.jsonl 2>&1
for s in "2048 3456 1152" "2048 1152 4608" "2048 1152 1152" "2048 4608 1152"; do
  set -- $s
  PRE=1 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p_$1_$2_$3 -o run -- python tools/gemm_one.py $1 $2 $3 -1 20 > $O/p_$1_$2_$3.log 2>&1
done
