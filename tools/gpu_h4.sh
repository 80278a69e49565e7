# tile 48 (split-operand LDS-DMA fp16x3 kernel) vs 47 / 44 / 36: kernel tests, per-shape times at 2048 / 16384
# rows, and a rocprofv3 kernel trace of the same bench; usage: bash tools/gpu_h4.sh TAG
set -e
T=${1:-h4}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 250 --timeout-method thread -k "gemm" > gpurun_out/$T/tests.log 2>&1
echo tests-ok
TILES=47,48,44,36 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m1.jsonl 2>&1
MROWS=8 TILES=47,48,44 timeout -k 10 200 python tools/h3_bench.py > gpurun_out/$T/m8.jsonl 2>&1
echo bench-ok
TILES=47,48 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/$T/rp -o run -- python tools/h3_bench.py > gpurun_out/$T/rp.log 2>&1
find gpurun_out/$T/rp -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/kernel_stats.csv \;
rm -rf gpurun_out/$T/rp
echo ok
