# per-launch kernel trace of the config-2 closure (tools/quick_time.py) for per-shape timing of the small
# kernels (attention, LayerNorm, tower GEMMs); usage: bash tools/gpu_trace_shapes.sh TAG
set -e
T=${1:-trace}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- python tools/quick_time.py > gpurun_out/$T/qt.log 2>&1
f=$(find /tmp/kt -name "*kernel_trace.csv" | head -1)
python tools/trace_shapes.py "$f" > gpurun_out/$T/shapes.txt
