# per-shape kernel traces of the config-2 closure (tools/quick_time.py) under two settings of one tuning knob, on
# one box; usage: bash tools/gpu_trace_ab.sh TAG KEY VA VB  -> gpurun_out/TAG/shapes_KEY_V.txt, qt_KEY_V.log
set -e
T=$1; KEY=$2; shift 2
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
ENVK=VAEVAR_$(echo $KEY | tr a-z A-Z)
for V in "$@"; do
  rm -rf /tmp/kt_$V
  env $ENVK=$V timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_$V -o run -- python tools/quick_time.py > gpurun_out/$T/qt_${KEY}_$V.log 2>&1
  python tools/trace_shapes.py $(find /tmp/kt_$V -name "*kernel_trace.csv" | head -1) > gpurun_out/$T/shapes_${KEY}_$V.txt
done
