# r04: fused fixup + LN1 walking GEMM rows (fixup_ln_rows): bitwise tests + kernel A/B (knob, same box)
set -e
mkdir -p gpurun_out/r04u
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "bitwise or fixup_ln or config2_traj or g3" > gpurun_out/r04u/focus.log 2>&1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for v in 0 1; do
  VAEVAR_FIXUP_LN_ROWS=$v T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04u/prof_${v}_$i -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04u/qt_${v}_$i.log 2>&1
done; done
