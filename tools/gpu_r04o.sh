# r04: tile-48 gathered scales (h4_gather) + batched-scalar bitwise test: focused tests, closure A/B
set -e
mkdir -p gpurun_out/r04o
rc=0
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "bitwise_knobs or batched_scalars or config2_traj or fixup_ln or ln_planes or gelu_planes or g3" > gpurun_out/r04o/focus.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do for v in 0 1; do
  VAEVAR_H4_GATHER=$v T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04o/qt.log 2>&1 && (echo "h4_gather $v"; grep closure gpurun_out/r04o/qt.log) >> gpurun_out/r04o/ab.log
done; done
