# r04: tile-49 LDS epilogue + mlp_hc A/B; usage: bash tools/gpu_r04i.sh
set -e
mkdir -p gpurun_out/r04i
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "h5 or fused_tower or config2_traj or gelu_planes" > gpurun_out/r04i/focus.log 2>&1
for hc in 32 64 2 32 64 2; do
  VAEVAR_MLP_HC=$hc T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04i/qt_hc$hc.log 2>&1 && (echo "mlp_hc $hc"; cat gpurun_out/r04i/qt_hc$hc.log) >> gpurun_out/r04i/qt_all.log
done
for v in 5 4 5 4; do
  VAEVAR_H5_VAR=$v T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04i/qt_v$v.log 2>&1 && (echo "h5_var $v"; cat gpurun_out/r04i/qt_v$v.log) >> gpurun_out/r04i/qt_all.log
done
cd /tmp && export TMPDIR=/tmp
VAEVAR_MLP_HC=2 T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04i/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04i/qt_prof.log 2>&1
VAEVAR_FUSE_ATTN=3 T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04i/prof_fa3 -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04i/qt_fa3.log 2>&1
