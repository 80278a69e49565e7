# r04: kernel-level A/B of the GELU builds (rocprof, same box), twice each
set -e
mkdir -p gpurun_out/r04l
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fused_tower or config2_traj or g3 or tiny or h5 or gelu_planes" > gpurun_out/r04l/focus.log 2>&1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for lib in ab/libvaevar_erff.so libvaevar.so; do
  tag=$(basename $lib .so)_$i
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04l/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04l/qt_$tag.log 2>&1
done
done
