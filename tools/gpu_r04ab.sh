# r04: fused-MLP weight blocks padded by 64 B in LDS: tests + kernel A/B against the unpadded build (same box)
set -e
mkdir -p gpurun_out/r04ab
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "fused_tower or config2_traj or config3_traj or g3 or swin or tiny" > gpurun_out/r04ab/focus.log 2>&1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for lib in ab/libvaevar_pad0.so libvaevar.so; do
  tag=$(basename $lib .so)_$i
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04ab/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04ab/qt_$tag.log 2>&1
done
done
