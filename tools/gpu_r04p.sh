# r04: MLP chunk-loop unroll A/B (rocprof kernel durations, same box) + closure timing
set -e
mkdir -p gpurun_out/r04p
cd /tmp && export TMPDIR=/tmp
for lib in ab/libvaevar_unr1.so libvaevar.so; do
  tag=$(basename $lib .so)
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04p/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04p/qt_$tag.log 2>&1
done
cd $GRAFT_REPO_ROOT
for i in 1 2; do for lib in ab/libvaevar_unr1.so libvaevar.so; do
  VAEVAR_LIB=$PWD/vae-var_amd/vaevar/$lib T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04p/qt.log 2>&1 && (echo "lib $lib"; grep closure gpurun_out/r04p/qt.log) >> gpurun_out/r04p/ab.log
done; done
