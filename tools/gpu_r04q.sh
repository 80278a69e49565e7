# r04: tile-49 row epilogue with 16-byte plane stores: bitwise tests + kernel A/B against the previous build
set -e
mkdir -p gpurun_out/r04q
rc=0
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "bitwise_knobs or h5 or gelu_planes or config2_traj or g3" > gpurun_out/r04q/focus.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for lib in ab/libvaevar_prev.so libvaevar.so; do
  tag=$(basename $lib .so)
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04q/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04q/qt_$tag.log 2>&1
done
cd $GRAFT_REPO_ROOT
for i in 1 2; do for lib in ab/libvaevar_prev.so libvaevar.so; do
  VAEVAR_LIB=$PWD/vae-var_amd/vaevar/$lib T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04q/qt.log 2>&1 && (echo "lib $lib"; grep closure gpurun_out/r04q/qt.log) >> gpurun_out/r04q/ab.log
done; done
