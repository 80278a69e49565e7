# r04: tile-48 row-scale placement A/B (prefetched before the k loop vs loaded in the epilogue), same box
set -e
mkdir -p gpurun_out/r04s
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
for lib in ab/libvaevar_late.so libvaevar.so; do
  tag=$(basename $lib .so)_$i
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04s/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04s/qt_$tag.log 2>&1
done
done
