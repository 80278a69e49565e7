# r04: kernel-level A/B of the GELU builds (rocprof, same box) + config-2 bench A/B of fuse_attn 1 / 3
set -e
mkdir -p gpurun_out/r04k
B="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar"
for i in 1 2; do
  for fa in 1 3; do
    VAEVAR_FUSE_ATTN=$fa timeout -k 10 300 python3 bench.py $B > gpurun_out/r04k/c2_fa${fa}_$i.json 2> gpurun_out/r04k/c2_fa${fa}_$i.err
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in ab/libvaevar_erff.so libvaevar.so; do
  tag=$(basename $lib .so)
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04k/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04k/qt_$tag.log 2>&1
done
