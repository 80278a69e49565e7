# r04: batched L-BFGS scalars + interleaved GELU: focused GPU tests, config-2 bench x2, GELU kernel A/B (rocprof)
set -e
mkdir -p gpurun_out/r04m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "trajectory or lbfgs or one_step or sc4dvar or fused_tower or h5 or gelu or g3 or tiny" > gpurun_out/r04m/focus.log 2>&1
B="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $B > gpurun_out/r04m/c2_$i.json 2> gpurun_out/r04m/c2_$i.err
done
cd /tmp && export TMPDIR=/tmp
for lib in ab/libvaevar_erff.so libvaevar.so; do
  tag=$(basename $lib .so)
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04m/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04m/qt_$tag.log 2>&1
done
