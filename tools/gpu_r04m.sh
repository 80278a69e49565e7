# r04: batched L-BFGS scalars + interleaved GELU: focused GPU tests, config-2 bench x2, GELU kernel A/B (rocprof)
set -e
mkdir -p gpurun_out/r04m
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "trajectory or lbfgs or one_step or sc4dvar or fused_tower or h5 or gelu or g3 or tiny or closure" > gpurun_out/r04m/focus.log 2>&1 || rc=$?
# test failures (1) do not stop the measurements; a crash, fault or time-out does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-config3 --no-config4 --no-config5 --no-exact-f32 --no-sc4dvar"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $B > gpurun_out/r04m/c2_$i.json 2> gpurun_out/r04m/c2_$i.err
done
for i in 1 2; do for fa in 3 15 7; do
  VAEVAR_FUSE_ATTN=$fa T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04m/qt.log 2>&1 && (echo "fuse_attn $fa"; grep closure gpurun_out/r04m/qt.log) >> gpurun_out/r04m/ab.log
done; done
cd /tmp && export TMPDIR=/tmp
for lib in ab/libvaevar_erff.so libvaevar.so; do
  tag=$(basename $lib .so)
  VAEVAR_LIB=$GRAFT_REPO_ROOT/vae-var_amd/vaevar/$lib T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04m/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04m/qt_$tag.log 2>&1
done
cd $GRAFT_REPO_ROOT
T=1 bash tools/pmc_kernel.sh "k_mlp|k_ablk" tower python3 tools/quick_time.py
