# r04: full suite with the branch-free GELU + mlp_hc 2 defaults; A/Bs: erff build vs fast GELU, fuse_attn 1 vs 3
set -e
bash tools/gpu_tests.sh r04j
for i in 1 2; do
  for lib in ab/libvaevar_erff.so libvaevar.so; do
    VAEVAR_LIB=$PWD/vae-var_amd/vaevar/$lib T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04j/qt.log 2>&1 && (echo "lib $lib"; grep closure gpurun_out/r04j/qt.log) >> gpurun_out/r04j/ab.log
  done
  for fa in 1 3; do
    VAEVAR_FUSE_ATTN=$fa T=1 timeout -k 10 120 python3 tools/quick_time.py > gpurun_out/r04j/qt.log 2>&1 && (echo "fuse_attn $fa"; grep closure gpurun_out/r04j/qt.log) >> gpurun_out/r04j/ab.log
  done
done
cd /tmp && export TMPDIR=/tmp
T=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04j/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04j/qt_prof.log 2>&1
