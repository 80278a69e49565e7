# r04: tile-49 schedule variants, on/off A/B in the closure; MFMA patch kernels (parity subset + per-kernel times)
set -e
mkdir -p gpurun_out/r04f
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "g1 or g3 or g5b or h5 or rejects" > gpurun_out/r04f/tests.log 2>&1
H5_VARS=0,3,4 timeout -k 10 200 python tools/h5_check.py > gpurun_out/r04f/h5.log 2>&1
cd /tmp && export TMPDIR=/tmp
T=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04f/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04f/qt.log 2>&1
cd $GRAFT_REPO_ROOT
bash tools/gpu_sweep.sh r04f h5_var 0 4
bash tools/gpu_sweep.sh r04f h5 0 1
