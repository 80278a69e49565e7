set -e
mkdir -p gpurun_out/r04e
H5_VARS=3,4 timeout -k 10 200 python tools/h5_check.py > gpurun_out/r04e/h5.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -v --timeout 200 --timeout-method thread -k "g1 or g3 or g5b or t6_closure or g12 or dropin" > gpurun_out/r04e/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
T=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04e/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04e/qt.log 2>&1
