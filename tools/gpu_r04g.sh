set -e
mkdir -p gpurun_out/r04g
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_config4.py tests/test_gpu_fcst.py -x -v --timeout 200 --timeout-method thread -k "g1 or g3 or g5b or h5 or t6_closure or g12 or fcst or integrate" > gpurun_out/r04g/tests.log 2>&1
timeout -k 10 300 python tools/fcst_time.py > gpurun_out/r04g/fcst_on.log 2>&1
VAEVAR_FC_CONV_MF=0 timeout -k 10 300 python tools/fcst_time.py > gpurun_out/r04g/fcst_off.log 2>&1
cd /tmp && export TMPDIR=/tmp
T=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04g/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04g/qt.log 2>&1
N=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04g/proff -o run -- python3 $GRAFT_REPO_ROOT/tools/fcst_time.py > $GRAFT_REPO_ROOT/gpurun_out/r04g/fcst_prof.log 2>&1
