set -e
mkdir -p gpurun_out/win
timeout -k 10 400 python -u -m pytest tests/test_gpu_fcst.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/win/tests.log 2>&1
VAEVAR_WIN_ATTN=0 N=3 timeout -k 10 200 python tools/fcst_time.py > gpurun_out/win/f_off.log 2>&1
N=3 timeout -k 10 200 python tools/fcst_time.py > gpurun_out/win/f_on.log 2>&1
