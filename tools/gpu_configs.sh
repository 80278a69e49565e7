# bench lines for BASELINE configs 3, 4, 5 (1 GPU, no CPU baseline) + the 0.25-degree forecast timing
set -e
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > gpurun_out/cfg/c3.json 2> gpurun_out/cfg/c3.err
echo c3
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > gpurun_out/cfg/c4.json 2> gpurun_out/cfg/c4.err
echo c4
timeout -k 10 300 python bench.py --config 5 --steps 5 --no-cpu-baseline > gpurun_out/cfg/c5.json 2> gpurun_out/cfg/c5.err
echo c5
timeout -k 10 300 python tools/fcst_time.py > gpurun_out/cfg/fcst.log 2>&1
echo fcst
