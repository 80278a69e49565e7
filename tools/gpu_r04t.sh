# r04: confirm the tile-48 late row-scale loads: bitwise / trajectory tests
set -e
mkdir -p gpurun_out/r04t
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "bitwise or h5 or config2_traj or config3_traj or fixup_ln or ln_planes or g3 or gemm" > gpurun_out/r04t/focus.log 2>&1
