# r04: PMC stall breakdown of the fused tower kernels and the tile-48 / 49 GEMMs (per kernel)
set -e
T=1 bash tools/pmc_kernel.sh "k_mlp|k_ablk|k_gemm_h4|k_gemm_h5|k_fixup_ln" tower_r04 python3 tools/quick_time.py
