#!/bin/bash
# Builds the timing-only microbenchmarks (binaries stay out of git; they travel via gpurun).
set -e
D=$(cd "$(dirname "$0")" && pwd)
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$D/../../include"
$H -x hip $D/bs_ablate.cpp -o $D/bs_ablate_full &
$H -x hip -DEZRS_BS_ABLATE_DMA $D/bs_ablate.cpp -o $D/bs_ablate_nodma &
$H -x hip -DEZRS_BS_ABLATE_COMPUTE $D/bs_ablate.cpp -o $D/bs_ablate_nocomp &
$H -x hip -DEZRS_BS_ABLATE_TRANSPOSE $D/bs_ablate.cpp -o $D/bs_ablate_notr &
$H -x hip -DEZRS_BS_ABLATE_DMA -DEZRS_BS_ABLATE_TRANSPOSE $D/bs_ablate.cpp -o $D/bs_ablate_computeonly &
wait
