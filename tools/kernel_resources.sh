#!/bin/bash
# Per-kernel resource usage (VGPRs, SGPRs, scratch, LDS, occupancy) of the
# library's gfx950 code, from the compiler's kernel-resource-usage remarks.
#   tools/kernel_resources.sh [extra hipcc flags]   -> stdout
set -e
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /tmp/lfg_res.o \
    -I include -Rpass-analysis=kernel-resource-usage "$@" lfit_python_amd/csrc/lfg.hip 2>&1 |
    grep -E "remark: .*(Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:)" |
    sed -E 's/^.*remark: //'
