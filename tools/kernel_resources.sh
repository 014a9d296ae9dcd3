#!/bin/bash
# Per-kernel resource usage (VGPRs, SGPRs, spills, scratch, LDS, occupancy) of
# the library's gfx950 code, from the compiler's kernel-resource-usage
# remarks: lfg.hip, then lfg_pair_split.hip (k_pair's fold and LONG
# instantiations, compiled without machine LICM as the library builds them).
#   tools/kernel_resources.sh [extra hipcc flags]   -> stdout
set -e
cd "$(dirname "$0")/.."
unit() {  # unit <source> [flags...]
  local src=$1; shift
  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /tmp/lfg_res.o \
      -I include -Rpass-analysis=kernel-resource-usage "$@" lfit_python_amd/csrc/$src 2>&1 |
      grep -E "remark: .*(Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:|Spill)" |
      sed -E 's/^.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//'
}
unit lfg.hip "$@"
unit lfg_pair_split.hip -mllvm -disable-machine-licm "$@"
