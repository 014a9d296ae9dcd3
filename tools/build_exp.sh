#!/bin/bash
# Experiment/diagnostic builds of liblfg_hip.so: build/exp/liblfg_<name>.so
# with extra compile flags, loaded through LFG_LIB (lfit_python_amd/_native.py).
# usage: tools/build_exp.sh <name> [-DFLAG ...]   (LFG_SRC=<file>: another lfg.hip, e.g. a commit's)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p $R/build/exp
# k_pair's fold and LONG instantiations: lfg_pair_split.hip without machine
# LICM (LFG_SRC builds of older sources have no split unit: LFG_SPLIT=0;
# SPLIT_FLAGS: flags for that unit only)
split=
if [ "${LFG_SPLIT:-1}" = 1 ]; then
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -disable-machine-licm $SPLIT_FLAGS -I $R/include "$@" \
    -c -o $R/build/exp/split_$name.o $R/lfit_python_amd/csrc/lfg_pair_split.hip
  split="-x none $R/build/exp/split_$name.o"
fi
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include "$@" \
  -o $R/build/exp/liblfg_$name.so ${LFG_SRC:-$R/lfit_python_amd/csrc/lfg.hip} $R/lfit_python_amd/csrc/lfg_components.hip $split
rm -f $R/build/exp/split_$name.o
