#!/bin/bash
# Experiment/diagnostic builds of liblfg_hip.so: build/exp/liblfg_<name>.so
# with extra compile flags, loaded through LFG_LIB (lfit_python_amd/_native.py).
# usage: tools/build_exp.sh <name> [-DFLAG ...]   (LFG_SRC=<file>: another lfg.hip, e.g. a commit's)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p $R/build/exp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include "$@" \
  -o $R/build/exp/liblfg_$name.so ${LFG_SRC:-$R/lfit_python_amd/csrc/lfg.hip} $R/lfit_python_amd/csrc/lfg_components.hip
