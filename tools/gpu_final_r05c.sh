#!/bin/bash
# Round-5 closing pass on the final library: pytest -m gpu, smoke, config 5
# (bench, rocprofv3 kernel trace, LONG phase profile, PMC passes).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
bash tools/gpu_pass.sh r05h test smoke c5 p5 || exit $?
LFG_DIAGNOSTIC=1 LFG_LIB=$E/liblfg_PAIRPROF.so timeout -k 10 120 python3 tools/pair_profile.py 4096 10000 5 > gpurun_out/r05h_pair_profile_c5.txt 2>&1 || exit $?
timeout -k 10 600 bash tools/pmc_profile.sh r05hc5 --config 5 --steps 2 --warmup 1 || exit $?
