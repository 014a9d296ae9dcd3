#!/bin/bash
# Round-5 measurement pass, in two calls (each under gpurun's limit):
#   gpurun --timeout 1200 -- 'bash tools/gpu_final_r05.sh A'
#   gpurun --timeout 1200 -- 'bash tools/gpu_final_r05.sh B'
# A: pytest -m gpu, smoke, config 2 (100 and the driver's 20 steps), config 5,
#    rocprofv3 kernel traces of configs 2 and 5, the LONG phase profile.
# B: PMC passes of configs 2 and 5, configs 3 and 4, the one-of-eight
#    rehearsal, the GP example, the exchange path, the GP kernel trace.
part=${1:?A or B}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
if [ "$part" = A ]; then
  bash tools/gpu_pass.sh r05 test smoke c2 c2_20 c5 p2 p5 || exit $?
  LFG_DIAGNOSTIC=1 LFG_LIB=$E/liblfg_PAIRPROF.so timeout -k 10 120 python3 tools/pair_profile.py 4096 10000 5 > gpurun_out/r05_pair_profile_c5.txt 2>&1 || exit $?
  LFG_DIAGNOSTIC=1 LFG_LIB=$E/liblfg_PAIRPROF.so timeout -k 10 120 python3 tools/pair_profile.py 1024 300 1 > gpurun_out/r05_pair_profile_c2.txt 2>&1 || exit $?
else
  bash tools/gpu_pass.sh r05 pmc2 c3 c4 c4e gp xch pgp || exit $?
  timeout -k 10 600 bash tools/pmc_profile.sh r05c5 --config 5 --steps 2 --warmup 1 || exit $?
fi
