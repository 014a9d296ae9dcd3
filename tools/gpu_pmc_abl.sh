#!/bin/bash
# One SQ PMC pass per ablation build of the LONG point phase (config 5), then
# the main build's bench and per-wave profile.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_abl
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
grp="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for v in Q_BASE Q_LSUB Q_LWD Q_SCDONOR Q_SCTRIG Q_SCSPOT; do
  LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $out/$v -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu --config 5 --steps 2 --warmup 1 > $out/$v.log 2>&1 || { echo "pass $v failed"; exit 3; }
done
cd $R
timeout -k 10 120 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/r5o_c5.json 2>gpurun_out/r5o_c5.err
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_PAIRPROF.so timeout -k 10 120 python tools/pair_profile.py 4096 10000 5 > gpurun_out/r5o_prof.log 2>&1
