#!/bin/bash
# LDS counters of k_pair at config 2 with each element sink's LDS work
# skipped in turn (diagnostic builds: tools/build_exp.sh S<x> -DLFG_ABL_SINK_<x>);
# attribution of the bank-conflict cycles per sink kind.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_sinks
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
grp="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY"
for v in ${VARIANTS:-SBASE SWD SSPOT SDON}; do
  LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $out/$v -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $out/$v.log 2>&1 || { echo "pass $v failed"; exit 3; }
done
