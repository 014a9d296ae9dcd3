#!/bin/bash
# Round 6: k_pair (config 2) counters per diagnostic build on one FIXED batch
# of 512 walkers (tools/pair_fixed.py: one round of 512 workgroups, no
# speculative lanes), three PMC passes per build; then the bench's own k_pair
# (speculative lanes included) on the main library.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r6_pmc.sh [variants...]'
# Builds: tools/build_exp.sh A_FULL; A_EMPTY -DLFG_ABL_EMPTY; A_ELEM -DLFG_ABL_ELEM;
#         A_LIKE -DLFG_ABL_LIKE; A_SINKS -DLFG_ABL_SINK_WD -DLFG_ABL_SINK_SPOT -DLFG_ABL_SINK_DON
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
vars=${*:-"A_FULL A_EMPTY A_ELEM A_LIKE A_SINKS"}
g1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES"
g2="FETCH_SIZE TCC_MISS_sum"
g3="WRITE_SIZE TCC_HIT_sum"
timeout -s KILL 60 rocprofv3 --list-avail > $out/counters.txt 2>&1 || echo "list-avail rc=$?"
for v in $vars; do
  i=0
  for grp in "$g1" "$g2" "$g3"; do
    i=$((i+1))
    LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp \
      -d $out/$v/p$i -o run --output-format csv -- python3 $R/tools/pair_fixed.py 512 $R/gpurun_out/pf512.npy \
      > $out/$v.p$i.log 2>&1 || { echo "pass $v $i failed"; exit 3; }
    echo "pass $v $i done"
  done
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g1 -d $out/bench/p1 -o run --output-format csv \
  -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $out/bench.p1.log 2>&1 || { echo "bench pass failed"; exit 3; }
echo done
