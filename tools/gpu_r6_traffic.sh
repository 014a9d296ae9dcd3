#!/bin/bash
# Round 6: where k_pair's L2 and memory traffic comes from on the bench's own
# path (config 2, speculative lanes, 5 timed steps): per build, PMC passes
#   a: FETCH_SIZE (memory reads, KB), TCC_MISS_sum
#   b: L2 read requests by client: instruction fetch (SQC_TC_INST_REQ), scalar
#      data (SQC_TC_DATA_READ_REQ), and the instruction / scalar cache misses
#   c: vector L2 reads and writes (TCP_TCC_READ_REQ_sum, TCP_TCC_WRITE_REQ_sum), WRITE_SIZE
# Builds: main; A_EMPTY (k_pair returns at entry); A_ELEM (no element jobs);
# A_STTAB (-DLFG_ABL_STTAB: every stream lane reads one table patch); nospec
# (the main library with LFG_SPEC=0: the plain path, k_setup + k_pair, no
# speculative lanes and no candidate selection in k_pair).
#   gpurun --timeout 900 -- 'bash tools/gpu_r6_traffic.sh [variants]'
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6_traffic
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in ${*:-main A_EMPTY A_ELEM}; do
  i=0
  for grp in "FETCH_SIZE TCC_MISS_sum" "SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ SQC_ICACHE_MISSES SQC_DCACHE_MISSES" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum WRITE_SIZE"; do
    i=$((i+1))
    if [ $v = main ] || [ $v = nospec ]; then
      [ $v = nospec ] && export LFG_SPEC=0
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $out/$v/p$i -o run --output-format csv \
        -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $out/$v.p$i.log 2>&1 || { echo "pass $v $i failed"; exit 3; }
      unset LFG_SPEC
    else
      LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp \
        -d $out/$v/p$i -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 \
        > $out/$v.p$i.log 2>&1 || { echo "pass $v $i failed"; exit 3; }
    fi
    echo "pass $v $i done"
  done
done
