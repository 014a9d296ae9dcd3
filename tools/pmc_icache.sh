#!/bin/bash
# Instruction-fetch counters over a short bench run (two passes).
tag=${1:-ic}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
set -e
mkdir -p $R/gpurun_out/pmc_$tag
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $R/gpurun_out/pmc_$tag/p$i -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 > $R/gpurun_out/pmc_$tag/p$i.log 2>&1
  echo "pass $i done"
done
