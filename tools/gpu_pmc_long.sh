#!/bin/bash
# PMC passes on config 5 (k_pair LONG): the SQ wait/issue mix, then the
# instruction-cache counters.  One counter group per pass, --kernel-trace only.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_long
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || echo "list-avail failed"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu --config 5 --steps 2 --warmup 1 > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 3; }
  echo "pass $i done ($grp)"
done
