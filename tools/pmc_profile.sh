#!/bin/bash
# PMC passes over a short bench run, one counter group per pass and only
# --kernel-trace beside --pmc (no sys/runtime trace).  Each pass has its own
# time limit; the first failing pass ends the script.
# usage: tools/pmc_profile.sh <tag> [bench.py args, default: config 2]
# Output: gpurun_out/pmc_<tag>/p<i>/...
tag=${1:-r03}
shift
args=${*:-"--steps 5 --warmup 2"}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$tag
echo "bench args: $args" > $R/gpurun_out/pmc_$tag/args.txt
i=0
for grp in \
  "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
  "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $R/gpurun_out/pmc_$tag/p$i -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu $args > $R/gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed"; exit 3; }
  echo "pass $i done ($grp)"
done
