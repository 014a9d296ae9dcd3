#!/bin/bash
# A/B of the main library against an experiment build on one box:
# config-2 bench (the driver's 20 steps and 100 steps) alternating, N rounds.
#   gpurun -- 'bash tools/gpu_ab3.sh <exp-name> [rounds] [bench args]'
R=$GRAFT_REPO_ROOT
b=$1; n=${2:-3}; shift; shift
args=${*:-"--steps 20 --warmup 5 --no-cpu"}
cd $R
for i in $(seq $n); do
  timeout -k 10 120 python3 bench.py $args > gpurun_out/ab_main_$i.json 2>/dev/null || exit 3
  LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$b.so timeout -k 10 120 python3 bench.py $args > gpurun_out/ab_${b}_$i.json 2>/dev/null || exit 3
  python3 - <<PY
import json
def v(f):
    d = json.loads(open(f).read().strip().splitlines()[-1]); return d["value"] / 1e6, d["ms_per_step"] * 1e3
print("round $i: main %.3f M (%.1f us/step)   $b %.3f M (%.1f us/step)" % (*v("gpurun_out/ab_main_$i.json"), *v("gpurun_out/ab_${b}_$i.json")))
PY
done
