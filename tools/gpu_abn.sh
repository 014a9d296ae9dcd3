#!/bin/bash
# A/B/n of experiment builds against the main library on one box: the bench
# (default: the driver's config-2 command) for each build in turn, N rounds.
#   gpurun -- 'bash tools/gpu_abn.sh "<exp names>" [rounds] [bench args]'
R=$GRAFT_REPO_ROOT
names=$1; n=${2:-3}; shift; shift
args=${*:-"--steps 20 --warmup 5 --no-cpu"}
cd $R
for i in $(seq $n); do
  line="round $i:"
  for b in main $names; do
    if [ $b = main ]; then
      timeout -k 10 120 python3 bench.py $args > gpurun_out/abn_main.json 2>/dev/null || exit 3
    else
      LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$b.so timeout -k 10 120 python3 bench.py $args > gpurun_out/abn_$b.json 2>/dev/null || exit 3
    fi
    v=$(python3 -c "import json; d=json.loads(open('gpurun_out/abn_$b.json').read().strip().splitlines()[-1]); print('%.3f M %.1f us' % (d['value'] / 1e6, d['ms_per_step'] * 1e3))")
    line="$line  $b $v |"
  done
  echo "$line"
done
