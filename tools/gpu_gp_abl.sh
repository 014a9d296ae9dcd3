#!/bin/bash
# k_gp_like experiment builds against the main library on one box: a
# rocprofv3 kernel trace of the GP example for each (per-grid medians), then
# the A/B/n bench line, then the GP parity tests on the candidate build.
#   gpurun -- 'bash tools/gpu_gp_abl.sh "<exp names>" <candidate>'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
names=$1; cand=$2
for b in main $names; do
  if [ $b = main ]; then
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/gpabl_$b -o run --output-format csv -- \
      python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu > $O/gpabl_$b.log 2>&1 || exit 3
  else
    LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$b.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d $O/gpabl_$b -o run --output-format csv -- \
      python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu > $O/gpabl_$b.log 2>&1 || exit 3
  fi
  echo "== $b"
  python3 tools/trace_by_grid.py $(find $O/gpabl_$b -name "*kernel_trace.csv" | head -n 1) | grep -E "k_gp_like|k_pair|k_combine" || true
done
bash tools/gpu_abn.sh "$names" 3 --config gp --steps 100 --warmup 5 --no-cpu || exit 3
if [ -n "$cand" ]; then
  LFG_DIAGNOSTIC=1 LFG_LIB=$R/build/exp/liblfg_$cand.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "gp or GP" || exit 4
fi
