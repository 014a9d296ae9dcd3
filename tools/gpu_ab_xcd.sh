# setup lanes dealt to the XCD that reads their pair (XCDSET) against the committed build (PREV)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
steps=("x_test:900:LFG_LIB=$E/liblfg_XCDSET.so python -u -m pytest tests -m 'gpu and not perf' -x -q --timeout 300 --timeout-method thread")
for r in a b; do
  for v in XCDSET PREV; do
    steps+=("x_b_${v}_$r:200:LFG_LIB=$E/liblfg_$v.so python3 bench.py --no-cpu > gpurun_out/xc_c2_${v}_$r.json")
  done
done
for v in XCDSET PREV; do
  steps+=("x_p_$v:200:LFG_LIB=$E/liblfg_$v.so rocprofv3 --kernel-trace -d gpurun_out/xc_prof_$v -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
  steps+=("x_gp_$v:300:LFG_LIB=$E/liblfg_$v.so python3 bench.py --config gp --steps 50 --no-cpu > gpurun_out/xc_gp_$v.json")
  steps+=("x_nospec_$v:200:LFG_SPEC=0 LFG_LIB=$E/liblfg_$v.so python3 bench.py --no-cpu > gpurun_out/xc_c2ns_$v.json")
done
tools/gpu_steps.sh "${steps[@]}"
