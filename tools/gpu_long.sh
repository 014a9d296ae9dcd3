# long chains with the round-3 solver: step time per 50-step block over 1000 config-2 steps, its solver
# counts at the saved snapshots (LFG_COUNT_ITERS build), and long config-3 / GP benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "l_drift:400:python3 tools/chain_drift.py 1000 50 > gpurun_out/l_drift.txt" \
 "l_count:300:LFG_LIB=$E/liblfg_COUNT.so python3 tools/chain_drift.py count > gpurun_out/l_count.txt" \
 "l_c3:600:python3 bench.py --config 3 --steps 300 --warmup 5 --no-cpu > gpurun_out/l_c3_300.json" \
 "l_gp:600:python3 bench.py --config gp --steps 500 --warmup 5 --no-cpu > gpurun_out/l_gp_500.json"
