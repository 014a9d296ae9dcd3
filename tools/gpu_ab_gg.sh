# k_accept_regen with its first row chunks fetched before the acceptance (shard path) against the committed build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "gg_test:600:python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread" \
 "gg_x:200:python3 bench.py --exchange-path --no-cpu > gpurun_out/gg_xch.json" \
 "gg_xp:200:LFG_LIB=$E/liblfg_PREV.so python3 bench.py --exchange-path --no-cpu > gpurun_out/gg_xch_prev.json" \
 "gg_x_b:200:python3 bench.py --exchange-path --no-cpu > gpurun_out/gg_xch_b.json" \
 "gg_xp_b:200:LFG_LIB=$E/liblfg_PREV.so python3 bench.py --exchange-path --no-cpu > gpurun_out/gg_xch_prev_b.json" \
 "gg_e8:200:python3 bench.py --walkers 8192 --emulate-rank 0/8 --no-cpu > gpurun_out/gg_emu8.json" \
 "gg_e8p:200:LFG_LIB=$E/liblfg_PREV.so python3 bench.py --walkers 8192 --emulate-rank 0/8 --no-cpu > gpurun_out/gg_emu8_prev.json" \
 "gg_px:200:rocprofv3 --kernel-trace --stats -d gpurun_out/gg_profx -o run --output-format csv -- python3 bench.py --walkers 8192 --emulate-rank 0/8 --steps 50 --no-cpu" \
 "gg_pxp:200:LFG_LIB=$E/liblfg_PREV.so rocprofv3 --kernel-trace --stats -d gpurun_out/gg_profx_prev -o run --output-format csv -- python3 bench.py --walkers 8192 --emulate-rank 0/8 --steps 50 --no-cpu"
