# tangency solver A/B: TH_LAST 1e-6, T_LAST 3e-5, Halley first step, t guess (HT); t guess only (T)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "x_test:900:LFG_LIB=$E/liblfg_HT.so python -u -m pytest tests -m 'gpu and not perf' -x -q --timeout 300 --timeout-method thread" \
 "x_b2_base:200:python3 bench.py --no-cpu > gpurun_out/x_c2_base.json" \
 "x_b2_ht:200:LFG_LIB=$E/liblfg_HT.so python3 bench.py --no-cpu > gpurun_out/x_c2_ht.json" \
 "x_b2_t:200:LFG_LIB=$E/liblfg_T.so python3 bench.py --no-cpu > gpurun_out/x_c2_t.json" \
 "x_b2_base2:200:python3 bench.py --no-cpu > gpurun_out/x_c2_base2.json" \
 "x_b2_ht2:200:LFG_LIB=$E/liblfg_HT.so python3 bench.py --no-cpu > gpurun_out/x_c2_ht2.json" \
 "x_b3_base:300:python3 bench.py --config 3 --steps 30 --no-cpu > gpurun_out/x_c3_base.json" \
 "x_b3_ht:300:LFG_LIB=$E/liblfg_HT.so python3 bench.py --config 3 --steps 30 --no-cpu > gpurun_out/x_c3_ht.json" \
 "x_p2_ht:200:LFG_LIB=$E/liblfg_HT.so rocprofv3 --kernel-trace --stats -d gpurun_out/x_prof2_ht -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "x_bx:200:python3 bench.py --exchange-path --no-cpu > gpurun_out/x_c2_xch.json" \
 "x_px:200:rocprofv3 --kernel-trace --stats -d gpurun_out/x_prof_xch -o run --output-format csv -- python3 bench.py --exchange-path --steps 50 --warmup 5 --no-cpu"
