# new tangency solver (NEW); chunk orders: longest-first (NEWORD), donor-first (ORD2), + donor rcp (ORD2R)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "y_test:900:LFG_LIB=$E/liblfg_ORD2R.so python -u -m pytest tests -m 'gpu and not perf' -x -q --timeout 300 --timeout-method thread" \
 "y_b2_new:200:LFG_LIB=$E/liblfg_NEW.so python3 bench.py --no-cpu > gpurun_out/y_c2_new.json" \
 "y_b2_ord:200:LFG_LIB=$E/liblfg_NEWORD.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord.json" \
 "y_b2_ord2:200:LFG_LIB=$E/liblfg_ORD2.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord2.json" \
 "y_b2_ord2r:200:LFG_LIB=$E/liblfg_ORD2R.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord2r.json" \
 "y_b2_new_b:200:LFG_LIB=$E/liblfg_NEW.so python3 bench.py --no-cpu > gpurun_out/y_c2_new_b.json" \
 "y_b2_ord_b:200:LFG_LIB=$E/liblfg_NEWORD.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord_b.json" \
 "y_b2_ord2_b:200:LFG_LIB=$E/liblfg_ORD2.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord2_b.json" \
 "y_b2_ord2r_b:200:LFG_LIB=$E/liblfg_ORD2R.so python3 bench.py --no-cpu > gpurun_out/y_c2_ord2r_b.json" \
 "y_tl_new:200:LFG_LIB=$E/liblfg_NEWPROF.so python3 tools/elem_timeline.py --config 2" \
 "y_tl_ord2r:200:LFG_LIB=$E/liblfg_ORD2RPROF.so python3 tools/elem_timeline.py --config 2" \
 "y_b3_ord2r:300:LFG_LIB=$E/liblfg_ORD2R.so python3 bench.py --config 3 --steps 30 --no-cpu > gpurun_out/y_c3_ord2r.json" \
 "y_bgp_new:300:LFG_LIB=$E/liblfg_NEW.so python3 bench.py --config gp --steps 50 --no-cpu > gpurun_out/y_gp_new.json" \
 "y_bgp_ord2r:300:LFG_LIB=$E/liblfg_ORD2R.so python3 bench.py --config gp --steps 50 --no-cpu > gpurun_out/y_gp_ord2r.json"
