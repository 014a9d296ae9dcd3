# final state (+ k_elements occupancy experiment at the end) of the solver / chunk-order / accept_regen changes: tests, smoke, benches, traces, PMC (config 2)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "z_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "z_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "z_b2:300:python3 bench.py > gpurun_out/z_c2.json" \
 "z_b2_20:200:python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/z_c2_20.json" \
 "z_b2_head:200:LFG_LIB=$E/liblfg_HEAD.so python3 bench.py --no-cpu > gpurun_out/z_c2_head.json" \
 "z_p2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/z_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "z_pmc2:900:bash tools/pmc_profile.sh z2" \
 "z_b3:300:python3 bench.py --config 3 --steps 30 > gpurun_out/z_c3.json" \
 "z_b4:300:python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/z_c4.json" \
 "z_b4e:300:python3 bench.py --config 4 --emulate-rank 0/8 --steps 20 --warmup 3 --no-cpu > gpurun_out/z_c4_emu8.json" \
 "z_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/z_c5.json" \
 "z_bgp:300:python3 bench.py --config gp --steps 100 --warmup 5 > gpurun_out/z_gp.json" \
 "z_bgp_head:300:LFG_LIB=$E/liblfg_HEAD.so python3 bench.py --config gp --steps 100 --warmup 5 --no-cpu > gpurun_out/z_gp_head.json" \
 "z_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/z_profgp -o run --output-format csv -- python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu" \
 "z_p5:300:rocprofv3 --kernel-trace --stats -d gpurun_out/z_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu" \
 "z_bx:200:python3 bench.py --exchange-path --no-cpu > gpurun_out/z_c2_xch.json" \
 "z_o_spec4:200:LFG_SPEC=0 python3 bench.py --no-cpu > gpurun_out/z_o_spec4_nospecpath.json" \
 "z_o_nospec4:200:LFG_SPEC=0 LFG_LIB=$E/liblfg_NOSPEC4.so python3 bench.py --no-cpu > gpurun_out/z_o_nospec4.json" \
 "z_o_nospec5:200:LFG_SPEC=0 LFG_LIB=$E/liblfg_NOSPEC5.so python3 bench.py --no-cpu > gpurun_out/z_o_nospec5.json" \
 "z_o_spec5:200:LFG_LIB=$E/liblfg_SPEC5.so python3 bench.py --no-cpu > gpurun_out/z_o_spec5.json"
