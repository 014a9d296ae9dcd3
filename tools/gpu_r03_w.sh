# re-entry check of HEAD: GPU tests, smoke, config 2/5/gp benches + kernel traces, k_elements timeline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "w_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "w_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "w_b2:300:python3 bench.py > gpurun_out/w_c2.json" \
 "w_b2_20:300:python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/w_c2_20.json" \
 "w_p2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/w_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "w_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/w_c5.json" \
 "w_p5:300:rocprofv3 --kernel-trace --stats -d gpurun_out/w_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu" \
 "w_bgp:300:python3 bench.py --config gp --steps 100 --warmup 5 > gpurun_out/w_gp.json" \
 "w_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/w_profgp -o run --output-format csv -- python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu" \
 "w_tl2:200:LFG_LIB=$GRAFT_REPO_ROOT/build/exp/liblfg_ELEMPROF.so python3 tools/elem_timeline.py --config 2"
