cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench2:400:python bench.py > gpurun_out/bench_c2_bc.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_bc -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "pmc:600:bash tools/pmc_profile.sh r02bc" \
 "bench3:300:python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c3_bc.json" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_bc.json" \
 "bench4:300:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_bc.json"
[ $? -eq 0 ] && tools/gpu_steps.sh \
 "gpv2test:300:LFG_LIB=build/exp/liblfg_gpv2.so python -u -m pytest tests/test_gpu_lnprob.py -m gpu -x -q --timeout 120 --timeout-method thread -k gp" \
 "gpv2prof:200:LFG_LIB=build/exp/liblfg_gpv2.so rocprofv3 --kernel-trace -d gpurun_out/gp_bc_v2 -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "gpv1prof:200:rocprofv3 --kernel-trace -d gpurun_out/gp_bc_v1 -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu"
