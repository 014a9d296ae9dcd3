cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gptest:300:python -u -m pytest tests/test_gpu_lnprob.py -x -q --timeout 120 --timeout-method thread -k 'gp or GP'" \
 "gp64:200:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp64.json" \
 "gp16:200:LFG_LIB=build/exp/liblfg_gp16.so python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp16.json" \
 "gp4:200:LFG_LIB=build/exp/liblfg_gp4.so python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp4.json" \
 "prof16:200:LFG_LIB=build/exp/liblfg_gp16.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gp16 -o run -- python3 bench.py --config gp --steps 20 --warmup 2 --no-cpu" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_v10 -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
