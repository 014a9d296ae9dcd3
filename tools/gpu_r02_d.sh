cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gptest:300:python -u -m pytest tests/test_gpu_lnprob.py -x -v --timeout 120 --timeout-method thread -k 'gp or GP'" \
 "benchgp:200:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_r02_gp_d.json" \
 "profgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gp_d -o run -- python3 bench.py --config gp --steps 20 --warmup 2 --no-cpu"
