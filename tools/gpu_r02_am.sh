cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_am.json" \
 "bench3:300:python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c3_am.json" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_am.json" \
 "c3prof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/c3_am -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
