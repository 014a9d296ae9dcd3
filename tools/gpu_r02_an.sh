cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench3:300:python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c3_an.json" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_an.json" \
 "c3prof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/c3_an -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
