cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gptest:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'gp or reference'" \
 "gpprof:200:rocprofv3 --kernel-trace -d gpurun_out/gp_as -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_as.json"
