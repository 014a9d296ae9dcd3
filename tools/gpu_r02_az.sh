cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gptest:600:python -u -m pytest tests/test_gpu_lnprob.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "gpprof:200:rocprofv3 --kernel-trace -d gpurun_out/gp_az -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_az.json"
