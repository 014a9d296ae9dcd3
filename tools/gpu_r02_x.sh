cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests/test_gpu_lnprob.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_x.json" \
 "icache:600:bash tools/pmc_icache.sh r02ic"
