cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "drift:300:python -u tools/chain_drift.py 1000 50" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_ak.json" \
 "bench2l:300:python bench.py --steps 1000 --warmup 5 --no-cpu > gpurun_out/bench_c2_ak_1000.json"
