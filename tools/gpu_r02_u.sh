cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchsh:300:python bench.py --steps 100 --warmup 5 --no-cpu --shard-path > gpurun_out/bench_c2_shard_spec.json" \
 "benchsh0:300:LFG_SPEC=0 python bench.py --steps 100 --warmup 5 --no-cpu --shard-path > gpurun_out/bench_c2_shard_nospec.json" \
 "benchxch:300:python bench.py --steps 100 --warmup 5 --no-cpu --exchange-path > gpurun_out/bench_c2_xch_spec.json" \
 "bench2r:300:LFG_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c2_2r_gloo.json"
