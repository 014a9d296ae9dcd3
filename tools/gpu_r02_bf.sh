cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "c3long:300:python bench.py --config 3 --steps 300 --warmup 3 --no-cpu > gpurun_out/bench_c3_bf_300.json" \
 "gplong:300:python bench.py --config gp --steps 500 --warmup 3 --no-cpu > gpurun_out/bench_gp_bf_500.json" \
 "c5long:300:python bench.py --config 5 --steps 40 --warmup 2 --no-cpu > gpurun_out/bench_c5_bf_40.json"
