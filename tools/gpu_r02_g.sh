cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench2:200:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_fused_c2.json" \
 "bench4:200:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_fused_c4.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_fused -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
