cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests/test_gpu_lnprob.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread" \
 "iters:120:LFG_LIB=build/exp/liblfg_iters.so python tools/iter_count.py" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_y.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_y -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
