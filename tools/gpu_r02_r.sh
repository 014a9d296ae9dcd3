cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "plike:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 512 300 1" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_r.json" \
 "bench6:300:LFG_LIB=build/exp/liblfg_ew6.so python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_ew6.json" \
 "bench8:300:LFG_LIB=build/exp/liblfg_ew8.so python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_ew8.json"
