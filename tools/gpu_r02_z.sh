cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "plike:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 512 300 1" \
 "plike5:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 64 10000 5" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_z.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_z -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
