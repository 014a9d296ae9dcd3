cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "psetup:120:LFG_LIB=build/exp/liblfg_psetup.so python tools/setup_profile.py" \
 "bench2:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_q.json" \
 "bench2k:300:HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_q_devk.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_q -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
