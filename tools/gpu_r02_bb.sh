cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "b_main:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/bb_main.json" \
 "b_prev:200:LFG_LIB=build/exp/liblfg_prev.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/bb_prev.json" \
 "b_main2:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/bb_main2.json" \
 "b_prev2:200:LFG_LIB=build/exp/liblfg_prev.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/bb_prev2.json"
