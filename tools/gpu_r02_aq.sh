cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "b_main:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/aq_main.json" \
 "b_ipl2:200:LFG_LIB=build/exp/liblfg_ipl2.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/aq_ipl2.json" \
 "b_ipl2w4:200:LFG_LIB=build/exp/liblfg_ipl2w4.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/aq_ipl2w4.json" \
 "b_main2:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/aq_main2.json"
