cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "drift0:200:python -u tools/chain_drift.py 100 100" \
 "iters:200:LFG_LIB=build/exp/liblfg_count.so python -u tools/chain_drift.py count" \
 "b_main:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/ba_main.json" \
 "b_rcpx:200:LFG_LIB=build/exp/liblfg_rcpx.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/ba_rcpx.json" \
 "b_main2:200:python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/ba_main2.json" \
 "b_rcpx2:200:LFG_LIB=build/exp/liblfg_rcpx.so python bench.py --steps 300 --warmup 5 --no-cpu > gpurun_out/ba_rcpx2.json"
