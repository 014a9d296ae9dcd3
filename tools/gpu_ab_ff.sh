# one-eclipse k_lnlike without the offset load (A/B against the committed build PREV) + the weak-scaling rehearsal
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
tools/gpu_steps.sh \
 "ff_test:900:python -u -m pytest tests -m 'gpu and not perf' -x -q --timeout 300 --timeout-method thread" \
 "ff_b2:200:python3 bench.py --no-cpu > gpurun_out/ff_c2.json" \
 "ff_b2p:200:LFG_LIB=$E/liblfg_PREV.so python3 bench.py --no-cpu > gpurun_out/ff_c2_prev.json" \
 "ff_b2b:200:python3 bench.py --no-cpu > gpurun_out/ff_c2_b.json" \
 "ff_b2pb:200:LFG_LIB=$E/liblfg_PREV.so python3 bench.py --no-cpu > gpurun_out/ff_c2_prev_b.json" \
 "ff_p2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/ff_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "ff_p2p:200:LFG_LIB=$E/liblfg_PREV.so rocprofv3 --kernel-trace --stats -d gpurun_out/ff_prof2_prev -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu"
bash tools/gpu_emu_weak.sh
tools/gpu_steps.sh \
 "ff_gloo2:300:LFG_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/ff_c2_gloo2.json" \
 "ff_gloo4:300:LFG_BENCH_BACKEND=gloo python3 bench.py --gpus 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/ff_c2_gloo4.json"
