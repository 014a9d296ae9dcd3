cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "gp2prof:200:rocprofv3 --kernel-trace -d gpurun_out/gp_aw2 -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "gp1prof:200:LFG_LIB=build/exp/liblfg_gp1.so rocprofv3 --kernel-trace -d gpurun_out/gp_aw1 -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_aw.json"
