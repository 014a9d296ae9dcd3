cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gpspec:200:rocprofv3 --kernel-trace -d gpurun_out/gp_spec -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu" \
 "gpnospec:200:LFG_SPEC=0 rocprofv3 --kernel-trace -d gpurun_out/gp_nospec -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu"
