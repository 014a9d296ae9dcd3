cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "b2:200:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/f_c2.json" \
 "b5:300:python bench.py --config 5 --steps 20 --warmup 3 --no-cpu > gpurun_out/f_c5.json" \
 "p5:300:rocprofv3 --kernel-trace -d gpurun_out/f_prof_c5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu" \
 "p2:200:rocprofv3 --kernel-trace -d gpurun_out/f_prof_c2 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu"
