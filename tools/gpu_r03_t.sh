# LDS address space in sub_point; gather reads without flat loads
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "t_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "t_p5:300:rocprofv3 --kernel-trace -d gpurun_out/t_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu" \
 "t_p2:200:rocprofv3 --kernel-trace -d gpurun_out/t_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "t_pgp:200:rocprofv3 --kernel-trace -d gpurun_out/t_profgp -o run --output-format csv -- python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu"
