# spot cursor; DPP moves without old-value copies
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "u_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "u_p5:300:rocprofv3 --kernel-trace -d gpurun_out/u_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu" \
 "u_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/u_c5.json" \
 "u_p2:200:rocprofv3 --kernel-trace -d gpurun_out/u_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "u_pgp:200:rocprofv3 --kernel-trace -d gpurun_out/u_profgp -o run --output-format csv -- python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu" \
 "u_bgp:300:python3 bench.py --config gp --steps 100 --warmup 5 > gpurun_out/u_gp.json"
