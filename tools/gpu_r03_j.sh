# GP wave-per-eclipse k_gp_like; config-5 donor cursor
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "j_test:600:python -u -m pytest tests/test_gpu_lnprob.py tests/test_gpu_anchor.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
 "j_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 --no-cpu > gpurun_out/j_c5.json" \
 "j_bgp:200:python3 bench.py --config gp --steps 50 --warmup 5 --no-cpu > gpurun_out/j_gp.json" \
 "j_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/j_prof_gp -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu"
