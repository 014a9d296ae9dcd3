# GP k_gp_like: wave per eclipse, g-only chunks
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "i_test:300:python -u -m pytest tests/test_gpu_lnprob.py tests/test_gpu_anchor.py -x -q --timeout 120 --timeout-method thread -k 'gp or anchor'" \
 "i_bgp:200:python3 bench.py --config gp --steps 50 --warmup 5 --no-cpu > gpurun_out/i_gp.json" \
 "i_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/i_prof_gp -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu"
