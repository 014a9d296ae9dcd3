# k_lnlike tile flags: one atomic per wave
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "p_test:600:python -u -m pytest tests/test_gpu_lnprob.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread" \
 "p_c3:200:python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/p_c3.json" \
 "p_c2:200:python3 bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/p_c2.json" \
 "p_p3:200:rocprofv3 --kernel-trace --stats -d gpurun_out/p_prof_c3 -o run --output-format csv -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu"
