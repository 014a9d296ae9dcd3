# GP filter: branch-free block reset; FP64 latency probe
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "k_lat:60:./build/lat_probe" \
 "k_test:300:python -u -m pytest tests/test_gpu_lnprob.py -x -q --timeout 120 --timeout-method thread -k gp" \
 "k_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/k_prof_gp -o run --output-format csv -- python3 bench.py --config gp --steps 20 --warmup 3 --no-cpu"
