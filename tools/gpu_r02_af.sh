cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench2:400:python bench.py > gpurun_out/bench_c2_af.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_af -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "pmc:600:bash tools/pmc_profile.sh r02af"
