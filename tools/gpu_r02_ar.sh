cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench2:400:python bench.py > gpurun_out/bench_c2_ar.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_ar -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "pmc:600:bash tools/pmc_profile.sh r02ar" \
 "bench4:300:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_ar.json" \
 "bench5:300:python bench.py --config 5 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c5_ar.json" \
 "benchx:300:python bench.py --steps 100 --warmup 5 --no-cpu --exchange-path > gpurun_out/bench_c2_xch_ar.json" \
 "bench2g:300:LFG_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c2_2r_gloo_ar.json"
