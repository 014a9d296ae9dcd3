cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "b20a:300:python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_a_20.json" \
 "b100a:300:python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/bench_c2_a_100.json" \
 "b20b:300:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_c2_a_20b.json" \
 "prof2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_a -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu" \
 "prof5:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_a -o run --output-format csv -- python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu" \
 "pmc5:900:bash tools/pmc_profile.sh c5a --config 5 --steps 3 --warmup 1"
