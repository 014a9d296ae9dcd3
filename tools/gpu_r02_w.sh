cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "bench2:400:python bench.py > gpurun_out/bench_c2_w.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_w -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "pmc:600:bash tools/pmc_profile.sh r02w" \
 "bench3:300:python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c3_w.json" \
 "bench4:300:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_w.json" \
 "bench5:300:python bench.py --config 5 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c5_w.json" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_w.json"
