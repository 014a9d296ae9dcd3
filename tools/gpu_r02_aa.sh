cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "bench2:400:python bench.py > gpurun_out/bench_c2_aa.json" \
 "profc2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_aa -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "pmc:600:bash tools/pmc_profile.sh r02aa" \
 "bench3:300:python bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c3_aa.json" \
 "bench4:300:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_aa.json" \
 "bench5:300:python bench.py --config 5 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c5_aa.json" \
 "benchgp:300:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_gp_aa.json" \
 "benchsh:300:python bench.py --steps 100 --warmup 5 --no-cpu --exchange-path > gpurun_out/bench_c2_xch_aa.json"
