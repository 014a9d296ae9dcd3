# profiles/r03 evidence: bench lines (100 and 20 steps), kernel-trace stats,
# PMC passes of configs 2 and 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "h_b2_100:200:python3 bench.py --steps 100 --warmup 5 > gpurun_out/h_b2_100.json" \
 "h_b2_20:200:python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/h_b2_20.json" \
 "h_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/h_b5.json" \
 "h_p2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/h_prof_c2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu" \
 "h_p5:300:rocprofv3 --kernel-trace --stats -d gpurun_out/h_prof_c5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu" \
 "h_pmc2:900:bash tools/pmc_profile.sh r03c2 --steps 5 --warmup 2" \
 "h_pmc5:900:bash tools/pmc_profile.sh r03c5 --config 5 --steps 3 --warmup 1"
