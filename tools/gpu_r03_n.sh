# profiles/r03 evidence for configs 3, 4, gp (bench lines, rocprof stats, GP PMC)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "n_b3:300:python3 bench.py --config 3 --steps 50 --warmup 5 > gpurun_out/n_c3.json" \
 "n_b4:300:python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/n_c4.json" \
 "n_e4:300:python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu --emulate-rank 0/8 > gpurun_out/n_c4_emu8.json" \
 "n_bgp:300:python3 bench.py --config gp --steps 100 --warmup 5 > gpurun_out/n_gp.json" \
 "n_pgp:200:rocprofv3 --kernel-trace --stats -d gpurun_out/n_prof_gp -o run --output-format csv -- python3 bench.py --config gp --steps 50 --warmup 5 --no-cpu" \
 "n_p3:200:rocprofv3 --kernel-trace --stats -d gpurun_out/n_prof_c3 -o run --output-format csv -- python3 bench.py --config 3 --steps 30 --warmup 3 --no-cpu" \
 "n_pmcgp:900:bash tools/pmc_profile.sh r03gp --config gp --steps 3 --warmup 1"
