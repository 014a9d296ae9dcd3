nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo OMP=$OMP_NUM_THREADS
tools/gpu_steps.sh \
 "gputest:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "bench2:200:python bench.py --steps 100 --warmup 5 > gpurun_out/bench_r02_c2.json" \
 "bench4:200:python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_r02_c4n1.json" \
 "benchgp:200:python bench.py --config gp --steps 50 --warmup 3 --no-cpu > gpurun_out/bench_r02_gp.json" \
 "spawn2:200:LFG_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_r02_spawn2_gloo.json"
