cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "gputest:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "emu8:300:python bench.py --config 4 --emulate-rank 0/8 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_c4_emu8_b.json" \
 "emu8k7:300:python bench.py --config 4 --emulate-rank 7/8 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_c4_emu8k7_b.json" \
 "profemu:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_emu8_b -o run --output-format csv -- python3 bench.py --config 4 --emulate-rank 0/8 --steps 20 --warmup 5 --no-cpu"
