# config-4 eight-rank emulation: kernel breakdown of one rank
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "r_pe:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r_prof_emu8 -o run --output-format csv -- python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu --emulate-rank 0/8"
