# config-2 weak scaling rehearsed on one GPU: one rank of N (1024 walkers per GPU) vs the one-GPU run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "e_n1:200:python3 bench.py --no-cpu > gpurun_out/e_c2_n1.json" \
 "e_n2:200:python3 bench.py --walkers 2048 --emulate-rank 0/2 --no-cpu > gpurun_out/e_c2_emu2.json" \
 "e_n4:200:python3 bench.py --walkers 4096 --emulate-rank 0/4 --no-cpu > gpurun_out/e_c2_emu4.json" \
 "e_n8:200:python3 bench.py --walkers 8192 --emulate-rank 0/8 --no-cpu > gpurun_out/e_c2_emu8.json" \
 "e_n8b:200:python3 bench.py --walkers 8192 --emulate-rank 7/8 --no-cpu > gpurun_out/e_c2_emu8_r7.json"
