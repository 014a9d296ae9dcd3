set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5z_test.log 2>&1
bash tools/gpu_ab2.sh z5 3 "--config 5 --steps 10 --warmup 3" PREV NEW
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_PAIRPROF.so timeout -k 10 120 python tools/pair_profile.py 4096 10000 5 > gpurun_out/r5z_prof.log 2>&1
