set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n_test.log 2>&1
timeout -k 10 120 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/r5n_c5.json 2>gpurun_out/r5n_c5.err
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_PAIRPROF.so timeout -k 10 120 python tools/pair_profile.py 4096 10000 5 > gpurun_out/r5n_prof.log 2>&1
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_SPOT.so timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n_test_spot.log 2>&1
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_SPOT.so timeout -k 10 120 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/r5n_c5_spot.json 2>gpurun_out/r5n_c5_spot.err
timeout -k 10 120 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/r5n_c5b.json 2>>gpurun_out/r5n_c5.err
