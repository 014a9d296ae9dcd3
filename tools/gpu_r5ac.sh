set -e
mkdir -p gpurun_out
LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_VD.so timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ac_test.log 2>&1
bash tools/gpu_ab2.sh ac5 3 "--config 5 --steps 10 --warmup 3" BASE VD
