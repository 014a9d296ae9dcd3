set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5r_test.log 2>&1
bash tools/gpu_ab2.sh r5 2 "--config 5 --steps 10 --warmup 3" W82 W31 W11 W00
