cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "ptest:300:python -u -m pytest tests/test_gpu_lnprob.py -m gpu -x -q --timeout 120 --timeout-method thread -k prior_rejected" \
 "c3main:200:rocprofv3 --kernel-trace --stats -d gpurun_out/c3_main -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu" \
 "c3nofence:200:LFG_LIB=build/exp/liblfg_nofence.so rocprofv3 --kernel-trace --stats -d gpurun_out/c3_nofence -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
