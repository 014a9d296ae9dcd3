cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in main v0 w4; do
  lib=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so; [ $v = main ] && lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
  steps+=("b_$v:200:LFG_LIB=$lib python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/c_$v.json")
  steps+=("p_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/c_prof_$v -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu")
  steps+=("w_$v:200:LFG_LIB=$lib timeout -s KILL 100 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/c_pmcw_$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu")
  steps+=("i_$v:200:LFG_LIB=$lib timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SCRATCH -d gpurun_out/c_pmci_$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu")
done
tools/gpu_steps.sh \
 "gputest:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "${steps[@]}"
