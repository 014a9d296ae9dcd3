# k_elements: round-2 library vs now (configs 3 and 2), kernel-trace medians
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in main 70056c4; do
  lib=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so; [ $v = main ] && lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
  steps+=("q3_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/q_prof3_$v -o run --output-format csv -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu")
  steps+=("q2_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/q_prof2_$v -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
done
tools/gpu_steps.sh "${steps[@]}"
