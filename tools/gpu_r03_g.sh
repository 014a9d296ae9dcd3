cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=("b2:200:python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/g_b2.json")
for v in main NOQ NOWDD; do
  lib=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so; [ $v = main ] && lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
  steps+=("p5_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace --stats -d gpurun_out/g_prof5_$v -o run --output-format csv -- python3 bench.py --config 5 --steps 4 --warmup 1 --no-cpu")
done
tools/gpu_steps.sh "${steps[@]}"
