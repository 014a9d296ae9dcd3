cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
B=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
steps=()
for v in base WALK1 WALK3; do
  lib=$B; [ $v != base ] && lib=$E/liblfg_$v.so
  steps+=("w_p_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/w_prof_$v -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
  steps+=("w_p3_$v:300:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/w_prof3_$v -o run --output-format csv -- python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu")
done
tools/gpu_steps.sh "${steps[@]}"
