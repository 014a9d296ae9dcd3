# LLVM scheduling strategies for the whole library (max-ilp, max-memory-clause) against the default
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
steps=()
for v in base MAXILP MEMCL; do
  lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so; [ $v != base ] && lib=$E/liblfg_$v.so
  steps+=("s_b_$v:200:LFG_LIB=$lib python3 bench.py --no-cpu > gpurun_out/s_c2_$v.json")
  steps+=("s_p_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/s_prof_$v -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
done
for v in base MAXILP MEMCL; do
  lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so; [ $v != base ] && lib=$E/liblfg_$v.so
  steps+=("s_b2_$v:200:LFG_LIB=$lib python3 bench.py --no-cpu > gpurun_out/s_c2b_$v.json")
done
tools/gpu_steps.sh "${steps[@]}"
