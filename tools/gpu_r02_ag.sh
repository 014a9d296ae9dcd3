cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in main o5 o6 o8 i6 i8; do
  if [ $v = main ]; then lib=lfit_python_amd/_lib/liblfg_hip.so; else lib=build/exp/liblfg_$v.so; fi
  steps+=("b_$v:200:LFG_LIB=$lib python bench.py --steps 200 --warmup 5 --no-cpu > gpurun_out/ag_$v.json")
done
steps+=("b_main2:200:python bench.py --steps 200 --warmup 5 --no-cpu > gpurun_out/ag_main2.json")
tools/gpu_steps.sh "${steps[@]}"
