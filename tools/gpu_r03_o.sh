# config-3 regression hunt: the same bench on libraries of earlier commits
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in main 70056c4 7f5b60b 34a4e4f 8058fb0; do
  lib=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so; [ $v = main ] && lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
  steps+=("o_$v:200:LFG_LIB=$lib python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/o_c3_$v.json")
done
tools/gpu_steps.sh "${steps[@]}"
