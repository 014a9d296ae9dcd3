# k_gp_like ablation: element pass vs combine
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in NOELEM NOCOMB; do
  steps+=("l_$v:200:LFG_LIB=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so rocprofv3 --kernel-trace -d gpurun_out/l_prof_$v -o run --output-format csv -- python3 bench.py --config gp --steps 10 --warmup 2 --no-cpu")
done
tools/gpu_steps.sh "${steps[@]}"
