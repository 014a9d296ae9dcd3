cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in gp1c16 gp1c32 gp2c16 gp2c32; do
  steps+=("p_$v:200:LFG_LIB=build/exp/liblfg_$v.so rocprofv3 --kernel-trace -d gpurun_out/ax_$v -o run --output-format csv -- python3 bench.py --config gp --steps 10 --warmup 2 --no-cpu")
done
tools/gpu_steps.sh "${steps[@]}"
