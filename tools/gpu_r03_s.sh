# k_elements at 5 waves/SIMD vs 4; and the emulation profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
steps=()
for v in main MINW5; do
  lib=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so; [ $v = main ] && lib=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
  steps+=("s2_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/s_prof2_$v -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
  steps+=("s3_$v:200:LFG_LIB=$lib rocprofv3 --kernel-trace -d gpurun_out/s_prof3_$v -o run --output-format csv -- python3 bench.py --config 3 --steps 20 --warmup 3 --no-cpu")
done
for v in nospot nodon; do
  steps+=("s5_$v:300:LFG_LIB=$GRAFT_REPO_ROOT/build/exp/liblfg_$v.so rocprofv3 --kernel-trace -d gpurun_out/s_prof5_$v -o run --output-format csv -- python3 bench.py --config 5 --steps 4 --warmup 1 --no-cpu")
done
steps+=("s_pe:300:rocprofv3 --kernel-trace --stats -d gpurun_out/s_prof_emu8 -o run --output-format csv -- python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu --emulate-rank 0/8")
tools/gpu_steps.sh "${steps[@]}"
