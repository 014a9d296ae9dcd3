# two donor tiles per k_elements lane (14 chunks per pair instead of 15) against the in-tree build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
B=$GRAFT_REPO_ROOT/lfit_python_amd/_lib/liblfg_hip.so
steps=("d_test:900:LFG_LIB=$E/liblfg_DONOR2.so python -u -m pytest tests -m 'gpu and not perf' -x -q --timeout 300 --timeout-method thread")
for r in a b; do
  steps+=("d_b_D2_$r:200:LFG_LIB=$E/liblfg_DONOR2.so python3 bench.py --no-cpu > gpurun_out/d_c2_D2_$r.json")
  steps+=("d_b_base_$r:200:LFG_LIB=$B python3 bench.py --no-cpu > gpurun_out/d_c2_base_$r.json")
done
steps+=("d_p_D2:200:LFG_LIB=$E/liblfg_DONOR2.so rocprofv3 --kernel-trace -d gpurun_out/d_prof_D2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
steps+=("d_p_base:200:LFG_LIB=$B rocprofv3 --kernel-trace -d gpurun_out/d_prof_base -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu")
steps+=("d_c3_D2:300:LFG_LIB=$E/liblfg_DONOR2.so python3 bench.py --config 3 --steps 30 --no-cpu > gpurun_out/d_c3_D2.json")
steps+=("d_c3_base:300:LFG_LIB=$B python3 bench.py --config 3 --steps 30 --no-cpu > gpurun_out/d_c3_base.json")
steps+=("d_gp_D2:300:LFG_LIB=$E/liblfg_DONOR2.so python3 bench.py --config gp --steps 50 --no-cpu > gpurun_out/d_gp_D2.json")
steps+=("d_gp_base:300:LFG_LIB=$B python3 bench.py --config gp --steps 50 --no-cpu > gpurun_out/d_gp_base.json")
tools/gpu_steps.sh "${steps[@]}"
