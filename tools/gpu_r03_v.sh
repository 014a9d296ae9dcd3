# k_elements per-wave timeline (diagnostic build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "v_tl2:200:LFG_LIB=$GRAFT_REPO_ROOT/build/exp/liblfg_ELEMPROF.so python3 tools/elem_timeline.py --config 2" \
 "v_tl3:200:LFG_LIB=$GRAFT_REPO_ROOT/build/exp/liblfg_ELEMPROF.so python3 tools/elem_timeline.py --config 3 --walkers 2048"
