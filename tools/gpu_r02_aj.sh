cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "hunt:400:LFG_LIB=build/exp/liblfg_count.so python -u tools/fallback_hunt.py 1000"
