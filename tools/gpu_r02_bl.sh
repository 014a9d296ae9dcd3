cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "plike2:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 512 300 1" \
 "plike5:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 64 10000 5"
