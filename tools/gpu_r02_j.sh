cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "psetup:120:LFG_LIB=build/exp/liblfg_psetup.so python tools/setup_profile.py" \
 "plike:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 512 300 1"
