cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "exptimes:400:bash tools/exp_times.sh th6 th4 atomtid" \
 "plike:120:LFG_LIB=build/exp/liblfg_plike.so python tools/like_profile.py 512 300 1"
