cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "drift:300:python -u tools/chain_drift.py 2000 50" \
 "count:200:LFG_LIB=build/exp/liblfg_count.so python -u tools/chain_drift.py count"
