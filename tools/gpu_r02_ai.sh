cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "tr_spec:300:rocprofv3 --kernel-trace -d gpurun_out/drift_spec -o run --output-format csv -- python3 tools/chain_drift.py 1000 50" \
 "tr_nospec:300:LFG_SPEC=0 rocprofv3 --kernel-trace -d gpurun_out/drift_nospec -o run --output-format csv -- python3 tools/chain_drift.py 1000 50"
