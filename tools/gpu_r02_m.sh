cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "psetup:120:LFG_LIB=build/exp/liblfg_psetup.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_psetup -o run -- python3 tools/setup_profile.py"
