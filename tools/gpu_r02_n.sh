cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 env LFG_LIB=build/exp/liblfg_psetup.so python tools/setup_profile.py > gpurun_out/psetup.log 2>&1 &&
timeout -k 10 600 bash tools/exp_times.sh empty noprior nostream > gpurun_out/exp_n.log 2>&1
