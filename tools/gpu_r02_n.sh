cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/exp_times.sh empty noprior nostream > gpurun_out/exp_n.log 2>&1
