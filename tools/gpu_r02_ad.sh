cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "exptimes:300:bash tools/exp_times.sh"
