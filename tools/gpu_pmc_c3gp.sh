# PMC passes of config 3 and the GP example (traffic and executed FP64 tables for bench.py's roofline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "pm_c3:900:bash tools/pmc_profile.sh c3z --config 3 --steps 15 --warmup 2" \
 "pm_gp:900:bash tools/pmc_profile.sh gpz --config gp --steps 15 --warmup 2"
