#!/bin/bash
# One measurement pass on a GPU box (run through gpurun from the repo root):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_pass.sh <tag> [steps...]'
# Steps (default: all, in this order; each under its own time limit, the
# first fault / abort / timeout ends the pass -- tools/gpu_steps.sh):
#   test   pytest -m gpu                    smoke  __graft_entry__.smoke()
#   c2     bench config 2 (100 steps, CPU baselines)   c2_20  the driver's 20-step command
#   c2_20two, gp_two, c3_two  the same on the two-kernel layout (LFG_PAIR=0)
#   p2     rocprofv3 kernel trace of config 2          pmc2   PMC passes of config 2 (tools/pmc_profile.sh)
#   c3 c4 c4e c5 gp xch   benches (config 4 one-of-eight rehearsal, GP example, exchange path)
#   p5 pgp rocprofv3 kernel traces of config 5 and the GP example
#   tl2    k_elements per-wave timeline (needs build/exp/liblfg_ELEMPROF.so: tools/build_exp.sh ELEMPROF -DLFG_PROFILE_ELEM)
#   like2  k_lnlike phase stamps (needs build/exp/liblfg_LIKEPROF.so: tools/build_exp.sh LIKEPROF -DLFG_PROFILE_LIKE)
# LFG_LIB=<path> in the environment runs every step on that build instead.
# Outputs: gpurun_out/<tag>_<step>.{log,json}, gpurun_out/<tag>_prof*/, gpurun_out/pmc_<tag>2/.
tag=${1:?usage: gpu_pass.sh <tag> [steps...]}
shift
steps=${*:-"test smoke c2 c2_20 p2 pmc2 c3 c4 c4e c5 gp xch p5 pgp"}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E=$GRAFT_REPO_ROOT/build/exp
O=gpurun_out
args=()
for s in $steps; do
  case $s in
    test)  args+=("${tag}_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread") ;;
    smoke) args+=("${tag}_smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'") ;;
    c2)    args+=("${tag}_c2:300:python3 bench.py > $O/${tag}_c2.json") ;;
    c2_20) args+=("${tag}_c2_20:200:python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/${tag}_c2_20.json") ;;
    c2_20two) args+=("${tag}_c2_20two:200:LFG_PAIR=0 python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/${tag}_c2_20_two.json") ;;
    p2)    args+=("${tag}_p2:200:rocprofv3 --kernel-trace --stats -d $O/${tag}_prof2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu") ;;
    pmc2)  args+=("${tag}_pmc2:900:bash tools/pmc_profile.sh ${tag}2") ;;
    c3)    args+=("${tag}_c3:300:python3 bench.py --config 3 --steps 30 > $O/${tag}_c3.json") ;;
    c4)    args+=("${tag}_c4:300:python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/${tag}_c4.json") ;;
    c4e)   args+=("${tag}_c4e:300:python3 bench.py --config 4 --emulate-rank 0/8 --steps 20 --warmup 3 --no-cpu > $O/${tag}_c4_emu8.json") ;;
    c5)    args+=("${tag}_c5:300:python3 bench.py --config 5 --steps 20 --warmup 3 > $O/${tag}_c5.json") ;;
    gp)    args+=("${tag}_gp:300:python3 bench.py --config gp --steps 100 --warmup 5 > $O/${tag}_gp.json") ;;
    gp_two) args+=("${tag}_gp_two:300:LFG_PAIR=0 python3 bench.py --config gp --steps 100 --warmup 5 > $O/${tag}_gp_two.json") ;;
    c3_two) args+=("${tag}_c3_two:300:LFG_PAIR=0 python3 bench.py --config 3 --steps 30 --no-cpu > $O/${tag}_c3_two.json") ;;
    xch)   args+=("${tag}_xch:200:python3 bench.py --exchange-path --no-cpu > $O/${tag}_c2_xch.json") ;;
    p5)    args+=("${tag}_p5:300:rocprofv3 --kernel-trace --stats -d $O/${tag}_prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 6 --warmup 2 --no-cpu") ;;
    pgp)   args+=("${tag}_pgp:200:rocprofv3 --kernel-trace --stats -d $O/${tag}_profgp -o run --output-format csv -- python3 bench.py --config gp --steps 30 --warmup 3 --no-cpu") ;;
    tl2)   args+=("${tag}_tl2:200:LFG_DIAGNOSTIC=1 LFG_LIB=$E/liblfg_ELEMPROF.so python3 tools/elem_timeline.py --config 2") ;;
    like2) args+=("${tag}_like2:200:LFG_DIAGNOSTIC=1 LFG_LIB=$E/liblfg_LIKEPROF.so python3 tools/like_profile.py 512 300 1") ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
tools/gpu_steps.sh "${args[@]}"
exit $?
