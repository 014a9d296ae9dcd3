#!/bin/bash
# A/B of experiment builds (tools/build_exp.sh <name>) on one GPU box:
#   gpurun -- 'bash tools/gpu_ab.sh <tag> "<env>" name1 name2 ...'
# per build: the GPU ln_prob parity tests (not with AB_NOTEST=1), then the driver's 20-step config-2
# bench line, each under its own time limit; the first failure ends the pass.
tag=$1; envs=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
for n in "$@"; do
  L=build/exp/liblfg_$n.so
  [ -n "$AB_NOTEST" ] || env $envs LFG_DIAGNOSTIC=1 LFG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_lnprob.py -m gpu -x -q \
      --timeout 200 --timeout-method thread > $O/${tag}_${n}_test.log 2>&1 || { echo "$n tests failed"; tail -30 $O/${tag}_${n}_test.log; exit 1; }
  [ -n "$AB_NOTEST" ] || tail -1 $O/${tag}_${n}_test.log
  for r in 1 2; do
    env $envs LFG_DIAGNOSTIC=1 LFG_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/${tag}_${n}_c2_$r.json || { echo "$n bench failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))" $O/${tag}_${n}_c2_$r.json $n
  done
done
