#!/bin/bash
# Interleaved A/B of experiment builds (tools/build_exp.sh <name>) on one box:
#   gpurun -- 'bash tools/gpu_ab2.sh <tag> <rounds> "<bench.py args>" name1 name2 ...'
# rounds x (each build once, in order), so drift on the box hits every build
# alike; prints value and ms_per_step per run, then the median per build.
tag=$1; rounds=$2; bargs=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
for r in $(seq 1 $rounds); do
  for n in "$@"; do
    L=build/exp/liblfg_$n.so
    LFG_DIAGNOSTIC=1 LFG_LIB=$L timeout -k 10 200 python3 bench.py $bargs --no-cpu > $O/${tag}_${n}_$r.json 2> $O/${tag}_${n}_$r.err || { echo "$n bench failed"; tail -5 $O/${tag}_${n}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline'].get('kernel',{}); print(sys.argv[2], round(d['value']/1e6,4), round(d['ms_per_step']*1e3,2), round(k.get('avg_launch_ms',0)*1e3,2))" $O/${tag}_${n}_$r.json $n
  done
done
python3 - "$O" "$tag" "$rounds" "$@" <<'PY'
import json, sys, statistics
O, tag, rounds, names = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
for n in names:
    v = [json.load(open("%s/%s_%s_%d.json" % (O, tag, n, r)))["value"] / 1e6 for r in range(1, rounds + 1)]
    print("median", n, round(statistics.median(v), 4), "runs", [round(x, 3) for x in v])
PY
