#!/bin/bash
# A/B of exp builds on configs 5, 2, gp, and config 4's one-of-eight rehearsal
cd $GRAFT_REPO_ROOT
n=${NAMES:-nolicm}
bash tools/gpu_abn.sh "$n" 2 --config 5 --steps 20 --warmup 5 --no-cpu && \
bash tools/gpu_abn.sh "$n" 3 --steps 20 --warmup 5 --no-cpu && \
bash tools/gpu_abn.sh "$n" 1 --config gp --steps 10 --warmup 3 --no-cpu && \
bash tools/gpu_abn.sh "$n" 1 --config 4 --emulate-rank 0/8 --steps 20 --warmup 5 --no-cpu
