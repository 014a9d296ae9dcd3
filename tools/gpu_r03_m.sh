# full GPU suite + GP / config-5 / config-2 bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "m_test:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "m_bgp:200:python3 bench.py --config gp --steps 50 --warmup 5 --no-cpu > gpurun_out/m_gp.json" \
 "m_b5:300:python3 bench.py --config 5 --steps 20 --warmup 3 --no-cpu > gpurun_out/m_c5.json" \
 "m_b2:200:python3 bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/m_c2.json"
