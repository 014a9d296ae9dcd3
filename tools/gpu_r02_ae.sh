cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "kt_k0:300:HIP_FORCE_DEV_KERNARG=0 bash tools/exp_times.sh" \
 "kt_k1:300:HIP_FORCE_DEV_KERNARG=1 bash tools/exp_times.sh" \
 "b_k0:300:HIP_FORCE_DEV_KERNARG=0 python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/b_k0.json" \
 "b_k1:300:HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/b_k1.json"
