cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_gp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_gp/p1 -o run --output-format csv -- python3 $R/bench.py --config gp --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/pmc_gp/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -d $R/gpurun_out/pmc_gp/p2 -o run --output-format csv -- python3 $R/bench.py --config gp --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/pmc_gp/p2.log 2>&1 && echo done
