set -e
mkdir -p gpurun_out/abl
for v in PAIRPROF P_SCDONOR P_SCTRIG P_SCSPOT P_LSUB P_LWD; do
  LFG_DIAGNOSTIC=1 LFG_LIB=build/exp/liblfg_$v.so timeout -k 10 120 python tools/pair_profile.py 4096 10000 5 > gpurun_out/abl/$v.log 2>&1
done
