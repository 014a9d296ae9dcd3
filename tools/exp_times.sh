#!/bin/bash
# rocprofv3 kernel stats of tools/kernel_time.py for the main library and
# each experiment build given on the command line (build/exp/liblfg_<name>.so, tools/build_exp.sh)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -f $R/gpurun_out/kernel_time_walkers.npy
for v in main "$@"; do
  if [ "$v" = main ]; then lib=$R/lfit_python_amd/_lib/liblfg_hip.so; else lib=$R/build/exp/liblfg_$v.so; fi
  LFG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp_$v -o run --output-format csv \
    -- python3 $R/tools/kernel_time.py 30 > $R/gpurun_out/exp_$v.log 2>&1 || { echo "$v failed"; exit 3; }
  echo "== $v"
  python3 - $R/gpurun_out/exp_$v/run_kernel_trace.csv <<'PY'
import csv, collections, sys
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
    if r['Grid_Size_X'] and n.startswith('k_'):
        d[(n, r['Grid_Size_X'])].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in sorted(d.items()):
    if len(v) >= 10:
        v = sorted(v); print('  %-22s grid %8s n %3d median %7.1f us' % (k[0], k[1], len(v), v[len(v)//2] / 1e3))
PY
done
python3 - $R/gpurun_out <<'PY'
import glob, os, sys, numpy as np
d = sys.argv[1]
ref = np.load(os.path.join(d, "kt_lnp_hip.npy")) if os.path.exists(os.path.join(d, "kt_lnp_hip.npy")) else None
for f in sorted(glob.glob(os.path.join(d, "kt_lnp_*.npy"))):
    v = np.load(f)
    if ref is not None:
        ok = np.isfinite(ref) & np.isfinite(v)
        print("  %-28s max |dlnp| vs main %.3g  finite-pattern same %s" % (os.path.basename(f), np.abs(v[ok] - ref[ok]).max(), bool((np.isfinite(ref) == np.isfinite(v)).all())))
PY
