import numpy as np, sys
t = np.load(sys.argv[1]).astype(np.float64)
t0 = t[0]; fin = (t[15] - t0.min())/100.0
hw = t[14].astype(np.int64)
# HW_ID (gfx9): wave_id[3:0], simd_id[5:4], pipe[7:6], cu_id[11:8], sh_id[12], se_id[15:13] (gfx950: se bits wider?)
cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7
xcc = t[18].astype(np.int64) & 0xF
key = xcc * 256 + se * 32 + sh * 16 + cu
print("distinct (se,sh,cu):", len(np.unique(key)), "of", len(key))
vals, cnt = np.unique(key, return_counts=True)
print("blocks per slot histogram:", np.bincount(cnt))
# per slot: max finish
slow = fin > np.percentile(fin, 80)
sk = key[slow]
print("slow blocks:", slow.sum(), "distinct slots among them:", len(np.unique(sk)))
order = np.argsort(fin)
print("slowest 10 blocks: block, finish, slot, start:", [(int(b), round(fin[b],1), int(key[b]), round((t0[b]-t0.min())/100,2)) for b in order[-10:]])
