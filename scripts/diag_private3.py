import sys, os
sys.path.insert(0, "rl-rust_amd"); sys.path.insert(0, "tests")
import numpy as np, rlamd, oracle_ffi as O
os.environ["RLAMD_DEBUG_LANES"] = "gpurun_out/lanes.bin"
os.makedirs("gpurun_out", exist_ok=True)
if os.path.exists("gpurun_out/lanes.bin"): os.remove("gpurun_out/lanes.bin")
L, K = 64, 50
p = rlamd.default_params(env="frozen_lake", n_lanes=L, group_size=1, sync_every=K, n_episodes_for_decay=30)
d = rlamd.Agent(p); d.set_recording(True); d.train(30, 10)
dr = d.records()
core = np.fromfile("gpurun_out/lanes.bin", np.uint32).reshape(-1, L, 4)
print("launches", core.shape[0])
# record-derived train episodes completed by the end of each launch
te = np.cumsum(((dr["term"] == 1) & (dr["mode"] == 0)), axis=0)
for ln in range(core.shape[0]):
    rec_cnt = te[(ln + 1) * K - 1]
    dev_cnt = core[ln, :, 3]
    bad = np.nonzero(rec_cnt != dev_cnt)[0]
    if bad.size:
        l = bad[0]
        print("launch", ln, "lanes", bad[:8], "rec", rec_cnt[l], "core.w", dev_cnt[l], "y", hex(core[ln, l, 1]),
              "prev y", hex(core[ln - 1, l, 1]) if ln else None)
        ks = slice(max(0, ln * K - 3), (ln + 1) * K)
        m = dr[ks, l]
        print("  recs", [(int(x["s"]), int(x["s2"]), int(x["term"]), int(x["mode"])) for x in m][-K-3:])
        break
