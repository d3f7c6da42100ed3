import sys
sys.path.insert(0, "rl-rust_amd"); sys.path.insert(0, "tests")
import numpy as np, rlamd, oracle_ffi as O
for L, n_ep, eval_at, K in [(64, 30, 10, 50), (64, 30, 8, 50), (64, 30, 10, 5000)]:
    p = rlamd.default_params(env="frozen_lake", n_lanes=L, group_size=1, sync_every=K, n_episodes_for_decay=n_ep)
    d = rlamd.Agent(p); d.set_recording(True); st = d.train(n_ep, eval_at)
    r = O.Batch(p); r.set_record(True); r.train_episodes(n_ep, eval_at)
    dr, rr = d.records(), r.records()
    print("case", L, n_ep, eval_at, K, dr.shape, rr.shape, "train_eps", st["train_episodes"], "expect", L * n_ep)
    n = min(len(dr), len(rr))
    first = []
    for l in range(L):
        m = np.nonzero((dr[:n, l]["mode"] != rr[:n, l]["mode"]) | (dr[:n, l]["s2"] != rr[:n, l]["s2"]))[0]
        first.append(int(m[0]) if m.size else -1)
    print(" first mismatch per lane:", first)
    # per-lane train episodes on device
    te = ((dr["term"] == 1) & (dr["mode"] == 0)).sum(0)
    print(" dev train eps per lane:", te.tolist())
