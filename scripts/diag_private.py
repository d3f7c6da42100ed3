import sys, os
sys.path.insert(0, "rl-rust_amd"); sys.path.insert(0, "tests")
import numpy as np, rlamd, oracle_ffi as O
for L, n_ep, eval_at in [(1, 5, 0), (1, 20, 0), (1, 20, 5), (37, 60, 10)]:
    p = rlamd.default_params(env="frozen_lake", n_lanes=L, group_size=1, sync_every=50, n_episodes_for_decay=n_ep)
    d = rlamd.Agent(p); d.set_recording(True); st = d.train(n_ep, eval_at)
    r = O.Batch(p); r.set_record(True); r.train_episodes(n_ep, eval_at)
    dr, rr = d.records(), r.records()
    print("case", L, n_ep, eval_at, "shapes", dr.shape, rr.shape, "stats", st)
    n = min(len(dr), len(rr))
    bad = None
    for k in range(n):
        for f in ["s", "s2", "a", "a2", "term", "mode", "r", "td"]:
            m = dr[k][f] != rr[k][f]
            if m.any():
                bad = (k, int(np.nonzero(m)[0][0]), f); break
        if bad: break
    print(" first mismatch", bad)
    if bad:
        k, l, f = bad
        for kk in range(max(0, k - 3), min(n, k + 2)):
            print("  dev", kk, dr[kk][l]); print("  ref", kk, rr[kk][l])
    print(" eps dev", d.epsilon()[:3], "ref", r.lane_eps()[:3])
