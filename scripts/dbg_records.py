"""Debug helper (GPU box): run one shared-mode case on the device and in the
oracle launch by launch and print where the step records / Q first diverge.
usage: python scripts/dbg_records.py 'env=taxi,agent=traces,selector=ucb,algo=expected_sarsa,group_size=256'"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi  # noqa: E402
import rlamd  # noqa: E402

kw = {}
for part in sys.argv[1].split(","):
    k, v = part.split("=")
    kw[k] = int(v) if v.lstrip("-").isdigit() else v
L = int(os.environ.get("LANES", 600))
p = rlamd.default_params(n_lanes=L, sync_every=int(os.environ.get("SYNC", 16)), n_episodes_for_decay=40, **kw)
dev = rlamd.Agent(p)
dev.set_recording(True)
ref = oracle_ffi.Batch(p)
ref.set_record(True)
for launch in range(6):
    dev.run(1)
    ref.run(1)
    d, r = dev.records(), ref.records()
    bad = np.zeros(d.shape, bool)
    for f in ["s", "s2", "a", "a2", "term", "mode"]:
        bad |= d[f] != r[f]
    for f in ["r", "td"]:
        a, b = d[f], r[f]
        bad |= (a.view(np.uint64) != b.view(np.uint64)) & ~(np.isnan(a) & np.isnan(b))
    qd, qr = dev.q_raw(), ref.q_raw()
    nq = int(np.sum(qd != qr))
    fd, fr = np.isnan(dev.q()), np.isnan(ref.q())
    print("NaN entries dev", int(fd.sum()), "ref", int(fr.sum()), "mask diffs", int((fd != fr).sum()),
          "first", np.argwhere(fd != fr)[:6].tolist())
    print(f"launch {launch}: record diffs {int(bad.sum())}, Q raw diffs {nq}")
    if bad.any() or nq:
        k0 = int(np.argwhere(bad.any(axis=1))[0][0]) if bad.any() else -1
        lanes = np.argwhere(bad[k0])[:, 0][:8] if k0 >= 0 else []
        print("first bad step", k0, "lanes", lanes, "n lanes bad at that step", int(bad[k0].sum()) if k0 >= 0 else 0)
        for ln in lanes[:3]:
            for k in range(max(0, k0 - 3), min(d.shape[0], k0 + 2)):
                print(f"  k={k} lane={ln} dev={d[k, ln]} ref={r[k, ln]}")
        if nq:
            idx = np.argwhere(qd != qr)[:8]
            print("Q diffs at", idx.tolist(), qd[qd != qr][:8], qr[qd != qr][:8])
        break
