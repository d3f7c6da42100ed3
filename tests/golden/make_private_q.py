"""Known answers for the private bench rows at full size:
bench.py --config 6 / 7 run 2^20 private lanes (one agent per lane: cfg 6
frozen_lake_neural's NeuralPolicy, cfg 7 cliffwalking_model's Dyna-Q).  Private
lanes are independent and seeded by their global lane id, so the LAST 4096 lanes
of the 2^20-lane run are the oracle's 4096 lanes at lane_offset 2^20 - 4096 —
past 2^32 bytes into cfg 7's per-lane tables, where a 32-bit offset would first
go wrong.  Stored per case: the SHA-256 of those lanes' Q ([lane][P][S][A] f64
bits, NaN canonical; cfg 6: get_values of every state) and, for cfg 6, of their
network parameters ([lane][n_params]), plus the window's training env-steps.

Cases: the driver's window (--steps 20 --warmup 5: 25 launches) and the default
bench run (1 + 64 launches).  bench.py's q_check compares with them;
tests/test_gpu_private_bench.py runs the oracle itself for the 25-launch case.

    python tests/golden/make_private_q.py        (a few minutes: the oracle is one core per case)
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))   # bench.py (its presets)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

GLOBAL = 1 << 20
WINDOW = 4096
CASES = {"cfg6_L1M_last4096_25": (6, 25), "cfg6_L1M_last4096_65": (6, 65),
         "cfg7_L1M_last4096_25": (7, 25), "cfg7_L1M_last4096_65": (7, 65)}


def window_params(cfg):
    """bench.py's preset for cfg 6 / 7 over the window's lanes (oracle_ffi keywords)"""
    import bench
    pr = dict(bench.PRESETS[cfg])
    extra = dict(pr.get("extra", {}))
    planning = extra.pop("planning", 0)
    kw = dict(env=pr["env"], agent=pr["agent"], policy=pr["policy"], selector=pr["selector"], algo=pr["algo"],
              n_lanes=WINDOW, lane_offset=GLOBAL - WINDOW, group_size=pr["group"], sync_every=64)
    kw.update(extra)
    return kw, planning


def f64_sha(x):
    """SHA-256 of f64 words with every NaN canonical (0x7ff8...): the network's NaN
    payloads are not part of the reference's semantics"""
    x = np.ascontiguousarray(x, "<f8")
    return hashlib.sha256(np.where(np.isnan(x), np.nan, x).astype("<f8").tobytes()).hexdigest()


def digests(q, w):
    out = {"q_sha256": f64_sha(q)}
    if w is not None:
        out["w_sha256"] = f64_sha(w)
    return out


def run(name):
    import oracle_ffi as O
    cfg, launches = CASES[name]
    kw, planning = window_params(cfg)
    b = O.Batch(O.default_params(**kw))
    if planning:
        b.set_planning(planning)
    b.run(launches)
    w = b.weights() if cfg == 6 else None
    return name, {"key": {"config": cfg, "global_lanes": GLOBAL, "lane0": GLOBAL - WINDOW, "window": WINDOW,
                          "sync": 64, "launches": launches},
                  **digests(b.q(), w), "train_steps_window": int(b.stats()[0])}


def main():
    import oracle_ffi
    oracle_ffi.build()
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, "private_q.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    out["source"] = ("oracle/rlref.c batched schedule, private lanes [2^20 - 4096, 2^20) of bench.py's cfg 6 / 7 "
                     "presets (tests/golden/make_private_q.py)")
    cases = out.setdefault("cases", {})
    with ProcessPoolExecutor(max_workers=min(len(names), 4)) as ex:
        for name, c in ex.map(run, names):
            cases[name] = c
            print(name, c["q_sha256"][:16], c["train_steps_window"], flush=True)
    out["cases"] = {k: cases[k] for k in sorted(cases)}
    json.dump(out, open(path, "w"), indent=1)
    open(path, "a").write("\n")


if __name__ == "__main__":
    main()
