"""The fixed point's drift from f64, launch by launch (VERDICT r05 weak item 1 /
next item 7): is cfg 2-slippery's 1.06e-4 L-inf after 65 launches a FLIP (the
two representations agree to the 2^-40 grid until one greedy argmax tie breaks
the other way, after which the lanes' trajectories part) or an ACCUMULATION (a
difference that grows every launch)?

Two oracle batches (oracle/rlref.c, the batched schedule bench.py runs) over the
same lanes, draws and merges: the fixed point (2^-40, "fixed_range": round 5's
"auto", which round 6 no longer takes on slippery maps) and f64 with
exact-grid sums ("f64"; both order-free, so the difference is the representation
alone).  After every launch: the L-inf of Q, the states whose greedy action
(utils::argmax, first maximum) differs, and whether the run statistics (train
env-steps, episodes, rewards) are still identical — they are exactly while every
lane took the same actions in both.

    python tests/golden/make_drift_curve.py [cfg2_slippery cfg2]   (minutes: 2 x 65 launches of 2^20 lanes)

Writes the curves into longrun.json[case]["repr_drift_curve"].
"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from make_longrun import CASES, LAUNCHES  # noqa: E402


def curve(name):
    import oracle_ffi as O
    from make_fullsize import bench_params
    cfg, extra = CASES[name]
    kw = bench_params(cfg, extra)
    bs = []
    for mode in ("fixed_range", "f64"):
        b = O.Batch(O.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
        b.set_reset_step(bool(kw["reset_step"]))
        b.set_q_mode(mode)
        bs.append(b)
    assert bs[0].q_repr() == "fixed40" and bs[1].q_repr() == "f64", [b.q_repr() for b in bs]
    rows = []
    for launch in range(1, LAUNCHES[name] + 1):
        for b in bs:
            b.run(1)
        qa, qb = bs[0].q(), bs[1].q()
        d = np.abs(qa - qb)
        s = [b.stats()[:6] for b in bs]
        rows.append({"launch": launch, "linf": float(d.max()),
                     "argmax_states_differ": int((np.argmax(qa, axis=-1) != np.argmax(qb, axis=-1)).sum()),
                     "stats_equal": bool(np.array_equal(s[0], s[1]))})
        print(name, rows[-1], flush=True)
    first_part = next((r["launch"] for r in rows if not r["stats_equal"]), None)
    return name, {"what": "fixed point 2^-40 vs f64 exact-grid sums (both order-free), after each launch: "
                          "Q L-inf, states whose greedy action differs, run stats identical (same trajectories)",
                  "first_launch_trajectories_part": first_part, "per_launch": rows}


def main():
    names = sys.argv[1:] or ["cfg2_slippery", "cfg2"]
    with ProcessPoolExecutor(max_workers=len(names)) as ex:
        res = dict(ex.map(curve, names))
    path = os.path.join(HERE, "longrun.json")
    lr = json.load(open(path))
    for k, v in res.items():
        lr[k]["repr_drift_curve"] = v
    json.dump(lr, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
