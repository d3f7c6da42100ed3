"""Bench-length golden fixtures: the oracle's batched
schedule at bench.py's exact configurations for as many launches as one default
bench run makes (1 warm-up + 64 timed = 65 launches of K = 64 synchronous steps),
so the device is pinned over the whole benchmarked window — past the point where
cfg 5's double tables leave the old fixed-point range (|Q| > 2048) and where
cfg 3's UCB + expected SARSA table is mostly NaN.

Stored per case: raw Q words (f64 bits, NaN canonical), the representation, the
NaN / +-inf counts and the largest finite |Q|, stats, UCB counters, a SHA-256 of
every lane's epsilon.  Also stored, as a MEASUREMENT (not a parity bar): the
same run with every step / merge sum formed sequentially in lane / group order
in f64 (the oracle's RLO_QMODE_F64_SEQ) — the L-inf and relative differences to
the order-free exponent-grid sums the device uses.

    python tests/golden/make_longrun.py          (several minutes: the oracle is one core per case)
"""
import base64
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

LAUNCHES = {"cfg2": 65, "cfg2_slippery": 65, "cfg3": 65, "cfg4": 65, "cfg5": 65, "cfg4_2p19": 65, "cfg8": 65}
# name -> (SURVEY cfg, extra bench.py arguments); cfg 2 is the headline (the
# proven fixed point, k_train_shared_o8: VERDICT r03 item 3)
CASES = {"cfg2": (2, {}), "cfg2_slippery": (2, {"slippery": 1}), "cfg3": (3, {}), "cfg4": (4, {}), "cfg5": (5, {}),
         "cfg8": (8, {}),
         # BASELINE's whole cfg 4 (2^19 lanes) on one GPU, as bench.py --config 4 --lanes 524288
         "cfg4_2p19": (4, {"n_lanes": 1 << 19})}


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run(name, mode):
    import oracle_ffi as O
    from make_fullsize import bench_params
    cfg, extra = CASES[name]
    kw = bench_params(cfg, extra)
    b = O.Batch(O.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    b.set_reset_step(bool(kw["reset_step"]))
    if mode != "auto":
        b.set_q_mode(mode)
    b.run(LAUNCHES[name])
    return kw, b


def _arrays(args):
    """one oracle run's results as plain arrays (picklable: the two modes of a case
    run in parallel processes)"""
    name, mode = args
    kw, b = run(name, mode)
    out = {"kw": kw, "q": b.q(), "q_raw": b.q_raw(), "q_repr": b.q_repr(), "stats": b.stats()[:10],
           "eps": b.lane_eps()}
    if kw.get("selector") == "ucb":
        out["ucb"] = b.ucb()
    return out


def _drift(q, qs):
    both = np.isfinite(q) & np.isfinite(qs)
    d = np.abs(q[both] - qs[both])
    return {"nan_masks_equal": bool(np.array_equal(np.isnan(q), np.isnan(qs))),
            "linf": float(d.max()) if d.size else 0.0,
            "rel_linf": float((d / np.maximum(np.abs(q[both]), 1.0)).max()) if d.size else 0.0}


def case(name):
    # fixed-point cases also run the order-free f64 (exact-grid) schedule, so the
    # drift splits into representation rounding (fixed point vs f64 exact grid,
    # both order-free) and summation order (f64 exact grid vs f64 sequential):
    # VERDICT r04 item 8
    kw0 = __import__("make_fullsize").bench_params(*CASES[name])
    fixed = kw0["agent"] == "one_step" and kw0["policy"] == "tabular" and not (
        kw0["selector"] == "ucb" and kw0["algo"] == "expected_sarsa") and not kw0.get("slippery")
    modes = [(name, "auto"), (name, "f64_seq")] + ([(name, "f64")] if fixed else [])
    with ProcessPoolExecutor(max_workers=len(modes)) as ex:
        res = list(ex.map(_arrays, modes))
    a, sq = res[0], res[1]
    kw = a["kw"]
    q = a["q"]
    fin = np.isfinite(q)
    out = {"survey_cfg": CASES[name][0], "params": kw, "launches": LAUNCHES[name], "q_repr": a["q_repr"],
           "q_raw_i64_b64": b64(a["q_raw"].astype("<i8")),
           "n_nan": int(np.isnan(q).sum()), "n_inf": int(np.isinf(q).sum()),
           "max_abs_finite": float(np.abs(q[fin]).max()) if fin.any() else 0.0,
           "stats_u64": [int(x) for x in a["stats"]],
           "eps_sha256": sha(a["eps"].astype("<f8"))}
    if "ucb" in a:
        n, t = a["ucb"]
        out["ucb_n_u64_b64"] = b64(np.asarray(n, "<u8"))
        out["ucb_t"] = int(t)
    # drift measurement: sequential f64 sums (same draws, same mean rule)
    out["seq_sum_drift"] = _drift(q, sq["q"])
    if fixed:
        qf = res[2]["q"]
        out["repr_drift"] = dict(_drift(q, qf), what="fixed point 2^-40 vs f64 exact-grid sums: both order-free, "
                                                       "the representation alone")
        out["order_drift"] = dict(_drift(qf, sq["q"]), what="f64 exact-grid vs f64 sequential sums: the "
                                                            "summation order alone")
    return name, out


def generate(workers=5, only=None, old=None):
    names = [k for k in LAUNCHES if only is None or k in only]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        res = dict(ex.map(case, names))
    return {"source": "tests/golden/make_longrun.py (oracle/rlref.c batched schedule, seed 0x5EED)",
            **{k: _keep_curve(res[k], old and old.get(k)) if k in res else old[k] for k in LAUNCHES
               if k in res or (old and k in old)}}


def _keep_curve(new, old):
    """the drift curve (make_drift_curve.py) survives a regeneration of its case"""
    if old and "repr_drift_curve" in old:
        new["repr_drift_curve"] = old["repr_drift_curve"]
    return new


if __name__ == "__main__":
    # python make_longrun.py [cfgN ...]: regenerate only these cases, keep the others
    path = os.path.join(HERE, "longrun.json")
    only = sys.argv[1:] or None
    old = json.load(open(path)) if only else None
    json.dump(generate(only=only, old=old), open(path, "w"), indent=1)
    print("wrote", path, os.path.getsize(path), "bytes")
