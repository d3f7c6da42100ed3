"""Full training horizon fixtures: ONE learner group per
SURVEY §8(d) configuration at bench.py's group size and K (cfg 2 / 3 / 5: 512
lanes, cfg 4: 256), trained with the reference CLI's schedule —
Agent::train(env, n_episodes = 1e5, eval_at = n_episodes / 10) per lane
(src/agent.rs:66-118, src/bin/frozen_lake.rs:35-84) with the ε decay over
1e5 episodes — so every ε-greedy lane ends at its stall residue
(uniform_epsilon_greed.rs:42-49).

Stored per case: raw Q words, representation, NaN / ±inf counts, stats, every
lane's final ε (its SHA-256 and the distinct values), UCB counters.  Also stored,
as a MEASUREMENT over the same horizon: the L∞ between this run and
  - cfg 2 (fixed point, range proven): the same schedule held in f64 (the
    oracle's RLO_QMODE_F64) — the fixed point's 2^-40 truncation drift;
  - cfg 3 / 4 / 5 (f64): the same schedule with every step / merge sum formed
    sequentially in lane / group order (RLO_QMODE_F64_SEQ).
A drift run whose trajectories part from the fixture's (a changed argmax moves a
lane elsewhere) shows it in `records_diverged`-free form: the step counts.

    python tests/golden/make_horizon.py      (~15 min on 8 cores: cfg 3's Taxi lanes run 1e7 steps each)
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

N_EPISODES = 100000
CASES = ("cfg2", "cfg3", "cfg4", "cfg5")


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def horizon_params(cfg):
    """bench.py's preset with ONE learner group (n_lanes = group size)"""
    from make_fullsize import bench_params
    kw = bench_params(cfg, {})
    kw["n_lanes"] = kw["group_size"]
    return kw


def run(job):
    import oracle_ffi as O
    name, mode = job
    kw = horizon_params(int(name[3:]))
    b = O.Batch(O.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    b.set_reset_step(bool(kw["reset_step"]))
    if mode != "auto":
        b.set_q_mode(mode)
    b.train_episodes(N_EPISODES, N_EPISODES // 10)
    q = b.q()
    out = {"q": q, "q_repr": b.q_repr(), "q_raw": b.q_raw().astype("<i8"), "stats": [int(x) for x in b.stats()[:10]],
           "eps": b.lane_eps().astype("<f8")}
    if kw.get("selector") == "ucb":
        n, t = b.ucb()
        out["ucb"] = (np.asarray(n, "<u8"), int(t))
    return name, mode, kw, out


def generate(workers=8, only=None, old=None):
    cases = [n for n in CASES if only is None or n in only]
    jobs = [(n, "auto") for n in cases] + [(n, "f64" if n == "cfg2" else "f64_seq") for n in cases]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(run, jobs))
    main = {n: (kw, o) for n, m, kw, o in res if m == "auto"}
    drift = {n: (m, o) for n, m, kw, o in res if m != "auto"}
    doc = {"source": "tests/golden/make_horizon.py (oracle/rlref.c batched schedule, seed 0x5EED)",
           "n_episodes": N_EPISODES, "eval_at": N_EPISODES // 10}
    for n in CASES:
        if n not in main:
            doc[n] = old[n]
            continue
        kw, o = main[n]
        q = o["q"]
        fin = np.isfinite(q)
        g = {"survey_cfg": int(n[3:]), "params": kw, "q_repr": o["q_repr"], "q_raw_i64_b64": b64(o["q_raw"]),
             "n_nan": int(np.isnan(q).sum()), "n_inf": int(np.isinf(q).sum()),
             "max_abs_finite": float(np.abs(q[fin]).max()) if fin.any() else 0.0,
             "stats_u64": o["stats"], "eps_sha256": sha(o["eps"]),
             "eps_values": sorted({float(x) for x in o["eps"]})}
        if "ucb" in o:
            g["ucb_n_u64_b64"] = b64(o["ucb"][0])
            g["ucb_t"] = o["ucb"][1]
        m, d = drift[n]
        qd = d["q"]
        both = np.isfinite(q) & np.isfinite(qd)
        diff = np.abs(q[both] - qd[both])
        g["drift"] = {"against": "f64 (RLO_QMODE_F64)" if m == "f64" else "sequential-order f64 sums (RLO_QMODE_F64_SEQ)",
                      "nan_masks_equal": bool(np.array_equal(np.isnan(q), np.isnan(qd))),
                      "linf": float(diff.max()) if diff.size else 0.0,
                      "rel_linf": float((diff / np.maximum(np.abs(q[both]), 1.0)).max()) if diff.size else 0.0,
                      "train_steps": [o["stats"][0], d["stats"][0]],
                      "eps_equal": bool(np.array_equal(o["eps"], d["eps"]))}
        doc[n] = g
    return doc


if __name__ == "__main__":
    # python make_horizon.py [cfgN ...]: regenerate only these cases, keep the others
    path = os.path.join(HERE, "horizon.json")
    only = sys.argv[1:] or None
    old = json.load(open(path)) if only else None
    json.dump(generate(only=only, old=old), open(path, "w"), indent=1)
    print("wrote", path, os.path.getsize(path), "bytes")
