"""Full-size golden fixtures (VERDICT r01 "next" 2): the oracle's batched
schedule at the EXACT configurations bench.py measures (SURVEY §8(d) cfg 2-5,
plus the slippery cfg 2 variant): per-GPU lane counts, learner-group sizes,
K = 64, the batched schedule bench.py uses (reset-and-step for cfg 4 / 5) and
the reference CLI's default ε schedule (n_episodes 1e5,
src/bin/frozen_lake.rs:35-73,84), two launches (128 synchronous steps of every
lane, two merges).  Stored: raw fixed-point Q, a SHA-256 of Q as f64 bits
(covers the NaN/±inf flags of cfg 3), UCB counters and t, stats (clamp and
saturation counts included) and a SHA-256 of every lane's ε.

The GPU suite (`tests/test_gpu_fullsize.py`) runs the device with bench.py's
own presets, i.e. the same kernel instantiations the bench launches, and
compares bit for bit against this file; the CPU suite regenerates it from the
oracle (`tests/test_oracle_fullsize.py`).  Reference loop:
/root/reference/src/agent.rs:86-106.

    python tests/golden/make_fullsize.py        (about a minute on 5 cores)
"""
import base64
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)

LAUNCHES = 2
SYNC = 64
CASES = {"cfg2": (2, {}), "cfg2_slippery": (2, {"slippery": 1}), "cfg3": (3, {}), "cfg4": (4, {}),
         "cfg5": (5, {}), "cfg8": (8, {}),
         # BASELINE's whole cfg 4 (2^19 lanes) on one GPU, as bench.py --config 4 --lanes 524288
         "cfg4_2p19": (4, {"n_lanes": 1 << 19})}


def bench_params(cfg, extra):
    """bench.py's preset for SURVEY cfg `cfg`, as default_params keyword arguments"""
    import bench
    pr = dict(bench.PRESETS[cfg])
    kw = dict(env=pr["env"], agent=pr["agent"], policy=pr["policy"], selector=pr["selector"],
              algo=pr["algo"], n_lanes=pr["lanes"], group_size=pr["group"], sync_every=SYNC,
              reset_step=pr.get("reset_step", 0))
    if pr["env"] == "frozen_lake":
        kw["map8x8"] = 1
    kw.update(extra)
    return kw


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case(name):
    import oracle_ffi as O
    cfg, extra = CASES[name]
    kw = bench_params(cfg, extra)
    b = O.Batch(O.default_params(**{k: v for k, v in kw.items() if k != "reset_step"}))
    b.set_reset_step(bool(kw["reset_step"]))
    b.run(LAUNCHES)
    out = {"survey_cfg": cfg, "params": kw, "launches": LAUNCHES,
           "q_raw_i64_b64": b64(b.q_raw().astype("<i8")),
           "q_f64_sha256": sha(b.q().astype("<f8")),
           "stats_u64": [int(x) for x in b.stats()[:10]],
           "eps_sha256": sha(b.lane_eps().astype("<f8"))}
    if kw.get("selector") == "ucb":
        n, t = b.ucb()
        out["ucb_n_u64_b64"] = b64(np.asarray(n, "<u8"))
        out["ucb_t"] = int(t)
    return name, out


def generate(workers=5, only=None, old=None):
    names = [k for k in CASES if only is None or k in only]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        res = dict(ex.map(case, names))
    return {"source": "tests/golden/make_fullsize.py (oracle/rlref.c batched schedule, seed 0x5EED)",
            **{k: res[k] if k in res else old[k] for k in CASES if k in res or (old and k in old)}}


if __name__ == "__main__":
    # python make_fullsize.py [name ...]: regenerate only these cases, keep the others
    path = os.path.join(HERE, "fullsize.json")
    only = sys.argv[1:] or None
    old = json.load(open(path)) if only else None
    json.dump(generate(only=only, old=old), open(path, "w"), indent=1)
    print("wrote", path, os.path.getsize(path), "bytes")
