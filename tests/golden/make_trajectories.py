"""Golden trajectories (SURVEY §8(c) ii): the oracle run on each BASELINE
config at small size, committed as data so that later changes to the oracle
or the kernels are checked against fixed vectors, not only against each other.

  cfg 1  FrozenLake 4x4 one-step Q-learning, one env, the faithful loop
         (src/agent.rs:66-118) with the eval interleave: final Q (f64 bits),
         reward / length histories, training-error checksum
  cfg 2-5  the batched shared-mode schedule (learner groups + merges) at 96
         lanes, groups of 32, K = 16, 6 launches: raw fixed-point Q, UCB
         counters, stats and a SHA-256 of the step records

The reference itself cannot run here (Rust), so these pin the
restatement, not the Rust binary.  Regenerate with
    python tests/golden/make_trajectories.py
"""
import base64
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi as O  # noqa: E402

SHARED = {
    "cfg2": dict(env="frozen_lake", map8x8=1, algo="qlearning"),
    "cfg2_slippery": dict(env="frozen_lake", map8x8=1, slippery=1, algo="qlearning"),
    "cfg3": dict(env="taxi", selector="ucb", algo="expected_sarsa"),
    "cfg4": dict(env="cliff_walking", agent="traces", algo="sarsa"),
    "cfg5": dict(env="blackjack", policy="double", algo="qlearning"),
}
SHARED_SIZE = dict(n_lanes=96, group_size=32, sync_every=16, n_episodes_for_decay=40)
LAUNCHES = 6


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def shared_case(kw):
    p = O.default_params(**SHARED_SIZE, **kw)
    b = O.Batch(p)
    b.set_record(True)
    b.run(LAUNCHES)
    out = {"params": {**SHARED_SIZE, **kw}, "launches": LAUNCHES,
           "q_raw_i64_b64": b64(b.q_raw().astype("<i8")),
           "stats_u64": [int(x) for x in b.stats()[:10]],
           "records_sha256": sha(b.records())}
    if kw.get("selector") == "ucb":
        n, t = b.ucb()
        out["ucb_n_u64_b64"] = b64(np.asarray(n, "<u8"))
        out["ucb_t"] = int(t)
    return out


def faithful_cfg1():
    n, eval_at = 2000, 200
    p = O.default_params(env="frozen_lake", n_episodes_for_decay=n)
    f = O.Faithful(p)
    f.train(n, eval_at)
    rh, el, te = f.histories()
    return {"params": {"env": "frozen_lake", "n_episodes": n, "eval_at": eval_at},
            "q_f64_b64": b64(f.q().astype("<f8")),
            "reward_history_f64_b64": b64(np.asarray(rh, "<f8")),
            "episode_length_u64_b64": b64(np.asarray(el, "<u8")),
            "training_error_sha256": sha(np.asarray(te, "<f8")),
            "n_training_error": int(len(te))}


def generate():
    out = {"source": "tests/golden/make_trajectories.py (oracle/rlref.c, seed 0x5EED)", "cfg1": faithful_cfg1()}
    for k, kw in SHARED.items():
        out[k] = shared_case(kw)
    return out


if __name__ == "__main__":
    path = os.path.join(HERE, "trajectories.json")
    json.dump(generate(), open(path, "w"), indent=1)
    print("wrote", path, os.path.getsize(path), "bytes")
