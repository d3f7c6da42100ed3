"""GPU: the known answers of the multi-GPU bench runs.

tests/golden/global_q.json holds, for the global lane sets bench.py runs at
N = 1, 2, 4, 8 GPUs (cfg 2, 2^20 lanes per GPU; cfg 5 at BASELINE's 2^22), the
oracle's one-process SHA-256 of the merged raw Q words and the training
env-steps after the driver's 25 launches (and cfg 2's default 65).  Integer
merges make an N-rank run end with one process's Q, so these are
the answers bench.py's `q_check` compares an N-rank run against.  Here each
global set runs on ONE GPU through bench.py's own presets (the kernels the bench
launches) and must reproduce them.  Reference loop: src/agent.rs:86-106.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))
GQ = json.load(open(os.path.join(HERE, "golden", "global_q.json")))["cases"]


@pytest.mark.parametrize("name", sorted(GQ))
def test_global_lane_set_matches_oracle(rl, name):
    c = GQ[name]
    k = c["key"]
    p = rl.default_params(env=k["env"], agent=k["agent"], policy=k["policy"], selector=k["selector"],
                          algo=k["algo"], map8x8=k["map8x8"], slippery=k["slippery"], n_lanes=k["global_lanes"],
                          group_size=k["group"], sync_every=k["sync"])
    a = rl.Agent(p)
    a.set_reset_step(bool(k["reset_step"]))
    a.run(k["launches"])
    a.synchronize()
    assert a.q_repr() == c["q_repr"]
    assert hashlib.sha256(a.q_raw().astype("<i8").tobytes()).hexdigest() == c["q_sha256"]
    assert a.stats()["train_steps"] == c["train_steps"]
    a.close()


def test_bench_q_check_matches_fixture(rl):
    """bench.py's own digest and fixture lookup on its driver-shape run (one GPU:
    cfg2_L1M_25, the case every --lanes-total 1048576 run shares)"""
    import subprocess
    root = os.path.dirname(HERE)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "20", "--warmup", "5",
                          "--no-cpu-baseline"], check=True, capture_output=True, text=True, timeout=300).stdout
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    qc = d["q_check"]
    assert qc["fixture"] == "cfg2_L1M_25" and qc["match"] is True and qc["ranks_agree"] is True
    assert qc["q_sha256"] == GQ["cfg2_L1M_25"]["q_sha256"]
