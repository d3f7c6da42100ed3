"""The private-agent bench presets (cfg 6 frozen_lake_neural, cfg 7
cliffwalking_model's Dyna-Q) through the kernels bench.py times — the register-
resident network (`k_train_private_net`) and the LDS-resident Q tables
(`k_train_private_lds`) — on a prefix of the bench's lanes (private lanes are
independent and seeded by global lane id, so lanes [0, 4096) of the 2^20-lane run
are these lanes), two launches of run mode as bench.py makes them, bit-exact
against the oracle's batched schedule (oracle/rlref.c).  Reference loop:
/root/reference/src/agent.rs:86-106; src/bin/frozen_lake_neural.rs:130-134,
src/bin/cliffwalking_model.rs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LANES = 4096


def preset_params(rl, cfg):
    import bench
    pr = dict(bench.PRESETS[cfg])
    extra = dict(pr.get("extra", {}))
    planning = extra.pop("planning", 0)
    kw = dict(env=pr["env"], agent=pr["agent"], policy=pr["policy"], selector=pr["selector"], algo=pr["algo"],
              n_lanes=LANES, group_size=pr["group"], sync_every=64)
    kw.update(extra)
    return rl.default_params(**kw), planning


@pytest.mark.parametrize("cfg", [6, 7])
def test_private_bench_preset_prefix_matches_oracle(rl, oracle, cfg):
    p, planning = preset_params(rl, cfg)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    if planning:
        dev.set_planning(planning)
        ref.set_planning(planning)
    dev.run(2)
    ref.run(2)
    if cfg == 6:
        dw, rw = dev.weights(), ref.weights()
        assert ((dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))).all()
    dq, rq = dev.q(), ref.q()
    assert ((dq.view(np.uint64) == rq.view(np.uint64)) | (np.isnan(dq) & np.isnan(rq))).all()
    assert np.array_equal(dev.epsilon().view(np.uint64), ref.lane_eps().view(np.uint64))
    d, r = dev.stats(), ref.stats().view(np.int64)
    assert d["train_steps"] == int(r[0]) and d["train_steps"] > 0
    assert d["train_episodes"] == int(r[2])
    assert d["reward_sum_q16"] == int(r[4])


@pytest.mark.parametrize("cfg", [6, 7])
def test_private_bench_full_set_last_lanes_match_oracle(rl, oracle, cfg):
    """the WHOLE 2^20-lane bench set of cfg 6 / 7 (cfg 7's
    per-lane tables pass 2^32 bytes: a 32-bit offset would first break there) over
    the driver's window (25 launches), and its LAST 4096 lanes — read alone, by
    rl_agent_get_q_lanes / _weights_lanes — bit-exact against the oracle run on
    exactly those lanes (lane_offset 2^20 - 4096: private lanes are independent and
    keyed by their global id), and against the committed digest bench.py's q_check
    uses (tests/golden/private_q.json)"""
    import json
    import os
    G = 1 << 20
    p, planning = preset_params(rl, cfg)
    full = dict(p, n_lanes=G)
    dev = rl.Agent(full)
    if planning:
        dev.set_planning(planning)
    dev.run(25)
    dev.synchronize()
    dq = dev.q_lanes(G - LANES, LANES)
    dw = dev.weights_lanes(G - LANES, LANES) if cfg == 6 else None
    st = dev.stats()["train_steps"]
    dev.close()
    ref = oracle.Batch(dict(p, lane_offset=G - LANES))
    if planning:
        ref.set_planning(planning)
    ref.run(25)
    rq = ref.q()
    assert ((dq.view(np.uint64) == rq.view(np.uint64)) | (np.isnan(dq) & np.isnan(rq))).all()
    if cfg == 6:
        rw = ref.weights()
        assert ((dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))).all()
    assert 0 < int(ref.stats()[0]) < st
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "private_q.json")))["cases"][f"cfg{cfg}_L1M_last4096_25"]
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_private_q import f64_sha
    assert f64_sha(dq) == gold["q_sha256"]
    if cfg == 6:
        assert f64_sha(dw) == gold["w_sha256"]
