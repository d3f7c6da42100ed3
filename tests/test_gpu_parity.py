"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact bar: integer streams (s, a, r, term, s', a'), the TD error stream and
Q (raw fixed point in shared mode, f64 bits in private mode) must be EQUAL to
the oracle's on the same seeded inputs.  Tolerance for Q: exact (the looser
north-star bound |dQ| < 1e-5 is asserted too, as a floor).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INT_FIELDS = ["s", "s2", "a", "a2", "term", "mode"]


def _params(rl, **kw):
    return rl.default_params(**kw)


def _first_diff(dev, ref, field):
    if field in ("r", "td"):
        a, b = dev[field], ref[field]
        diff = (a.view(np.uint64) != b.view(np.uint64)) & ~(np.isnan(a) & np.isnan(b))
    else:
        diff = dev[field] != ref[field]
    idx = np.argwhere(diff)
    if idx.size == 0:
        return None
    k, lane = idx[0]
    return f"{field} differs at step {k} lane {lane}: dev {dev[k, lane]} ref {ref[k, lane]}"


def _assert_records_equal(dev, ref):
    """Integer streams and the f64 reward / TD streams bit-exact (NaN == NaN)."""
    assert dev.shape == ref.shape, (dev.shape, ref.shape)
    for f in INT_FIELDS + ["r", "td"]:
        msg = _first_diff(dev, ref, f)
        assert msg is None, msg


def _assert_q_equal(dq, rq):
    """NaN masks equal, finite entries within 1e-5 (the north-star bound, as a
    floor), and every non-NaN entry (+-inf included) bit-identical."""
    assert dq.shape == rq.shape
    nan_d, nan_r = np.isnan(dq), np.isnan(rq)
    assert np.array_equal(nan_d, nan_r), "NaN masks differ"
    fin = np.isfinite(dq) & np.isfinite(rq)
    assert np.max(np.abs(dq[fin] - rq[fin]), initial=0.0) < 1e-5
    assert np.array_equal(dq[~nan_d].view(np.uint64), rq[~nan_d].view(np.uint64))


def test_kat_rng(rl, oracle):
    for lane in (0, 1, 12345, 2**40 + 7):
        d = rl.kat_rng(0x5EED, lane, 4096)
        r = oracle.rng_stream(0x5EED, lane, 4096)
        assert np.array_equal(d, r)


def test_kat_log_bit_exact(rl, oracle):
    rng = np.random.default_rng(1)
    x = np.concatenate([np.arange(1, 200001, dtype=np.float64),
                        rng.uniform(1e-300, 1e300, 100000),
                        np.array([2.0**k for k in range(-1074, 1024, 7)]),
                        np.array([0.0, -1.0, np.inf, np.nan, 5e-324])])
    d = rl.kat_log(x)
    r = np.array([oracle.lib().rlo_log(float(v)) for v in x])
    same = (d.view(np.uint64) == r.view(np.uint64)) | (np.isnan(d) & np.isnan(r))
    assert same.all(), x[~same][:10]


def test_kat_ucb_bit_exact(rl, oracle):
    rng = np.random.default_rng(2)
    n = 50000
    q = rng.normal(0, 5, n)
    nc = rng.integers(0, 1000, n).astype(np.float64)
    t = rng.integers(1, 10**9, n).astype(np.uint64)
    t[:100] = np.arange(1, 101)
    d = rl.kat_ucb(q, nc, t, 0.5)
    L = oracle.lib()
    r = np.array([qq + 0.5 * np.sqrt(L.rlo_log(float(tt)) / (cc + 2.2250738585072014e-308))
                  for qq, cc, tt in zip(q, nc, t)])
    same = (d.view(np.uint64) == r.view(np.uint64)) | (np.isnan(d) & np.isnan(r))
    assert same.all()


@pytest.mark.parametrize("env,map8,slip", [("frozen_lake", 0, 0), ("frozen_lake", 1, 1),
                                            ("cliff_walking", 0, 0), ("taxi", 0, 0),
                                            ("blackjack", 0, 0), ("frozen_lake_edited", 0, 0),
                                            ("frozen_lake_edited", 1, 1)])
def test_env_trait_streams(rl, oracle, env, map8, slip):
    """Batched Env::reset/step on the GPU == the oracle's env walked with the
    same per-lane stream and actions (obs as the reference's usize ids)."""
    p = _params(rl, env=env, map8x8=map8, slippery=slip, max_steps=12, seed=77)
    n, T = 64, 16
    e = rl.Env(p, n_envs=n, seed=77)
    rng = np.random.default_rng(3)
    acts = rng.integers(0, e.A, (T, n)).astype(np.uint32)
    obs0 = e.reset()
    dev_s, dev_r, dev_t = [], [], []
    alive = np.ones(n, bool)
    for k in range(T):
        if not alive.all():
            break
        s2, r, t = e.step(acts[k])
        dev_s.append(s2); dev_r.append(r); dev_t.append(t)
        alive &= ~t
    steps = len(dev_s)
    if steps < T:
        with pytest.raises(rl.RLError) as ex:      # some lane terminated: batched EnvNotReady
            e.step(acts[steps])
        assert ex.value.code == 1
    for lane in range(n):
        s0, s2, r, t, k = oracle.env_walk(p, acts[:steps, lane], lane=lane)
        ref0 = s0 if env != "blackjack" else oracle.lib().rlo_blackjack_obs_id(
            s0 >> 6, (s0 >> 1) & 31, s0 & 1)
        assert obs0[lane] == ref0
        m = min(k, steps)
        for j in range(m):
            ref = s2[j] if env != "blackjack" else oracle.lib().rlo_blackjack_obs_id(
                s2[j] >> 6, (s2[j] >> 1) & 31, s2[j] & 1)
            assert dev_s[j][lane] == ref and dev_r[j][lane] == r[j] and dev_t[j][lane] == t[j]


def test_env_trait_known_paths(rl):
    """Hand-derived KATs (tests/golden/tables.json) on the GPU env kernels."""
    import json, os
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tables.json")))["kat"]
    e = rl.Env(_params(rl, env="frozen_lake"), n_envs=1)
    assert e.reset()[0] == 0
    for a, s in zip(kat["fl4x4_path"]["actions"], kat["fl4x4_path"]["states"]):
        s2, r, t = e.step([a])
        assert s2[0] == s
    assert r[0] == 1.0 and t[0]
    e = rl.Env(_params(rl, env="cliff_walking"), n_envs=1)
    assert e.reset()[0] == 36
    tot = 0.0
    for a in kat["cliff_path"]["actions"]:
        s2, r, t = e.step([a])
        tot += r[0]
    assert tot == -13.0 and s2[0] == 47 and t[0]


PRIVATE_CASES = [
    dict(env="frozen_lake", map8x8=0, algo="qlearning"),
    dict(env="frozen_lake", map8x8=1, slippery=1, algo="sarsa"),
    dict(env="cliff_walking", agent="traces", algo="sarsa"),
    dict(env="taxi", selector="ucb", algo="expected_sarsa"),
    dict(env="taxi", policy="double", algo="qlearning"),
    dict(env="blackjack", policy="double", algo="qlearning"),
    dict(env="blackjack", agent="traces", selector="ucb", algo="sarsa"),
    dict(env="cliff_walking", policy="double", selector="ucb", algo="expected_sarsa", agent="traces"),
    dict(env="frozen_lake_edited", map8x8=1, slippery=1, algo="qlearning"),
]


@pytest.mark.parametrize("case", PRIVATE_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_private_mode_matches_reference_loop(rl, oracle, case):
    """group_size 1: every lane is a reference agent; bit-exact vs the oracle,
    including the eval interleave (src/agent.rs:107-113)."""
    n_ep = 60 if case["env"] != "blackjack" else 300
    p = _params(rl, n_lanes=37, group_size=1, sync_every=50, n_episodes_for_decay=n_ep, **case)
    dev = rl.Agent(p)
    dev.set_recording(True)
    dev.train(n_ep, n_ep // 6)
    ref = oracle.Batch(p)
    ref.set_record(True)
    ref.train_episodes(n_ep, n_ep // 6)
    _assert_records_equal(dev.records(), ref.records())
    _assert_q_equal(dev.q(), ref.q())
    assert np.array_equal(dev.epsilon().view(np.uint64), ref.lane_eps().view(np.uint64))
    # and lane 5 alone is the faithful single-env reference loop
    f = oracle.Faithful(dict(p, lane_offset=5))
    f.train(n_ep, n_ep // 6)
    _assert_q_equal(dev.q()[5], f.q())
    _assert_stats_equal(dev, ref)


STAT_KEYS = {0: "train_steps", 1: "eval_steps", 2: "train_episodes", 3: "eval_episodes",
             4: "reward_sum_q16", 7: "trace_states", 8: "q_clamp_hits", 9: "delta_saturations"}


def _assert_stats_equal(dev, ref):
    d, r = dev.stats(), ref.stats().view(np.int64)
    for i, k in STAT_KEYS.items():
        assert d[k] == int(r[i]), (k, d[k], int(r[i]))


SHARED_CASES = [
    dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256),
    dict(env="frozen_lake", map8x8=1, slippery=1, algo="expected_sarsa", group_size=64),
    dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),
    dict(env="taxi", selector="ucb", algo="expected_sarsa", group_size=128),
    dict(env="taxi", selector="ucb", algo="qlearning", group_size=100),
    dict(env="blackjack", policy="double", algo="qlearning", group_size=256),
    dict(env="cliff_walking", policy="double", selector="ucb", algo="sarsa", group_size=64),
    dict(env="frozen_lake", agent="traces", policy="double", algo="qlearning", group_size=2),
    dict(env="frozen_lake_edited", map8x8=1, algo="expected_sarsa", group_size=128),
    # compact Blackjack LDS rows (eps-greedy): terminal rows read from Q_base —
    # q_default != 0 makes them matter for the TD target and the argmax
    dict(env="blackjack", algo="sarsa", group_size=300, q_default=0.25),
    dict(env="blackjack", agent="traces", policy="double", algo="expected_sarsa", group_size=128,
         q_default=-0.5),
    dict(env="blackjack", selector="ucb", algo="qlearning", group_size=64),      # dense rows (UCB)
    # traces: one count per visited row; row list (rows > block) with UCB specials,
    # and UCB without expected SARSA (no barrier after the counter increments)
    dict(env="taxi", agent="traces", selector="ucb", algo="expected_sarsa", group_size=256),
    dict(env="cliff_walking", agent="traces", selector="ucb", algo="sarsa", group_size=64),
    # owner-form settle with > 64 contributions per entry: 1.0/n by division
    dict(env="frozen_lake", map8x8=1, algo="sarsa", group_size=200),
]


@pytest.mark.parametrize("case", SHARED_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_shared_mode_matches_batched_oracle(rl, oracle, case):
    """Learner groups in LDS + merge every K steps: bit-exact vs the oracle's
    batched schedule (raw fixed-point Q, UCB counters, streams)."""
    L = 600
    p = _params(rl, n_lanes=L, sync_every=16, n_episodes_for_decay=40, **case)
    dev = rl.Agent(p)
    dev.set_recording(True)
    ref = oracle.Batch(p)
    ref.set_record(True)
    dev.run(6)
    ref.run(6)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_q_equal(dev.q(), ref.q())
    if case.get("selector") == "ucb":
        dn, dt = dev.ucb()
        rn, rt = ref.ucb()
        assert np.array_equal(dn, rn) and dt == rt
    # episodes mode with eval interleave
    dev.train(12, 4)
    ref.train_episodes(12, 4)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def test_full_size_fl8x8_properties(rl):
    """BASELINE config 2 at full size (2^20 lanes): size-independent properties —
    finite Q in range, every lane stepped exactly K times per launch, merge
    reproducible (two identical runs give bit-identical Q)."""
    p = _params(rl, env="frozen_lake", map8x8=1, n_lanes=1 << 20, group_size=256, sync_every=64)
    qs = []
    for _ in range(2):
        a = rl.Agent(p)
        a.run(3)
        a.synchronize()
        st = a.stats()
        # every lane makes 64 synchronous steps per launch; RESET steps are not env steps
        assert 0.8 * 3 * 64 * (1 << 20) < st["train_steps"] < 3 * 64 * (1 << 20)
        q = a.q_raw()
        qs.append(q)
        qq = a.q()
        assert np.isfinite(qq).all() and qq.max() <= 1.0 + 1e-9 and qq.min() >= -1e-9
        a.close()
    assert np.array_equal(qs[0], qs[1])


def _episodes_from_records(recs, n_lanes):
    """reward_history / episode_length per lane from step records
    (src/agent.rs:83-100: epi_reward += r per step, pushed at termination)."""
    out = [[] for _ in range(n_lanes)]
    for lane in range(n_lanes):
        rew, n = 0.0, 0
        for rec in recs[:, lane]:
            if rec["kind"] == 1:
                rew, n = 0.0, 0
            elif rec["kind"] == 2:
                rew += float(rec["r"])
                n += 1
                if rec["term"]:
                    out[lane].append((int(rec["mode"]), n, rew))
    return out


@pytest.mark.parametrize("case", [dict(env="frozen_lake", group_size=1, algo="qlearning"),
                                  dict(env="taxi", group_size=64, selector="ucb", algo="sarsa"),
                                  dict(env="blackjack", group_size=32, policy="double", algo="expected_sarsa")],
                         ids=["fl-private", "taxi-shared-ucb", "bj-shared-double"])
def test_episode_log_matches_oracle(rl, oracle, case):
    """Device episode log (reward_history / episode_length of train and the
    interleaved evaluate) == the episodes in the oracle's step records."""
    L = 70
    p = _params(rl, n_lanes=L, sync_every=20, n_episodes_for_decay=40, eval_episodes=5, **case)
    dev = rl.Agent(p)
    dev.set_episode_log(64)
    ref = oracle.Batch(p)
    ref.set_record(True)
    dev.train(30, 10)
    ref.train_episodes(30, 10)
    eps, lost = dev.episodes()
    assert lost == 0
    want = _episodes_from_records(ref.records(), L)
    got = [[] for _ in range(L)]
    for e in eps:
        got[int(e["lane"])].append((int(e["mode"]), int(e["length"]), float(e["reward"])))
    for lane in range(L):
        assert len(got[lane]) == len(want[lane]), lane
        for g, w in zip(got[lane], want[lane]):
            assert g[0] == w[0] and g[1] == w[1] and np.float64(g[2]).tobytes() == np.float64(w[2]).tobytes()
    # every lane ran exactly 30 training episodes and 5 eval episodes at each of the
    # interleave points 0, 10, 20 (episode % eval_at == 0, src/agent.rs:107)
    assert {sum(1 for g in got[l] if g[0] == 0) for l in range(L)} == {30}
    assert {sum(1 for g in got[l] if g[0] == 1) for l in range(L)} == {15}


@pytest.mark.parametrize("case", [dict(env="cliff_walking", algo="qlearning"),
                                  dict(env="taxi", selector="ucb", algo="expected_sarsa"),
                                  dict(env="frozen_lake", map8x8=1, slippery=1, agent="traces",
                                       policy="double", algo="sarsa"),
                                  dict(env="blackjack", policy="double", algo="qlearning"),
                                  # one-step, one table: the pipelined planning batch (reads
                                  # ahead of the previous write, forwarded) for each TD target
                                  dict(env="cliff_walking", algo="sarsa"),
                                  dict(env="frozen_lake", map8x8=1, slippery=1, algo="expected_sarsa")],
                         ids=["cw-q", "taxi-ucb-es", "fl-traces-double", "bj-double", "cw-sarsa", "fl-es"])
def test_dyna_matches_oracle(rl, oracle, case):
    """InternalModelAgent + RandomModel, 10 planning steps (private agents):
    records, Q, ε and stats bit-exact vs the oracle (itself == the faithful loop)."""
    n = 40 if case["env"] != "blackjack" else 200
    p = _params(rl, n_lanes=33, group_size=1, sync_every=29, n_episodes_for_decay=n, **case)
    dev = rl.Agent(p)
    dev.set_planning(10)
    dev.set_recording(True)
    ref = oracle.Batch(p)
    ref.set_planning(10)
    ref.set_record(True)
    dev.train(n, n // 4)
    ref.train_episodes(n, n // 4)
    _assert_records_equal(dev.records(), ref.records())
    _assert_q_equal(dev.q(), ref.q())
    assert np.array_equal(dev.epsilon().view(np.uint64), ref.lane_eps().view(np.uint64))
    _assert_stats_equal(dev, ref)
    # Agent::reset empties the model too; a second run stays in lockstep
    dev.reset()
    ref.reset()
    dev.train(n // 2, n // 4)
    ref.train_episodes(n // 2, n // 4)
    _assert_q_equal(dev.q(), ref.q())


@pytest.mark.parametrize("lpw", ["64", "32", "16"])
@pytest.mark.parametrize("case", [dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=200),
                                  dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256)],
                         ids=["cw-traces", "fl-q"])
def test_lanes_per_wave_mapping(rl, oracle, case, lpw, monkeypatch):
    """Learner groups spread over more waves (16 / 32 lanes per wave, the
    layout small grids get) give the same results as 64 lanes per wave."""
    monkeypatch.setenv("RLAMD_LPW", lpw)
    p = _params(rl, n_lanes=1000, sync_every=16, n_episodes_for_decay=40, **case)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    dev.run(4)
    ref.run(4)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def _golden():
    import json, os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "trajectories.json")))


@pytest.mark.parametrize("cfg", ["cfg2", "cfg2_slippery", "cfg3", "cfg4", "cfg5"])
def test_device_matches_golden_trajectories(rl, cfg):
    """The device against the committed fixtures directly (no oracle in the
    loop): raw Q, UCB counters and stats after the fixture's launches."""
    import base64
    g = _golden()[cfg]
    dev = rl.Agent(_params(rl, **g["params"]))
    dev.run(g["launches"])
    want = np.frombuffer(base64.b64decode(g["q_raw_i64_b64"]), "<i8")
    assert np.array_equal(dev.q_raw().reshape(-1), want)
    st, ref = dev.stats(), np.array(g["stats_u64"], np.uint64).view(np.int64)
    for i, k in STAT_KEYS.items():
        assert st[k] == int(ref[i]), k
    if "ucb_t" in g:
        n, t = dev.ucb()
        assert t == g["ucb_t"]
        assert np.array_equal(np.asarray(n).reshape(-1), np.frombuffer(base64.b64decode(g["ucb_n_u64_b64"]), "<u8"))


def test_device_matches_golden_cfg1_faithful_loop(rl):
    """cfg 1 (FrozenLake 4x4, one env, eval interleave on) as one private
    device agent: the fixture's Q and per-episode histories."""
    import base64
    g = _golden()["cfg1"]
    n, eval_at = g["params"]["n_episodes"], g["params"]["eval_at"]
    dev = rl.Agent(_params(rl, env="frozen_lake", n_lanes=1, group_size=1, sync_every=64,
                           n_episodes_for_decay=n))
    dev.train(n, eval_at)
    q = dev.q()[0].reshape(-1)
    assert np.array_equal(q.view(np.uint64), np.frombuffer(base64.b64decode(g["q_f64_b64"]), "<u8"))


@pytest.mark.parametrize("L,G,kw", [(1, 64, dict(env="frozen_lake", map8x8=1, algo="qlearning")),
                                    (65, 64, dict(env="taxi", selector="ucb", algo="expected_sarsa")),
                                    (3, 256, dict(env="cliff_walking", agent="traces", algo="sarsa")),
                                    (130, 129, dict(env="blackjack", policy="double", algo="sarsa"))],
                         ids=["fl-L1", "taxi-L65-G64", "cw-traces-L3", "bj-L130-G129"])
def test_tiny_and_ragged_groups(rl, oracle, L, G, kw):
    """Edge sizes: one lane, a group larger than the lane count, a last group
    with a single lane, a group size that is not a multiple of 64."""
    p = _params(rl, n_lanes=L, group_size=G, sync_every=16, n_episodes_for_decay=40, **kw)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    dev.run(6)
    ref.run(6)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def test_full_size_determinism_and_range(rl):
    """cfg 2 at full size (2^20 lanes, G 512, K 64): two runs are bit-identical
    (integer LDS / HBM atomics make the merge order-free) and FrozenLake Q stays
    in [0, 1]; every lane steps or resets once per synchronous step."""
    p = _params(rl, env="frozen_lake", map8x8=1, algo="qlearning", n_lanes=1 << 20, group_size=512,
                sync_every=64)
    qs = []
    for _ in range(2):
        dev = rl.Agent(p)
        dev.run(3)
        qs.append(dev.q_raw())
        st = dev.stats()
        assert 0 < st["train_steps"] < 3 * 64 * (1 << 20)
    assert np.array_equal(qs[0], qs[1])
    q = qs[0].astype(np.float64) * 2.0**-40
    assert q.min() >= 0.0 and q.max() <= 1.0 and q.max() > 0.0


@pytest.mark.parametrize("trc_kb", ["0", "2", "150"])
def test_pair_trace_lds_slots(rl, oracle, trc_kb, monkeypatch):
    """Pair traces with no LDS slots (all in HBM), a few (long episodes spill
    past them) and every slot in LDS: bit-exact in all three."""
    monkeypatch.setenv("RLAMD_TRC_KB", trc_kb)
    p = _params(rl, env="cliff_walking", agent="traces", algo="qlearning", n_lanes=700, group_size=64,
                sync_every=16, n_episodes_for_decay=40)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    dev.run(5)
    ref.run(5)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


def test_trace_items_count_live_pairs(rl):
    """rl_agent_trace_items (ABI 7): the live trace entries bench.py's algorithmic
    bytes count — 0 before any step, bounded by every lane's S*A pairs, non-zero
    while episodes are open, and 0 again after train() (every episode ends and
    the sets are cleared: elegibility_traces_agent.rs:98-100)"""
    for kw in (dict(env="cliff_walking", group_size=256), dict(env="taxi", group_size=64)):
        p = rl.default_params(agent="traces", algo="sarsa", n_lanes=4096, sync_every=16, **kw)
        a = rl.Agent(p)
        assert a.trace_items() == 0
        a.run(3)
        n = a.trace_items()
        assert 0 < n <= 4096 * a.S * a.A, n
        a.train(1, 0)
        assert a.trace_items() == 0
        a.close()
    one = rl.Agent(rl.default_params(n_lanes=64, group_size=64))
    one.run(1)
    assert one.trace_items() == 0


@pytest.mark.parametrize("env", ["taxi", "blackjack"])
def test_pair_trace_cap_change_mid_episode(rl, oracle, env, monkeypatch):
    """a lane's pair list outlives the launch (p.tcnt) while its LDS
    slot count follows the carve, which a reconfiguration (selector / representation
    switch, the other kernel family) can change mid-episode.  Lists then continue
    under a grown cap (0 -> 8 KiB: HBM-indexed pairs now in LDS, stale visited-state
    bits) and a shrunk one (8 -> 1 KiB: pairs now in HBM without slot_of): the HBM
    index is rebuilt (k_pair_reindex) and Q stays bit-exact.  The reconfiguration is
    set_action_selector to the same eps-greedy selector (the reference replaces the
    selector: epsilon restarts) with RLAMD_TRC_KB changed in between."""
    p = _params(rl, env=env, agent="traces", algo="qlearning", n_lanes=700, group_size=64, sync_every=16,
                n_episodes_for_decay=40)
    monkeypatch.setenv("RLAMD_TRC_KB", "0")
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    for kb in ["8", "1"]:
        dev.run(3)
        ref.run(3)
        monkeypatch.setenv("RLAMD_TRC_KB", kb)
        dev.set_action_selector("eps_greedy")
        ref.set_selector("eps_greedy")
    dev.run(3)
    ref.run(3)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


@pytest.mark.parametrize("terminal", ["uniform", "mixed"])
def test_blackjack_terminal_rows_after_set_q(rl, oracle, terminal):
    """Compact Blackjack rows read terminal rows from Q_base, or from one
    per-table constant when set_q / reset left them uniform: both bit-exact."""
    p = _params(rl, env="blackjack", policy="double", algo="expected_sarsa", n_lanes=1200, group_size=512,
                sync_every=16, n_episodes_for_decay=40)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    P, S, A = ref.P, ref.S, ref.A
    rng = np.random.default_rng(11)
    q = rng.uniform(-1.0, 1.0, (P, S, A))
    s = np.arange(S)
    term = ~((s >> 6 <= 21) & ((s >> 1) & 31 <= 10))
    if terminal == "uniform":
        q[0][term] = 0.375
        q[1][term] = -0.125
    dev.set_q(q.reshape(-1))
    ref.set_q(q.reshape(-1))
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    dev.run(4)
    ref.run(4)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)


@pytest.mark.parametrize("case", [dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256),
                                  dict(env="cliff_walking", algo="sarsa", group_size=64),
                                  dict(env="taxi", selector="ucb", algo="expected_sarsa", group_size=128),
                                  dict(env="blackjack", policy="double", algo="qlearning", group_size=256),
                                  dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),
                                  dict(env="blackjack", algo="expected_sarsa", group_size=512, q_default=0.25)],
                         ids=["fl-q-o8", "cw-sarsa-o8", "taxi-ucb-es", "bj-double-o8", "cw-traces", "bj-es-o8"])
def test_throughput_variant_matches_oracle(rl, oracle, case):
    """The kernels the bench runs (no records, no episode log: the INSTR=false
    and occupancy-8 instantiations): raw Q, UCB counters and stats bit-exact."""
    p = _params(rl, n_lanes=1500, sync_every=16, n_episodes_for_decay=40, **case)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    dev.run(5)
    ref.run(5)
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    if case.get("selector") == "ucb":
        dn, dt = dev.ucb()
        rn, rt = ref.ucb()
        assert np.array_equal(dn, rn) and dt == rt
    _assert_stats_equal(dev, ref)


# ---------------------------------------------------------------- NeuralPolicy
ACTS = ["linear", "tanh", "relu", "leaky_relu", "relu6", "leaky_relu6", "sigmoid", "swish", "hard_swish"]


def test_kat_activations_bit_exact(rl, oracle):
    """device f, f' (src/network/activation.rs, fdlibm exp/tanh) == the oracle's"""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.normal(0, 4, 20000), rng.uniform(-800, 800, 2000), np.linspace(-7, 7, 1401),
                        [0.0, -0.0, 6.0, -3.0, np.inf, -np.inf, np.nan, 1e-310]])
    for a in ACTS:
        df, dfp = rl.kat_act(a, x)
        rf, rfp = oracle.act(a, x)
        for d, r in ((df, rf), (dfp, rfp)):
            same = (d.view(np.uint64) == r.view(np.uint64)) | (np.isnan(d) & np.isnan(r))
            assert same.all(), (a, x[~same][:5], d[~same][:5], r[~same][:5])


NEURAL_CASES = [
    # the neural bin (src/bin/frozen_lake_neural.rs): FL 4x4, 1-32-4 leaky_relu6/linear,
    # Q-learning, eps-greedy with the `a * 0.5` decay
    dict(env="frozen_lake", algo="qlearning", decay_kind=1, eps_decay=0.5),
    dict(env="frozen_lake_edited", map8x8=1, slippery=1, net_input="fl_obs", algo="sarsa", net_act1="tanh"),
    dict(env="cliff_walking", agent="traces", algo="qlearning", net_act1="relu", net_hidden=16),
    dict(env="taxi", selector="ucb", algo="expected_sarsa", net_act1="sigmoid", net_hidden=8),
    dict(env="blackjack", algo="expected_sarsa", net_act1="swish", net_act2="softmax", net_hidden=12),
    dict(env="frozen_lake", map8x8=1, algo="qlearning", net_act1="hard_swish", net_act2="leaky_relu"),
]


@pytest.mark.parametrize("case", NEURAL_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_neural_policy_matches_oracle(rl, oracle, case):
    """NeuralPolicy agents (private): step streams, TD errors, every lane's
    parameters and get_values of every state bit-exact vs the oracle; lane 3
    is the faithful single-agent loop; Agent::reset re-draws the network."""
    n_ep = 30 if case["env"] != "blackjack" else 120
    kw = dict(net_hidden=32, max_steps=40)
    kw.update(case)
    p = _params(rl, policy="neural", n_lanes=45, group_size=1, sync_every=40, n_episodes_for_decay=n_ep, **kw)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    assert np.array_equal(dev.weights().view(np.uint64), ref.weights().view(np.uint64)), "init"
    dev.set_recording(True)
    ref.set_record(True)
    dev.train(n_ep, n_ep // 3)
    ref.train_episodes(n_ep, n_ep // 3)
    _assert_records_equal(dev.records(), ref.records())
    dw, rw = dev.weights(), ref.weights()
    same = (dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))
    assert same.all()
    _assert_q_equal(dev.q(), ref.q())
    assert np.array_equal(dev.epsilon().view(np.uint64), ref.lane_eps().view(np.uint64))
    _assert_stats_equal(dev, ref)
    f = oracle.Faithful(dict(p, lane_offset=3))
    f.train(n_ep, n_ep // 3)
    fw = f.weights()
    assert ((fw.view(np.uint64) == dw[3].view(np.uint64)) | (np.isnan(fw) & np.isnan(dw[3]))).all()
    dev.reset()
    ref.reset()
    assert np.array_equal(dev.weights().view(np.uint64), ref.weights().view(np.uint64)), "reset"
    dev.train(n_ep // 3, 0)
    ref.train_episodes(n_ep // 3, 0)
    dw, rw = dev.weights(), ref.weights()
    assert ((dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))).all()


NET_BIN_CASES = [
    # the bin's network (1-32-4 leaky_relu6 / linear) on one-step agents: the
    # register-resident kernel (k_train_private_net); 300 lanes = a partial block
    dict(env="frozen_lake", algo="qlearning"),
    dict(env="frozen_lake", algo="sarsa", selector="ucb"),
    dict(env="frozen_lake", map8x8=1, slippery=1, algo="expected_sarsa"),
    dict(env="frozen_lake", algo="qlearning", planning=2),
]


@pytest.mark.parametrize("case", NET_BIN_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_neural_bin_shape_register_kernel(rl, oracle, case):
    """The bin's network with its parameters held in registers for a launch:
    episodic train and throughput run, every lane's parameters, Q values, eps and
    stats bit-exact vs the oracle (NaN-aware: payloads differ between gfx950 and x86)."""
    kw = dict(case)
    plan = kw.pop("planning", 0)
    p = _params(rl, policy="neural", n_lanes=300, group_size=1, sync_every=24, n_episodes_for_decay=40,
                net_hidden=32, net_act1="leaky_relu6", net_act2="linear", max_steps=30, **kw)
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    if plan:
        dev.set_planning(plan)
        ref.set_planning(plan)
    dev.train(12, 5)
    ref.train_episodes(12, 5)
    dev.run(3)
    ref.run(3)
    dw, rw = dev.weights(), ref.weights()
    assert ((dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))).all()
    _assert_q_equal(dev.q(), ref.q())
    assert np.array_equal(dev.epsilon().view(np.uint64), ref.lane_eps().view(np.uint64))
    _assert_stats_equal(dev, ref)


def test_neural_weights_roundtrip_and_dyna(rl, oracle):
    """set_weights (Layer::set_weights) then training stays in lockstep; Dyna
    planning over a neural policy (InternalModelAgent) matches too."""
    p = _params(rl, policy="neural", env="cliff_walking", n_lanes=20, group_size=1, sync_every=30,
                n_episodes_for_decay=20, net_hidden=16, max_steps=50, lr=0.001)   # finite weights
    dev = rl.Agent(p)
    ref = oracle.Batch(p)
    w = np.random.default_rng(9).normal(0, 0.05, dev.weights().shape)
    dev.set_weights(w)
    ref.set_weights(w)
    assert np.array_equal(dev.weights(), w)
    dev.set_planning(3)
    ref.set_planning(3)
    dev.train(15, 5)
    ref.train_episodes(15, 5)
    dw, rw = dev.weights(), ref.weights()   # NaN payloads differ between gfx950 and x86: NaN-aware
    assert ((dw.view(np.uint64) == rw.view(np.uint64)) | (np.isnan(dw) & np.isnan(rw))).all()
    _assert_stats_equal(dev, ref)


RESET_STEP_CASES = [
    dict(env="blackjack", policy="double", algo="qlearning", group_size=128),   # cfg 5's kernel (o8)
    dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=64),    # cfg 4's kernel
    dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256),       # o8, sweep form
    dict(env="taxi", algo="expected_sarsa", group_size=100),
    dict(env="frozen_lake", map8x8=1, slippery=1, agent="traces", policy="double", algo="expected_sarsa",
         group_size=64),
]


@pytest.mark.parametrize("case", RESET_STEP_CASES, ids=lambda c: "-".join(f"{v}" for v in c.values()))
def test_reset_step_schedule_matches_oracle(rl, oracle, case):
    """rl_agent_set_reset_step: a resetting lane resets, selects and steps in one
    synchronous step (kind 3 records) — device == oracle bit for bit, in run mode
    and with the eval interleave."""
    L = 500
    p = _params(rl, n_lanes=L, sync_every=16, n_episodes_for_decay=40, **case)
    dev = rl.Agent(p)
    dev.set_reset_step(True)
    dev.set_recording(True)
    ref = oracle.Batch(p)
    ref.set_reset_step(True)
    ref.set_record(True)
    dev.run(5)
    ref.run(5)
    recs = dev.records()
    _assert_records_equal(recs, ref.records())
    assert (recs["kind"] == 3).any() and not (recs["kind"] == 1).any()
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)
    dev.train(10, 4)
    ref.train_episodes(10, 4)
    _assert_records_equal(dev.records(), ref.records())
    assert np.array_equal(dev.q_raw(), ref.q_raw())
    _assert_stats_equal(dev, ref)
