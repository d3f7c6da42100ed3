"""CPU: semantics of the batched schedule (the GPU's contract), checked on the oracle.

* private mode (group_size 1) == the faithful single-env reference loop, bit for bit
* shared mode: single-group runs are launch-length invariant, Q stays in range,
  the merge is decomposable across ranks (world_size-2 gloo all-reduce == one
  process holding every lane), NaN stickiness for UCB + expected SARSA.
"""
import itertools
import os
import socket

import numpy as np
import pytest

CONFIGS = list(itertools.product(["frozen_lake", "cliff_walking", "taxi", "blackjack"],
                                 ["one_step", "traces"], ["tabular", "double"],
                                 ["eps_greedy", "ucb"], ["sarsa", "qlearning", "expected_sarsa"]))


def _eq_nan(a, b):
    return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
        np.nan_to_num(a).view(np.uint64), np.nan_to_num(b).view(np.uint64))


@pytest.mark.parametrize("env,agent,policy,sel,algo", CONFIGS[::5],
                         ids=lambda v: str(v))
def test_private_batch_equals_faithful(oracle, env, agent, policy, sel, algo):
    n = 40 if env != "blackjack" else 200
    p = oracle.default_params(env=env, agent=agent, policy=policy, selector=sel, algo=algo,
                              map8x8=1, n_episodes_for_decay=n, n_lanes=3, group_size=1,
                              sync_every=37)
    b = oracle.Batch(p)
    b.set_record(True)
    b.train_episodes(n, n // 4)
    recs = b.records()
    q = b.q()
    for lane in range(3):
        f = oracle.Faithful(dict(p, lane_offset=lane))
        f.set_record(True)
        f.train(n, n // 4)
        fr = f.records()
        br = recs[:, lane]
        br = br[(br["mode"] == oracle.MODE_TRAIN) & (br["kind"] == oracle.KIND_STEP)]
        assert len(fr) == len(br)
        for k in ("s", "s2", "a", "a2", "term", "r"):
            assert np.array_equal(fr[k], br[k]), k
        assert _eq_nan(fr["td"], br["td"])
        assert _eq_nan(f.q(), q[lane])


@pytest.mark.parametrize("env,algo", [("frozen_lake", "qlearning"), ("taxi", "sarsa")])
def test_single_group_is_launch_length_invariant(oracle, env, algo):
    """With one learner group every merge is the identity, so K only changes how
    the steps are cut into launches."""
    outs = []
    for K in (10, 50):
        p = oracle.default_params(env=env, algo=algo, map8x8=1, n_lanes=100, group_size=128,
                                  sync_every=K)
        b = oracle.Batch(p)
        b.set_record(True)
        b.run(100 // K)
        outs.append((b.q_raw(), b.records()))
    assert np.array_equal(outs[0][0], outs[1][0])
    for k in ("s", "a", "s2", "td"):
        assert np.array_equal(outs[0][1][k], outs[1][1][k])


def test_shared_mode_stays_in_range(oracle):
    """The mean combination rule keeps Q a convex-ish average of lane targets:
    FrozenLake Q stays in [0, 1] even with 4096 lanes and 16 groups."""
    p = oracle.default_params(env="frozen_lake", map8x8=1, n_lanes=4096, group_size=256, sync_every=32)
    b = oracle.Batch(p)
    b.run(20)
    q = b.q()
    assert q.min() >= 0.0 and q.max() <= 1.0 + 1e-12 and q.max() > 0.0


def test_set_q_representations_and_blackjack_terminal_rows(oracle):
    """rlo_batch_set_q keeps the values as given: the double policy has no range
    proof, so the table is f64 (5000, NaN, inf held exactly, NaN canonical); and
    Blackjack terminal rows (player > 21 or dealer card > 10) are never written
    by training."""
    p = oracle.default_params(env="blackjack", policy="double", algo="qlearning", n_lanes=512, group_size=128,
                              sync_every=16)
    b = oracle.Batch(p)
    assert b.q_repr() == "f64"
    P, S, A = b.P, b.S, b.A
    q = np.random.default_rng(4).uniform(-2.0, 2.0, (P, S, A))
    q[0, 5, 1] = np.nan
    q[1, 7, 0] = np.inf
    q[0, 9, 0] = 5000.0                      # no clamp: f64 keeps it
    b.set_q(q.reshape(-1))
    raw = b.q_raw()
    fin = np.isfinite(q)
    assert np.array_equal(raw[fin].view(np.float64), q[fin])
    assert raw[0, 5, 1] == 0x7FF8000000000000
    qq = b.q()
    assert np.isnan(qq[0, 5, 1]) and qq[1, 7, 0] == np.inf and qq[0, 9, 0] == 5000.0
    s = np.arange(S)
    term = ~((s >> 6 <= 21) & ((s >> 1) & 31 <= 10))
    before = raw[:, term, :].copy()
    b.run(6)
    assert np.array_equal(b.q_raw()[:, term, :], before)
    assert not np.array_equal(b.q_raw()[:, ~term, :], raw[:, ~term, :])


@pytest.mark.parametrize("kw,want", [
    (dict(env="frozen_lake", map8x8=1, algo="qlearning"), "fixed40"),
    (dict(env="taxi", algo="expected_sarsa"), "fixed40"),
    (dict(env="cliff_walking", selector="ucb", algo="sarsa"), "fixed40"),
    (dict(env="blackjack", policy="double", algo="qlearning"), "f64"),
    (dict(env="cliff_walking", agent="traces", algo="sarsa"), "f64"),
    (dict(env="taxi", selector="ucb", algo="expected_sarsa"), "f64"),
    (dict(env="frozen_lake", algo="qlearning", gamma=1.0), "f64"),
    (dict(env="frozen_lake", map8x8=1, slippery=1, algo="qlearning"), "f64"),
    (dict(env="frozen_lake_edited", slippery=1, algo="sarsa"), "f64"),
], ids=["fl-q", "taxi-es", "cw-ucb-sarsa", "bj-double", "cw-traces", "taxi-ucb-es", "gamma1", "fl-slippery",
        "fle-slippery"])
def test_representation_follows_the_range_proof(oracle, kw, want):
    """The fixed point only where the proof holds (one-step, single table,
    contracting bootstrap: rlref.c o_delta_bound) and on deterministic maps (round
    6: slippery FrozenLake leaves 1e-5 of f64, longrun.json repr_drift_curve), f64
    everywhere else; 'fixed_range' (oracle only) is round 5's rule without the map
    condition."""
    b = oracle.Batch(oracle.default_params(n_lanes=64, group_size=32, **kw))
    assert b.q_repr() == want
    if kw.get("slippery"):
        b.set_q_mode("fixed_range")
        assert b.q_repr() == "fixed40"


def test_representation_changes(oracle):
    """set_q with values the fixed point cannot hold exactly -> f64; a selector /
    algorithm change that breaks the proof moves a fixed-point table to f64 exactly
    (the proof follows the table's state); set_q_mode switches both ways."""
    p = oracle.default_params(env="frozen_lake", map8x8=1, algo="qlearning", n_lanes=256, group_size=64, sync_every=8)
    b = oracle.Batch(p)
    assert b.q_repr() == "fixed40"
    b.run(3)
    q0 = b.q()
    b.set_q_mode("f64")
    assert b.q_repr() == "f64" and np.array_equal(b.q(), q0)
    b.set_q_mode("auto")
    assert b.q_repr() == "fixed40" and np.array_equal(b.q(), q0)
    b.set_selector("ucb")
    b.set_algo("expected_sarsa")                  # UCB + expected SARSA: no proof
    assert b.q_repr() == "f64" and np.array_equal(b.q(), q0)
    b.set_q(np.full(b.P * b.S * b.A, 0.1))      # 0.1 is not a multiple of 2^-40
    assert b.q_repr() == "f64"


def test_f64_one_lane_is_the_reference_loop(oracle):
    """With one lane every step has one contribution per entry, added exactly
    (Q += lr * td, tabular_policy.rs:35-38 / double_tabular_policy.rs:50-57), and the
    merge of one group is its value: the shared f64 schedule IS the reference loop,
    bit for bit, including the double policy's growth to +-inf / NaN."""
    for kw in (dict(env="blackjack", policy="double", algo="qlearning"),
               dict(env="taxi", selector="ucb", algo="expected_sarsa"),
               dict(env="cliff_walking", policy="double", selector="ucb", algo="sarsa")):
        n = 2000
        p = oracle.default_params(n_episodes_for_decay=n, n_lanes=1, group_size=2, sync_every=37, **kw)
        b = oracle.Batch(p)
        b.set_q_mode("f64")
        b.train_episodes(n, n // 4)
        f = oracle.Faithful(p)
        f.train(n, n // 4)
        assert _eq_nan(b.q(), f.q()), kw


def test_f64_double_policy_grows_past_the_old_clamp(oracle):
    """cfg 5's update (double_tabular_policy.rs:50-57) is not a contraction: the
    values leave the fixed point's [-2048, 2048] within a few hundred steps of the
    bench geometry, and the f64 table follows them (no clamp, no saturation)."""
    p = oracle.default_params(env="blackjack", policy="double", algo="qlearning", n_lanes=2048, group_size=512,
                              sync_every=64)
    b = oracle.Batch(p)
    b.set_reset_step(True)
    b.run(12)
    q = b.q()
    assert b.q_repr() == "f64" and np.nanmax(np.abs(q)) > 2048.0
    st = b.stats()
    assert st[8] == 0 and st[9] == 0


def test_f64_sequential_variant_drift_is_small(oracle):
    """The exponent-grid sum vs f64 sums in lane / group order (rlref.c
    RLO_QMODE_F64_SEQ): same draws, same mean rule; the two only differ by
    rounding, bounded relative to the values over a short horizon."""
    kw = dict(env="cliff_walking", agent="traces", algo="sarsa", n_lanes=512, group_size=128, sync_every=16)
    a = oracle.Batch(oracle.default_params(**kw))
    s = oracle.Batch(oracle.default_params(**kw))
    s.set_q_mode("f64_seq")
    a.run(4)
    s.run(4)
    qa, qs = a.q(), s.q()
    assert np.isfinite(qa).all() and np.abs(qa - qs).max() < 1e-9 * max(1.0, np.abs(qa).max())


def test_expected_sarsa_ucb_nan_is_sticky(oracle):
    """UCB + expected SARSA produces NaN Q entries; they never heal."""
    p = oracle.default_params(env="taxi", selector="ucb", algo="expected_sarsa", n_lanes=64,
                              group_size=64, sync_every=64)
    b = oracle.Batch(p)
    b.run(4)
    nan1 = np.isnan(b.q())
    assert nan1.any()
    b.run(4)
    assert np.isnan(b.q())[nan1].all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, p, n_launch, out_q):
    import torch
    import torch.distributed as dist

    import oracle_ffi as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = p["n_lanes"] // world
    b = O.Batch(dict(p, n_lanes=L, lane_offset=rank * L))
    b.set_merge_groups(world * ((L + p["group_size"] - 1) // p["group_size"]))
    mw = b.delta_max_words()
    for _ in range(n_launch):
        d = np.zeros(b.delta_words(), np.int64)
        b.launch_groups(d)
        t = torch.from_numpy(d)                # the RCCL all-reduces of bench.py, on gloo
        dist.all_reduce(t[:mw], op=dist.ReduceOp.MAX)
        b.fold(d)
        dist.all_reduce(t[mw:])
        b.apply_delta(t.numpy())
    out_q.put((rank, b.q_raw().tobytes(), b.ucb()[0].tobytes(), b.ucb()[1]))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [dict(env="frozen_lake", map8x8=1, algo="qlearning"),
                                  dict(env="taxi", selector="ucb", algo="sarsa"),
                                  dict(env="blackjack", policy="double", algo="qlearning"),
                                  dict(env="cliff_walking", agent="traces", algo="sarsa"),
                                  dict(env="taxi", selector="ucb", algo="expected_sarsa")],
                         ids=["fl8x8-q", "taxi-ucb-sarsa", "bj-double-f64", "cw-traces-f64", "taxi-ucb-es-f64"])
def test_two_rank_merge_equals_one_process(oracle, case):
    """world_size-2 gloo: each rank holds half the lanes (contiguous global lane
    ids), all-reduces the merge buffer (MAX of the f64 grid codes, fold, SUM of the
    rest), applies it.  Q and UCB counters must be bit-identical to one process
    holding every lane (GPU-count independence of the N>1 bench path), in both
    Q representations."""
    import torch.multiprocessing as mp
    p = oracle.default_params(n_lanes=512, group_size=64, sync_every=16, **case)
    n_launch = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, p, n_launch, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict((r, (qb, nb, t)) for r, qb, nb, t in (q.get(timeout=300) for _ in procs))
    for pr in procs:
        pr.join(timeout=60)
    one = oracle.Batch(p)
    one.run(n_launch)
    ref_q = one.q_raw().tobytes()
    ref_n, ref_t = one.ucb()
    for r in (0, 1):
        assert res[r][0] == ref_q
        assert res[r][1] == ref_n.tobytes() and res[r][2] == ref_t


@pytest.mark.parametrize("kw", [dict(env="cliff_walking", algo="qlearning"),
                                dict(env="taxi", selector="ucb", algo="expected_sarsa"),
                                dict(env="frozen_lake", agent="traces", policy="double", algo="sarsa")],
                         ids=["cw-q", "taxi-ucb-es", "fl-traces-double"])
def test_dyna_private_batch_equals_faithful(oracle, kw):
    """InternalModelAgent + RandomModel (src/agent/internal_model_agent.rs:47-77,
    src/model/random_model.rs:27-40) with 10 planning steps: the batch's private
    lanes reproduce the faithful Dyna loop bit for bit."""
    n = 30
    p = oracle.default_params(map8x8=1, n_episodes_for_decay=n, n_lanes=2, group_size=1, sync_every=41, **kw)
    b = oracle.Batch(p)
    b.set_planning(10)
    b.train_episodes(n, n // 3)
    q = b.q()
    for lane in range(2):
        f = oracle.Faithful(dict(p, lane_offset=lane))
        f.set_planning(10)
        f.train(n, n // 3)
        assert _eq_nan(f.q(), q[lane])
    # planning changes the result (the model is used; FrozenLake's Q stays 0
    # until a goal is reached)
    if kw["env"] != "frozen_lake":
        b0 = oracle.Batch(p)
        b0.train_episodes(n, n // 3)
        assert not _eq_nan(b0.q(), q)


def test_gen_range_index_kat(oracle):
    """rand 0.8.5 sample_single_inclusive for usize: zone = (range << lz(range)) - 1."""
    L = oracle.lib()
    rej = __import__("ctypes").c_int()
    # range 3: lz = 62, zone = 0xBFFF_FFFF_FFFF_FFFF; v * 3 = lo + hi * 2^64
    v = 0x5555555555555556                       # v*3 = 2^64 + 2 -> hi 1, lo 2
    assert L.rlo_gen_index_u64(v, 3, __import__("ctypes").byref(rej)) == 1 and rej.value == 0
    v = 0x4000000000000000                       # v*3 = 0xC000...0 -> lo > zone: reject
    L.rlo_gen_index_u64(v, 3, __import__("ctypes").byref(rej))
    assert rej.value == 1
    # range 4 (power of two): zone = 2^64 - 1, never rejects; index = top 2 bits
    assert L.rlo_gen_index_u64(0xC000000000000000, 4, __import__("ctypes").byref(rej)) == 3 and rej.value == 0


def test_ucb_counters_are_u64_and_monotone(oracle):
    """UCB counts (u128 in upper_confidence_bound.rs:11-12) never wrap: seeded
    just below 2^32 they only grow, and t grows by one per selection."""
    p = oracle.default_params(env="taxi", selector="ucb", algo="qlearning", n_lanes=256, group_size=64,
                              sync_every=16)
    b = oracle.Batch(p)
    n0 = np.full((b.S, b.A), (1 << 32) - 3, np.uint64)
    b.set_ucb(n0, 1 << 40)
    b.run(2)
    n, t = b.ucb()
    assert n.dtype == np.uint64 and (n >= n0).all() and (n > (1 << 32)).any()
    # every live lane selects once per synchronous step (reset or step)
    assert t - (1 << 40) == int((n - n0).sum()) == 2 * 16 * 256


def test_train_then_run_keeps_training_oracle(oracle):
    p = oracle.default_params(env="cliff_walking", agent="traces", algo="sarsa", n_lanes=64, group_size=32,
                              sync_every=16, n_episodes_for_decay=40)
    b = oracle.Batch(p)
    b.train_episodes(3, 0)
    s0 = int(b.stats()[0])
    b.run(2)
    assert int(b.stats()[0]) > s0


def test_reset_step_schedule_is_the_reference_loop_per_lane(oracle):
    """Reset-and-step schedule (oracle/rlref.c, rl_agent_set_reset_step): every
    synchronous step of a live lane is an Env::step; a kind-3 record starts an
    episode (its s is the start state, src/env/frozen_lake.rs:106-113) and follows
    the lane's previous terminal step; run mode steps every lane K times per launch."""
    p = oracle.default_params(env="frozen_lake", map8x8=1, n_lanes=300, group_size=64, sync_every=20)
    b = oracle.Batch(p)
    b.set_reset_step(True)
    b.set_record(True)
    b.run(3)
    recs = b.records()
    assert set(np.unique(recs["kind"])) <= {oracle.KIND_STEP, oracle.KIND_RESET_STEP}
    assert (recs["s"][recs["kind"] == oracle.KIND_RESET_STEP] == 0).all()
    assert b.stats()[0] == 3 * 20 * 300
    for lane in range(0, 300, 37):
        r = recs[:, lane]
        starts = r["kind"] == oracle.KIND_RESET_STEP
        # an episode starts at step 0 or right after a terminal step, and only there
        prev_term = np.concatenate([[True], r["term"][:-1] == 1])
        assert np.array_equal(starts, prev_term)
        # consecutive steps inside an episode chain s2 -> s, a2 -> a
        cont = ~starts[1:]
        assert np.array_equal(r["s"][1:][cont], r["s2"][:-1][cont])
        assert np.array_equal(r["a"][1:][cont], r["a2"][:-1][cont])
