"""ctypes binding to the CPU oracle (oracle/_build/librlref.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the product path.
See oracle/rlref.h for what it restates and its parity status.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "librlref.so")

ENV = {"frozen_lake": 0, "cliff_walking": 1, "taxi": 2, "blackjack": 3, "frozen_lake_edited": 4}
AGENT = {"one_step": 0, "traces": 1}
POLICY = {"tabular": 0, "double": 1, "neural": 2}
ACT = {"linear": 0, "tanh": 1, "relu": 2, "leaky_relu": 3, "relu6": 4, "leaky_relu6": 5,
       "sigmoid": 6, "softmax": 7, "swish": 8, "hard_swish": 9}
INPUT = {"scalar": 0, "fl_obs": 1}
SELECTOR = {"eps_greedy": 0, "ucb": 1}
ALGO = {"sarsa": 0, "qlearning": 1, "expected_sarsa": 2}
MODE_TRAIN, MODE_EVAL, MODE_DONE = 0, 1, 2


class Config(C.Structure):
    _fields_ = [
        ("env", C.c_int32), ("map8x8", C.c_int32), ("slippery", C.c_int32),
        ("max_steps", C.c_uint32),
        ("agent", C.c_int32), ("policy", C.c_int32), ("selector", C.c_int32),
        ("algo", C.c_int32), ("decay_kind", C.c_int32),
        ("lr", C.c_double), ("gamma", C.c_double), ("lambda_", C.c_double),
        ("eps0", C.c_double), ("eps_decay", C.c_double), ("eps_final", C.c_double),
        ("ucb_c", C.c_double), ("q_default", C.c_double),
        ("seed", C.c_uint64), ("lane_offset", C.c_uint64),
        ("n_lanes", C.c_uint32), ("group_size", C.c_uint32), ("sync_every", C.c_uint32),
        ("eval_episodes", C.c_uint32),
        ("net_input", C.c_int32), ("net_hidden", C.c_uint32),
        ("net_act1", C.c_int32), ("net_act2", C.c_int32),
    ]


RECORD_DTYPE = np.dtype([("s", "<u4"), ("s2", "<u4"), ("a", "u1"), ("a2", "u1"),
                         ("term", "u1"), ("mode", "u1"), ("kind", "u1"), ("pad", "u1", (3,)),
                         ("r", "<f8"), ("td", "<f8")])
KIND_IDLE, KIND_RESET, KIND_STEP, KIND_RESET_STEP = 0, 1, 2, 3
# shared-Q representation (oracle/rlref.h): reported / requested
QREPR = {0: "fixed40", 1: "f64", 2: "private"}
QMODE = {"auto": 0, "f64": 1, "f64_seq": 2, "fixed_range": 3}
assert RECORD_DTYPE.itemsize == 32


def default_params(**kw):
    """Reference CLI defaults (src/bin/frozen_lake.rs:35-73, decay :84)."""
    p = dict(env="frozen_lake", map8x8=0, slippery=0, max_steps=100, agent="one_step",
             policy="tabular", selector="eps_greedy", algo="qlearning", decay_kind=0,
             lr=0.05, gamma=0.95, lambda_=0.5, eps0=1.0, n_episodes_for_decay=100000,
             exploration_time=0.5, eps_final=0.0, ucb_c=0.5, q_default=0.0, seed=0x5EED,
             lane_offset=0, n_lanes=1, group_size=1, sync_every=64, eval_episodes=100,
             net_input="scalar", net_hidden=32, net_act1="leaky_relu6", net_act2="linear")
    p.update(kw)
    if "eps_decay" not in p:
        p["eps_decay"] = p["eps0"] / (p["exploration_time"] * p["n_episodes_for_decay"])
    return p


def make_config(p):
    c = Config()
    c.env = ENV[p["env"]] if isinstance(p["env"], str) else p["env"]
    c.map8x8, c.slippery, c.max_steps = p["map8x8"], p["slippery"], p["max_steps"]
    c.agent = AGENT[p["agent"]] if isinstance(p["agent"], str) else p["agent"]
    c.policy = POLICY[p["policy"]] if isinstance(p["policy"], str) else p["policy"]
    c.selector = SELECTOR[p["selector"]] if isinstance(p["selector"], str) else p["selector"]
    c.algo = ALGO[p["algo"]] if isinstance(p["algo"], str) else p["algo"]
    c.decay_kind = p["decay_kind"]
    for k in ("lr", "gamma", "lambda_", "eps0", "eps_decay", "eps_final", "ucb_c", "q_default"):
        setattr(c, k, float(p[k]))
    c.seed, c.lane_offset = p["seed"], p["lane_offset"]
    c.n_lanes, c.group_size, c.sync_every = p["n_lanes"], p["group_size"], p["sync_every"]
    c.eval_episodes = p["eval_episodes"]
    c.net_input = INPUT[p.get("net_input", "scalar")]
    c.net_hidden = p.get("net_hidden", 32)
    c.net_act1 = ACT[p.get("net_act1", "leaky_relu6")]
    c.net_act2 = ACT[p.get("net_act2", "linear")]
    return c


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.rlo_log.restype = C.c_double
        L.rlo_log.argtypes = [C.c_double]
        L.rlo_rng_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, P(C.c_uint32)]
        L.rlo_u64_to_uniform01.restype = C.c_double
        L.rlo_u64_to_uniform01.argtypes = [C.c_uint64]
        L.rlo_uniform_int_u64.restype = C.c_uint32
        L.rlo_uniform_int_u64.argtypes = [C.c_uint64, C.c_uint64, P(C.c_int)]
        L.rlo_gen_index_u64.restype = C.c_uint64
        L.rlo_gen_index_u64.argtypes = [C.c_uint64, C.c_uint64, P(C.c_int)]
        L.rlo_faithful_set_planning.argtypes = [C.c_void_p, C.c_uint32]
        L.rlo_batch_set_reset_step.argtypes = [C.c_void_p, C.c_int]
        L.rlo_batch_set_planning.restype = C.c_int
        L.rlo_batch_set_planning.argtypes = [C.c_void_p, C.c_uint32]
        L.rlo_uniform_card_u32.restype = C.c_uint32
        L.rlo_uniform_card_u32.argtypes = [C.c_uint32, P(C.c_int)]
        L.rlo_uniform_card_u16.restype = C.c_uint32
        L.rlo_eps_test_words.restype = C.c_int
        L.rlo_eps_test_words.argtypes = [C.c_uint32, C.c_uint32, C.c_double, P(C.c_int)]
        L.rlo_uniform_card_u16.argtypes = [C.c_uint32, P(C.c_int)]
        L.rlo_blackjack_obs_id.restype = C.c_uint64
        L.rlo_blackjack_obs_id.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.rlo_env_dims.argtypes = [P(Config), P(C.c_uint32), P(C.c_uint32)]
        L.rlo_env_table.argtypes = [P(Config), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_env_start.argtypes = [P(Config), C.c_void_p]
        L.rlo_env_walk.argtypes = [P(Config), C.c_uint64, C.c_uint32, C.c_void_p, P(C.c_uint32),
                                   C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_faithful_create.restype = C.c_void_p
        L.rlo_faithful_create.argtypes = [P(Config)]
        L.rlo_faithful_destroy.argtypes = [C.c_void_p]
        L.rlo_faithful_train.restype = C.c_uint64
        L.rlo_faithful_train.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.rlo_faithful_evaluate.restype = C.c_uint64
        L.rlo_faithful_evaluate.argtypes = [C.c_void_p, C.c_uint64]
        L.rlo_faithful_reset.argtypes = [C.c_void_p]
        L.rlo_faithful_get_q.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_faithful_n_episodes.restype = C.c_uint64
        L.rlo_faithful_n_episodes.argtypes = [C.c_void_p]
        L.rlo_faithful_n_steps.restype = C.c_uint64
        L.rlo_faithful_n_steps.argtypes = [C.c_void_p]
        L.rlo_faithful_histories.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_faithful_get_records.restype = C.c_uint64
        L.rlo_faithful_get_records.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.rlo_faithful_set_record.argtypes = [C.c_void_p, C.c_int]
        L.rlo_faithful_epsilon.restype = C.c_double
        L.rlo_faithful_epsilon.argtypes = [C.c_void_p]
        L.rlo_batch_create.restype = C.c_void_p
        L.rlo_batch_create.argtypes = [P(Config)]
        L.rlo_batch_destroy.argtypes = [C.c_void_p]
        L.rlo_batch_run.argtypes = [C.c_void_p, C.c_uint32]
        L.rlo_batch_train_episodes.restype = C.c_uint64
        L.rlo_batch_train_episodes.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.rlo_batch_evaluate.restype = C.c_uint64
        L.rlo_batch_evaluate.argtypes = [C.c_void_p, C.c_uint64]
        L.rlo_batch_reset.argtypes = [C.c_void_p]
        L.rlo_batch_get_q.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_get_q_raw.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_set_q.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_get_qflags.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_get_ucb.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_batch_set_ucb.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_batch_set_record.argtypes = [C.c_void_p, C.c_int]
        L.rlo_batch_take_records.restype = C.c_uint64
        L.rlo_batch_take_records.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.rlo_batch_delta_words.restype = C.c_uint64
        L.rlo_batch_delta_words.argtypes = [C.c_void_p]
        L.rlo_batch_launch_groups.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_apply_delta.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_delta_max_words.restype = C.c_uint64
        L.rlo_batch_delta_max_words.argtypes = [C.c_void_p]
        L.rlo_batch_fold.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_set_q_mode.argtypes = [C.c_void_p, C.c_int]
        L.rlo_batch_q_repr.restype = C.c_int
        L.rlo_batch_q_repr.argtypes = [C.c_void_p]
        L.rlo_batch_set_merge_groups.argtypes = [C.c_void_p, C.c_uint64]
        L.rlo_trace_grid_k.restype = C.c_int
        L.rlo_trace_grid_k.argtypes = [C.c_double, C.c_double, C.c_double, C.c_uint32, C.c_int32]
        L.rlo_batch_n_records.restype = C.c_uint64
        L.rlo_batch_n_records.argtypes = [C.c_void_p]
        L.rlo_batch_stats.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_lane_eps.argtypes = [C.c_void_p, C.c_void_p]
        L.rlo_batch_set_selector.argtypes = [C.c_void_p, C.c_int32]
        L.rlo_batch_set_algo.argtypes = [C.c_void_p, C.c_int32]
        for fn in ("rlo_exp", "rlo_expm1", "rlo_tanh"):
            getattr(L, fn).restype = C.c_double
            getattr(L, fn).argtypes = [C.c_double]
        L.rlo_act.argtypes = [C.c_int32, C.c_double, P(C.c_double), P(C.c_double)]
        L.rlo_net_dims.argtypes = [P(Config), P(C.c_uint32), P(C.c_uint32)]
        L.rlo_net_features.argtypes = [P(Config), C.c_void_p]
        L.rlo_net_init.argtypes = [P(Config), C.c_uint64, C.c_uint32, C.c_void_p]
        L.rlo_net_forward.argtypes = [P(Config), C.c_void_p, C.c_void_p, C.c_void_p]
        L.rlo_net_fit.argtypes = [P(Config), C.c_void_p, C.c_void_p, C.c_void_p, C.c_double]
        for fn in ("rlo_faithful_get_weights", "rlo_faithful_set_weights", "rlo_batch_get_weights",
                   "rlo_batch_set_weights"):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def dims(p):
    c = make_config(p)
    S, A = C.c_uint32(), C.c_uint32()
    assert lib().rlo_env_dims(C.byref(c), C.byref(S), C.byref(A)) == 0
    return S.value, A.value


def env_table(p):
    S, A = dims(p)
    c = make_config(p)
    n = S * A * 3
    prob = np.zeros(n, np.float64)
    nxt = np.zeros(n, np.uint32)
    rew = np.zeros(n, np.float64)
    term = np.zeros(n, np.uint8)
    rc = lib().rlo_env_table(C.byref(c), prob.ctypes.data, nxt.ctypes.data, rew.ctypes.data,
                             term.ctypes.data)
    assert rc == 0
    start = np.zeros(S, np.float64)
    assert lib().rlo_env_start(C.byref(c), start.ctypes.data) == 0
    shp = (S, A, 3)
    return dict(prob=prob.reshape(shp), next=nxt.reshape(shp), reward=rew.reshape(shp),
                term=term.reshape(shp), start=start)


def env_walk(p, actions, lane=0):
    """Env::reset + Env::step(a) for each action; stops at EnvNotReady."""
    c = make_config(p)
    a = np.ascontiguousarray(actions, dtype=np.uint32)
    n = a.size
    s0 = C.c_uint32()
    s2 = np.zeros(n, np.uint32)
    r = np.zeros(n, np.float64)
    t = np.zeros(n, np.uint8)
    k = lib().rlo_env_walk(C.byref(c), lane, n, a.ctypes.data, C.byref(s0), s2.ctypes.data,
                           r.ctypes.data, t.ctypes.data)
    assert k >= 0
    return s0.value, s2[:k], r[:k], t[:k].astype(bool), k


def act(name, x):
    """activation f(x), f'(x) (src/network/activation.rs), elementwise"""
    x = np.asarray(x, np.float64).reshape(-1)
    f, fp = np.zeros_like(x), np.zeros_like(x)
    a, b = C.c_double(), C.c_double()
    for i, v in enumerate(x):
        lib().rlo_act(ACT[name], float(v), C.byref(a), C.byref(b))
        f[i], fp[i] = a.value, b.value
    return f, fp


def net_dims(p):
    c = make_config(p)
    n_in, n_par = C.c_uint32(), C.c_uint32()
    assert lib().rlo_net_dims(C.byref(c), C.byref(n_in), C.byref(n_par)) == 0, "no valid network"
    return n_in.value, n_par.value


def net_features(p):
    S, _ = dims(p)
    n_in, _ = net_dims(p)
    out = np.zeros(S * n_in, np.float64)
    c = make_config(p)
    assert lib().rlo_net_features(C.byref(c), out.ctypes.data) == 0
    return out.reshape(S, n_in)


def net_init(p, lane, gen=0):
    _, n_par = net_dims(p)
    w = np.zeros(n_par, np.float64)
    c = make_config(p)
    lib().rlo_net_init(C.byref(c), lane, gen, w.ctypes.data)
    return w


def net_forward(p, w, x):
    _, A = dims(p)
    y = np.zeros(A, np.float64)
    c = make_config(p)
    w = np.ascontiguousarray(w, np.float64)
    x = np.ascontiguousarray(x, np.float64)
    lib().rlo_net_forward(C.byref(c), w.ctypes.data, x.ctypes.data, y.ctypes.data)
    return y


def net_fit(p, w, x, y, lr):
    """Network::fit in place on a copy; returns the new parameters"""
    c = make_config(p)
    w = np.array(w, np.float64)
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    lib().rlo_net_fit(C.byref(c), w.ctypes.data, x.ctypes.data, y.ctypes.data, float(lr))
    return w


def rng_stream(seed, lane, n):
    out = np.zeros(n, np.uint32)
    lib().rlo_rng_stream(seed, lane, n, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


class Faithful:
    """Single env + agent, f64 Q: src/agent.rs:66-141 restated."""

    def __init__(self, p):
        self.p = p
        self.S, self.A = dims(p)
        self.P = 2 if p["policy"] == "double" else 1
        self.cfg = make_config(p)
        self.h = lib().rlo_faithful_create(C.byref(self.cfg))
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().rlo_faithful_destroy(self.h)
            self.h = None

    def set_record(self, on=True):
        lib().rlo_faithful_set_record(self.h, int(on))

    def set_planning(self, n):
        lib().rlo_faithful_set_planning(self.h, n)

    def train(self, n_episodes, eval_at=0):
        return lib().rlo_faithful_train(self.h, n_episodes, eval_at)

    def evaluate(self, n_episodes):
        return lib().rlo_faithful_evaluate(self.h, n_episodes)

    def reset(self):
        lib().rlo_faithful_reset(self.h)

    def q(self):
        out = np.zeros(self.P * self.S * self.A, np.float64)
        lib().rlo_faithful_get_q(self.h, out.ctypes.data)
        return out.reshape(self.P, self.S, self.A)

    def histories(self):
        ne = lib().rlo_faithful_n_episodes(self.h)
        ns = lib().rlo_faithful_n_steps(self.h)
        rh = np.zeros(ne, np.float64)
        el = np.zeros(ne, np.uint64)
        te = np.zeros(ns, np.float64)
        lib().rlo_faithful_histories(self.h, rh.ctypes.data, el.ctypes.data, te.ctypes.data)
        return rh, el, te

    def records(self):
        n = lib().rlo_faithful_get_records(self.h, None, 0)
        out = np.zeros(n, RECORD_DTYPE)
        lib().rlo_faithful_get_records(self.h, out.ctypes.data, n)
        return out

    def epsilon(self):
        return lib().rlo_faithful_epsilon(self.h)

    def weights(self):
        _, n_par = net_dims(self.p)
        out = np.zeros(n_par, np.float64)
        lib().rlo_faithful_get_weights(self.h, out.ctypes.data)
        return out

    def set_weights(self, w):
        w = np.ascontiguousarray(w, np.float64)
        lib().rlo_faithful_set_weights(self.h, w.ctypes.data)


class Batch:
    """The batched schedule the GPU implements (shared Q as 2^-40 fixed point where
    the range proof holds, else f64 with exponent-grid sums; rlref.c section 2)."""

    def __init__(self, p):
        self.p = p
        self.S, self.A = dims(p)
        self.P = 2 if p["policy"] == "double" else 1
        self.L = p["n_lanes"]
        self.cfg = make_config(p)
        self.h = lib().rlo_batch_create(C.byref(self.cfg))
        assert self.h

    def __del__(self):
        if getattr(self, "h", None):
            lib().rlo_batch_destroy(self.h)
            self.h = None

    def set_record(self, on=True):
        lib().rlo_batch_set_record(self.h, int(on))

    def run(self, n_launches):
        lib().rlo_batch_run(self.h, n_launches)

    def train_episodes(self, n, eval_at=0):
        return lib().rlo_batch_train_episodes(self.h, n, eval_at)

    def evaluate(self, n):
        return lib().rlo_batch_evaluate(self.h, n)

    def reset(self):
        lib().rlo_batch_reset(self.h)

    def set_selector(self, s):
        lib().rlo_batch_set_selector(self.h, SELECTOR[s])

    def set_algo(self, a):
        lib().rlo_batch_set_algo(self.h, ALGO[a])

    def set_planning(self, n):
        assert lib().rlo_batch_set_planning(self.h, n) == 0, "Dyna planning needs group_size 1"

    def set_reset_step(self, on=True):
        lib().rlo_batch_set_reset_step(self.h, int(on))

    @property
    def private(self):
        return self.p["group_size"] == 1

    def q(self):
        """shared mode: [P,S,A]; private mode (G == 1): [L,P,S,A]"""
        n = self.P * self.S * self.A * (self.L if self.private else 1)
        out = np.zeros(n, np.float64)
        lib().rlo_batch_get_q(self.h, out.ctypes.data)
        if self.private:
            return out.reshape(self.L, self.P, self.S, self.A)
        return out.reshape(self.P, self.S, self.A)

    def set_q(self, q):
        q = np.ascontiguousarray(q, dtype=np.float64)
        lib().rlo_batch_set_q(self.h, q.ctypes.data)

    def q_raw(self):
        out = np.zeros(self.P * self.S * self.A, np.int64)
        lib().rlo_batch_get_q_raw(self.h, out.ctypes.data)
        return out.reshape(self.P, self.S, self.A)

    def qflags(self):
        out = np.zeros(self.P * self.S * self.A, np.uint8)
        lib().rlo_batch_get_qflags(self.h, out.ctypes.data)
        return out.reshape(self.P, self.S, self.A)

    def ucb(self):
        if self.private:
            n = np.zeros(self.L * self.S * self.A, np.uint64)
            t = np.zeros(self.L, np.uint64)
            lib().rlo_batch_get_ucb(self.h, n.ctypes.data, t.ctypes.data)
            return n.reshape(self.L, self.S, self.A), t
        n = np.zeros(self.S * self.A, np.uint64)
        t = C.c_uint64()
        lib().rlo_batch_get_ucb(self.h, n.ctypes.data, C.byref(t))
        return n.reshape(self.S, self.A), t.value

    def set_ucb(self, counts, t):
        """UCB counters: shared [S][A] + t, private [L][S][A] + t[L] (u64)"""
        counts = np.ascontiguousarray(counts, np.uint64)
        t = np.ascontiguousarray(np.atleast_1d(t), np.uint64)
        lib().rlo_batch_set_ucb(self.h, counts.ctypes.data, t.ctypes.data)

    def records(self):
        """[n_steps, n_lanes] records since the last call (clears the buffer)."""
        n = lib().rlo_batch_n_records(self.h)
        out = np.zeros(n, RECORD_DTYPE)
        lib().rlo_batch_take_records(self.h, out.ctypes.data, n)
        return out.reshape(-1, self.L)

    def set_q_mode(self, mode):
        """'auto' (fixed point where proven), 'f64', 'f64_seq' (oracle only: f64
        with sequential lane-order / group-order sums, the drift reference) or
        'fixed_range' (oracle only: the fixed point wherever the range proof holds,
        slippery maps included — round 5's auto, for the drift curve)"""
        lib().rlo_batch_set_q_mode(self.h, QMODE[mode])

    def q_repr(self):
        return QREPR[lib().rlo_batch_q_repr(self.h)]

    def set_merge_groups(self, total_groups):
        lib().rlo_batch_set_merge_groups(self.h, total_groups)

    def delta_words(self):
        """merge buffer words: delta_max_words() MAX words, then the SUM words"""
        return lib().rlo_batch_delta_words(self.h)

    def delta_max_words(self):
        return lib().rlo_batch_delta_max_words(self.h)

    def launch_groups(self, delta):
        """run local groups for K steps, adding their merge delta into `delta` (int64)"""
        assert delta.dtype == np.int64 and delta.flags.c_contiguous
        lib().rlo_batch_launch_groups(self.h, delta.ctypes.data)

    def fold(self, delta):
        """second merge phase (after the MAX all-reduce of the first words)"""
        assert delta.dtype == np.int64 and delta.flags.c_contiguous
        lib().rlo_batch_fold(self.h, delta.ctypes.data)

    def apply_delta(self, delta):
        lib().rlo_batch_apply_delta(self.h, np.ascontiguousarray(delta, np.int64).ctypes.data)

    def stats(self):
        """rl_stats order: 0 train_steps .. 7 trace_states, 8 q_clamp_hits, 9 delta_saturations"""
        out = np.zeros(16, np.uint64)
        lib().rlo_batch_stats(self.h, out.ctypes.data)
        return out

    def lane_eps(self):
        out = np.zeros(self.L, np.float64)
        lib().rlo_batch_lane_eps(self.h, out.ctypes.data)
        return out

    def weights(self):
        _, n_par = net_dims(self.p)
        out = np.zeros(self.L * n_par, np.float64)
        lib().rlo_batch_get_weights(self.h, out.ctypes.data)
        return out.reshape(self.L, n_par)

    def set_weights(self, w):
        w = np.ascontiguousarray(w, np.float64)
        lib().rlo_batch_set_weights(self.h, w.ctypes.data)
