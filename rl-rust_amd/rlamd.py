"""ctypes binding to librlamd.so (include/rl.h) for tests and bench.py.

This is plumbing over the C ABI, shaped like the reference's Rust traits
(src/env.rs:19-49 Env, src/agent.rs:47-164 Agent).  All compute runs in the
gfx950 kernels of librlamd.so; there is no CPU fallback: if the library or a
GPU is missing, every compute call raises RLError.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("RLAMD_LIB", os.path.join(HERE, "lib", "librlamd.so"))
INCLUDE_H = os.path.join(ROOT, "include", "rl.h")

ENV = {"frozen_lake": 0, "cliff_walking": 1, "taxi": 2, "blackjack": 3, "frozen_lake_edited": 4}
AGENT = {"one_step": 0, "traces": 1}
POLICY = {"tabular": 0, "double": 1, "neural": 2}
ACT = {"linear": 0, "tanh": 1, "relu": 2, "leaky_relu": 3, "relu6": 4, "leaky_relu6": 5,
       "sigmoid": 6, "softmax": 7, "swish": 8, "hard_swish": 9}
INPUT = {"scalar": 0, "fl_obs": 1}
SELECTOR = {"eps_greedy": 0, "ucb": 1}
ALGO = {"sarsa": 0, "qlearning": 1, "expected_sarsa": 2}
RL_OK, RL_E_NOT_READY = 0, 1


class RLError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rl error {code}: {msg}")
        self.code = code


class EnvConfig(C.Structure):
    _fields_ = [("kind", C.c_int32), ("map8x8", C.c_int32), ("slippery", C.c_int32),
                ("max_steps", C.c_uint32)]


class NetConfig(C.Structure):
    _fields_ = [("input", C.c_int32), ("hidden", C.c_uint32), ("act_hidden", C.c_int32),
                ("act_out", C.c_int32)]


class AgentConfig(C.Structure):
    _fields_ = [
        ("env", EnvConfig),
        ("agent", C.c_int32), ("policy", C.c_int32), ("selector", C.c_int32),
        ("algo", C.c_int32), ("decay_kind", C.c_int32),
        ("lr", C.c_double), ("gamma", C.c_double), ("lambda_", C.c_double),
        ("eps0", C.c_double), ("eps_decay", C.c_double), ("eps_final", C.c_double),
        ("ucb_c", C.c_double), ("q_default", C.c_double),
        ("seed", C.c_uint64), ("lane_offset", C.c_uint64),
        ("n_lanes", C.c_uint32), ("group_size", C.c_uint32), ("sync_every", C.c_uint32),
        ("eval_episodes", C.c_uint32), ("device", C.c_int32),
        ("net", NetConfig),
    ]


class Stats(C.Structure):
    _fields_ = [("train_steps", C.c_uint64), ("eval_steps", C.c_uint64),
                ("train_episodes", C.c_uint64), ("eval_episodes", C.c_uint64),
                ("reward_sum_q16", C.c_int64), ("done_lanes", C.c_uint64),
                ("launches", C.c_uint64), ("trace_states", C.c_uint64),
                ("q_clamp_hits", C.c_uint64), ("delta_saturations", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


RECORD_DTYPE = np.dtype([("s", "<u4"), ("s2", "<u4"), ("a", "u1"), ("a2", "u1"),
                         ("term", "u1"), ("mode", "u1"), ("kind", "u1"), ("pad", "u1", (3,)),
                         ("r", "<f8"), ("td", "<f8")])
KIND_IDLE, KIND_RESET, KIND_STEP = 0, 1, 2
QREPR = {0: "fixed40", 1: "f64", 2: "private"}     # rl.h rl_q_repr
QMODE = {"auto": 0, "f64": 1}                       # rl.h rl_q_mode
EPISODE_DTYPE = np.dtype([("lane", "<u4"), ("length", "<u4"), ("seq", "<u4"), ("mode", "u1"),
                          ("pad", "u1", (3,)), ("reward", "<f8")])

# every function include/rl.h declares: name -> (restype, argtypes)
_P = C.POINTER
_V = C.c_void_p
SIGNATURES = {
    "rl_last_error": (C.c_char_p, []),
    "rl_abi_version": (C.c_int, []),
    "rl_build_info": (C.c_char_p, []),
    "rl_build_id": (C.c_char_p, []),
    "rl_obs_from_reference": (C.c_int, [C.c_int32, C.c_uint64, _P(C.c_uint32)]),
    "rl_agent_get_action": (C.c_int, [_V, C.c_uint32, C.c_uint64, _P(C.c_uint32)]),
    "rl_agent_update": (C.c_int, [_V, C.c_uint32, C.c_uint64, C.c_uint32, C.c_double, C.c_int32, C.c_uint64,
                                  C.c_uint32, _P(C.c_double)]),
    "rl_agent_get_actions": (C.c_int, [_V, _V, _V, C.c_uint64]),
    "rl_agent_updates": (C.c_int, [_V, _V, _V, _V, _V, _V, _V, _V, C.c_uint64]),
    "rl_agent_env": (C.c_int, [_V, _P(_V)]),
    "rl_env_reset_lane": (C.c_int, [_V, C.c_uint32, _P(C.c_uint64)]),
    "rl_env_step_lane": (C.c_int, [_V, C.c_uint32, C.c_uint32, _P(C.c_uint64), _P(C.c_double),
                                   _P(C.c_uint8)]),
    "rl_device_count": (C.c_int, [_P(C.c_int)]),
    "rl_blackjack_obs_id": (C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32]),
    "rl_obs_to_reference": (C.c_uint64, [C.c_int32, C.c_uint32]),
    "rl_env_dims": (C.c_int, [_P(EnvConfig), _P(C.c_uint32), _P(C.c_uint32)]),
    "rl_env_table": (C.c_int, [_P(EnvConfig), _V, _V, _V, _V, _V]),
    "rl_env_create": (C.c_int, [_P(EnvConfig), C.c_uint32, C.c_uint64, C.c_uint64, C.c_int32, _P(_V)]),
    "rl_env_destroy": (None, [_V]),
    "rl_env_reset": (C.c_int, [_V, _V]),
    "rl_env_step": (C.c_int, [_V, _V, _V, _V, _V]),
    "rl_agent_create": (C.c_int, [_P(AgentConfig), _P(_V)]),
    "rl_agent_destroy": (None, [_V]),
    "rl_agent_set_future_q_value_func": (C.c_int, [_V, C.c_int32]),
    "rl_agent_set_action_selector": (C.c_int, [_V, C.c_int32, C.c_double, C.c_double, C.c_double,
                                               C.c_int32, C.c_double]),
    "rl_agent_reset": (C.c_int, [_V]),
    "rl_agent_train": (C.c_int, [_V, C.c_uint64, C.c_uint64, _P(Stats)]),
    "rl_agent_evaluate": (C.c_int, [_V, C.c_uint64, _P(Stats)]),
    "rl_agent_run": (C.c_int, [_V, C.c_uint32]),
    "rl_agent_synchronize": (C.c_int, [_V]),
    "rl_agent_stats": (C.c_int, [_V, _P(Stats)]),
    "rl_agent_get_q": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_agent_set_q": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_agent_get_q_raw": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_agent_q_repr": (C.c_int, [_V, _P(C.c_int32)]),
    "rl_agent_set_q_mode": (C.c_int, [_V, C.c_int32]),
    "rl_agent_get_ucb": (C.c_int, [_V, _V, C.c_size_t, _V, C.c_size_t]),
    "rl_agent_set_ucb": (C.c_int, [_V, _V, C.c_size_t, _V, C.c_size_t]),
    "rl_agent_get_epsilon": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_agent_set_recording": (C.c_int, [_V, C.c_int32]),
    "rl_agent_take_records": (C.c_int, [_V, _V, C.c_uint64, _P(C.c_uint64)]),
    "rl_agent_set_episode_log": (C.c_int, [_V, C.c_uint32]),
    "rl_agent_set_planning": (C.c_int, [_V, C.c_uint32]),
    "rl_agent_set_reset_step": (C.c_int, [_V, C.c_int32]),
    "rl_agent_take_episodes": (C.c_int, [_V, _V, C.c_uint64, _P(C.c_uint64), _P(C.c_uint64)]),
    "rl_agent_dims": (C.c_int, [_V, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32)]),
    "rl_agent_lane_state": (C.c_int, [_V, _V, _V, C.c_size_t]),
    "rl_agent_delta_words": (C.c_int, [_V, _P(C.c_uint64)]),
    "rl_agent_delta_max_words": (C.c_int, [_V, _P(C.c_uint64)]),
    "rl_agent_delta_cap_words": (C.c_int, [_V, _P(C.c_uint64)]),
    "rl_agent_set_delta_buffer": (C.c_int, [_V, _V, C.c_uint64]),
    "rl_agent_set_merge_groups": (C.c_int, [_V, C.c_uint64]),
    "rl_agent_launch_train": (C.c_int, [_V]),
    "rl_agent_launch_fold": (C.c_int, [_V]),
    "rl_agent_launch_apply": (C.c_int, [_V]),
    "rl_agent_set_stream": (C.c_int, [_V, _V]),
    "rl_agent_occupancy": (C.c_int, [_V, _P(C.c_uint32), _P(C.c_uint64), _P(C.c_uint32)]),
    "rl_agent_set_timing": (C.c_int, [_V, C.c_int32]),
    "rl_agent_get_timing": (C.c_int, [_V, _P(C.c_double), _P(C.c_uint64)]),
    "rl_kat_log": (C.c_int, [C.c_int32, _V, _V, C.c_uint32]),
    "rl_kat_rng": (C.c_int, [C.c_int32, C.c_uint64, C.c_uint64, C.c_uint32, _V]),
    "rl_kat_ucb": (C.c_int, [C.c_int32, _V, _V, _V, C.c_double, _V, C.c_uint32]),
    "rl_kat_act": (C.c_int, [C.c_int32, C.c_int32, _V, _V, _V, C.c_uint32]),
    "rl_agent_net_dims": (C.c_int, [_V, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32)]),
    "rl_agent_get_weights": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_agent_set_weights": (C.c_int, [_V, _V, C.c_size_t]),
    "rl_net_features": (C.c_int, [_P(EnvConfig), C.c_int32, _V, C.c_size_t]),
    "rl_comm_unique_id": (C.c_int, [_V]),
    "rl_comm_init": (C.c_int, [C.c_int32, C.c_int32, _V, C.c_int32, _P(_V)]),
    "rl_comm_destroy": (None, [_V]),
    "rl_comm_rank": (C.c_int, [_V, _P(C.c_int32), _P(C.c_int32)]),
    "rl_agent_set_comm": (C.c_int, [_V, _V]),
    "rl_comm_allreduce_f64": (C.c_int, [_V, _V, C.c_uint32, C.c_int32]),
    "rl_agent_sync": (C.c_int, [_V]),
    "rl_agent_peer_handle": (C.c_int, [_V, _V]),
    "rl_agent_peer_attach": (C.c_int, [_V, C.c_int32, C.c_int32, _V]),
    "rl_agent_merge_path": (C.c_int, [_V, _P(C.c_int32)]),
    "rl_agent_get_q_lanes": (C.c_int, [_V, C.c_uint32, C.c_uint32, _V, C.c_size_t]),
    "rl_agent_get_weights_lanes": (C.c_int, [_V, C.c_uint32, C.c_uint32, _V, C.c_size_t]),
    "rl_agent_trace_items": (C.c_int, [_V, _P(C.c_uint64)]),
}
PEER_HANDLE_BYTES = 64
MERGE_PATHS = {0: "local", 1: "rccl", 2: "peer"}
COMM_ID_BYTES = 128

_lib = None


def source_id():
    """'src:<16 hex>' of this checkout's library sources, computed as the Makefile's
    ID_SRCS rule does (sha256 of csrc/*.{h,hip,cpp} sorted, include/rl.h, Makefile):
    equal to the loaded library's rl_build_id() prefix iff it was built from them"""
    import glob
    import hashlib
    files = sorted(os.path.relpath(f, HERE) for pat in ("csrc/*.h", "csrc/*.hip", "csrc/*.cpp")
                   for f in glob.glob(os.path.join(HERE, pat)))
    h = hashlib.sha256()
    for f in files + [os.path.join("..", "include", "rl.h"), "Makefile"]:
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    return "src:" + h.hexdigest()[:16]


def build_id():
    """rl_build_id() of the loaded library: 'src:<16 hex> git:<12 hex>'"""
    return lib().rl_build_id().decode()


def lib():
    """Load librlamd.so (fails loudly if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RLError(-1, f"{LIB_PATH} missing: build the HIP extension first (make -C rl-rust_amd)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != RL_OK:
        raise RLError(rc, lib().rl_last_error().decode())


def env_config(p):
    c = EnvConfig()
    c.kind = ENV[p["env"]] if isinstance(p["env"], str) else p["env"]
    c.map8x8, c.slippery, c.max_steps = p.get("map8x8", 0), p.get("slippery", 0), p.get("max_steps", 100)
    return c


def default_params(**kw):
    """Reference CLI defaults (src/bin/frozen_lake.rs:35-73; decay rule :84)."""
    p = dict(env="frozen_lake", map8x8=0, slippery=0, max_steps=100, agent="one_step",
             policy="tabular", selector="eps_greedy", algo="qlearning", decay_kind=0,
             lr=0.05, gamma=0.95, lambda_=0.5, eps0=1.0, n_episodes_for_decay=100000,
             exploration_time=0.5, eps_final=0.0, ucb_c=0.5, q_default=0.0, seed=0x5EED,
             lane_offset=0, n_lanes=1, group_size=1, sync_every=64, eval_episodes=100, device=0,
             net_input="scalar", net_hidden=32, net_act1="leaky_relu6", net_act2="linear")
    p.update(kw)
    if "eps_decay" not in p:
        p["eps_decay"] = p["eps0"] / (p["exploration_time"] * p["n_episodes_for_decay"])
    return p


def agent_config(p):
    c = AgentConfig()
    c.env = env_config(p)
    c.agent = AGENT[p["agent"]] if isinstance(p["agent"], str) else p["agent"]
    c.policy = POLICY[p["policy"]] if isinstance(p["policy"], str) else p["policy"]
    c.selector = SELECTOR[p["selector"]] if isinstance(p["selector"], str) else p["selector"]
    c.algo = ALGO[p["algo"]] if isinstance(p["algo"], str) else p["algo"]
    c.decay_kind = p["decay_kind"]
    for k in ("lr", "gamma", "lambda_", "eps0", "eps_decay", "eps_final", "ucb_c", "q_default"):
        setattr(c, k, float(p[k]))
    c.seed, c.lane_offset = p["seed"], p["lane_offset"]
    c.n_lanes, c.group_size, c.sync_every = p["n_lanes"], p["group_size"], p["sync_every"]
    c.eval_episodes, c.device = p["eval_episodes"], p["device"]
    c.net.input = INPUT[p.get("net_input", "scalar")]
    c.net.hidden = p.get("net_hidden", 32)
    c.net.act_hidden = ACT[p.get("net_act1", "leaky_relu6")]
    c.net.act_out = ACT[p.get("net_act2", "linear")]
    return c


def env_dims(p):
    c = env_config(p)
    S, A = C.c_uint32(), C.c_uint32()
    check(lib().rl_env_dims(C.byref(c), C.byref(S), C.byref(A)))
    return S.value, A.value


def env_table(p):
    """Decoded device transition tables (host-built, no GPU needed)."""
    S, A = env_dims(p)
    c = env_config(p)
    n = S * A * 3
    prob, nxt = np.zeros(n, np.float64), np.zeros(n, np.uint32)
    rew, term = np.zeros(n, np.float64), np.zeros(n, np.uint8)
    start = np.zeros(S, np.float64)
    check(lib().rl_env_table(C.byref(c), prob.ctypes.data, nxt.ctypes.data, rew.ctypes.data,
                             term.ctypes.data, start.ctypes.data))
    shp = (S, A, 3)
    return dict(prob=prob.reshape(shp), next=nxt.reshape(shp), reward=rew.reshape(shp),
                term=term.reshape(shp), start=start)


class Env:
    """Batched Env<usize, COUNT> (src/env.rs:19-49) on the GPU."""

    def __init__(self, p, n_envs=1, seed=0x5EED, lane_offset=0, device=0, _view_of=None):
        self.p = p
        self.n = n_envs
        self.S, self.A = env_dims(p)
        self.cfg = env_config(p)
        h = C.c_void_p()
        if _view_of is not None:     # Agent.env(): the agent's own lanes and RNG streams
            check(lib().rl_agent_env(_view_of.h, C.byref(h)))
            self._agent = _view_of
        else:
            check(lib().rl_env_create(C.byref(self.cfg), n_envs, seed, lane_offset, device, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().rl_env_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def action_size(self):
        return self.A

    def reset(self):
        obs = np.zeros(self.n, np.uint64)
        check(lib().rl_env_reset(self.h, obs.ctypes.data))
        return obs

    def reset_lane(self, lane):
        """Env::reset of one lane's env"""
        o = C.c_uint64()
        check(lib().rl_env_reset_lane(self.h, lane, C.byref(o)))
        return o.value

    def step_lane(self, lane, action):
        """Env::step of one lane's env: (obs, reward, terminated)"""
        o, r, t = C.c_uint64(), C.c_double(), C.c_uint8()
        check(lib().rl_env_step_lane(self.h, lane, int(action), C.byref(o), C.byref(r), C.byref(t)))
        return o.value, r.value, bool(t.value)

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.uint32)
        obs = np.zeros(self.n, np.uint64)
        rew = np.zeros(self.n, np.float64)
        term = np.zeros(self.n, np.uint8)
        check(lib().rl_env_step(self.h, a.ctypes.data, obs.ctypes.data, rew.ctypes.data,
                                term.ctypes.data))
        return obs, rew, term.astype(bool)


class Agent:
    """Batched Agent<usize, COUNT> (src/agent.rs:47-164) on the GPU."""

    def __init__(self, p):
        self.p = p
        self.cfg = agent_config(p)
        h = C.c_void_p()
        check(lib().rl_agent_create(C.byref(self.cfg), C.byref(h)))
        self.h = h
        S, A, P = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().rl_agent_dims(self.h, C.byref(S), C.byref(A), C.byref(P)))
        self.S, self.A, self.P = S.value, A.value, P.value
        self.L = p["n_lanes"]
        self.private = p["group_size"] == 1

    def close(self):
        v = getattr(self, "_env_view", None)
        if v is not None:
            v.close()
            self._env_view = None
        if getattr(self, "h", None):
            lib().rl_agent_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- the per-call Agent surface (trait Agent, src/agent.rs:52-62); private mode
    def env(self):
        """Env over this agent's lanes (rl_agent_env): one env per lane, drawing from
        the lane's RNG stream as the reference's thread_rng serves env and agent"""
        if getattr(self, "_env_view", None) is None:
            self._env_view = Env(self.p, self.L, _view_of=self)
        return self._env_view

    def get_action(self, obs, lane=0):
        a = C.c_uint32()
        check(lib().rl_agent_get_action(self.h, lane, int(obs), C.byref(a)))
        return a.value

    def update(self, curr_obs, curr_action, reward, terminated, next_obs, next_action, lane=0):
        td = C.c_double()
        check(lib().rl_agent_update(self.h, lane, int(curr_obs), int(curr_action), float(reward),
                                    int(bool(terminated)), int(next_obs), int(next_action), C.byref(td)))
        return td.value

    def _lane_arrays(self, **arrays):
        """every array exactly one entry per lane (the library reads
        n_lanes entries of each; rl.h ABI 6 also checks the length it is given)"""
        for name, x in arrays.items():
            if x.ndim != 1 or x.size != self.L:
                raise ValueError(f"{name}: {x.size} entries for {self.L} lanes")

    def get_actions(self, obs):
        obs = np.ascontiguousarray(obs, np.uint64)
        self._lane_arrays(obs=obs)
        out = np.zeros(self.L, np.uint32)
        check(lib().rl_agent_get_actions(self.h, obs.ctypes.data, out.ctypes.data, obs.size))
        return out

    def updates(self, s, a, r, term, s2, a2):
        s, s2 = np.ascontiguousarray(s, np.uint64), np.ascontiguousarray(s2, np.uint64)
        a, a2 = np.ascontiguousarray(a, np.uint32), np.ascontiguousarray(a2, np.uint32)
        r, term = np.ascontiguousarray(r, np.float64), np.ascontiguousarray(term, np.uint8)
        self._lane_arrays(s=s, a=a, r=r, term=term, s2=s2, a2=a2)
        td = np.zeros(self.L, np.float64)
        check(lib().rl_agent_updates(self.h, s.ctypes.data, a.ctypes.data, r.ctypes.data, term.ctypes.data,
                                     s2.ctypes.data, a2.ctypes.data, td.ctypes.data, s.size))
        return td

    def set_future_q_value_func(self, algo):
        check(lib().rl_agent_set_future_q_value_func(self.h, ALGO[algo]))

    def set_action_selector(self, selector, eps0=None, eps_decay=None, eps_final=None,
                            decay_kind=None, ucb_c=None):
        p = self.p
        check(lib().rl_agent_set_action_selector(
            self.h, SELECTOR[selector], p["eps0"] if eps0 is None else eps0,
            p["eps_decay"] if eps_decay is None else eps_decay,
            p["eps_final"] if eps_final is None else eps_final,
            p["decay_kind"] if decay_kind is None else decay_kind,
            p["ucb_c"] if ucb_c is None else ucb_c))

    def reset(self):
        check(lib().rl_agent_reset(self.h))

    def train(self, n_episodes, eval_at=0):
        st = Stats()
        check(lib().rl_agent_train(self.h, n_episodes, eval_at, C.byref(st)))
        return st.as_dict()

    def evaluate(self, n_episodes):
        st = Stats()
        check(lib().rl_agent_evaluate(self.h, n_episodes, C.byref(st)))
        return st.as_dict()

    def run(self, n_launches):
        check(lib().rl_agent_run(self.h, n_launches))

    def synchronize(self):
        check(lib().rl_agent_synchronize(self.h))

    def stats(self):
        st = Stats()
        check(lib().rl_agent_stats(self.h, C.byref(st)))
        return st.as_dict()

    def q(self):
        n = self.P * self.S * self.A * (self.L if self.private else 1)
        out = np.zeros(n, np.float64)
        check(lib().rl_agent_get_q(self.h, out.ctypes.data, n))
        if self.private:
            return out.reshape(self.L, self.P, self.S, self.A)
        return out.reshape(self.P, self.S, self.A)

    def set_q(self, q):
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1)
        check(lib().rl_agent_set_q(self.h, q.ctypes.data, q.size))

    def q_raw(self):
        """raw words of the shared Q: fixed-point integers or f64 bits (q_repr())"""
        n = self.P * self.S * self.A
        out = np.zeros(n, np.int64)
        check(lib().rl_agent_get_q_raw(self.h, out.ctypes.data, n))
        return out.reshape(self.P, self.S, self.A)

    def q_repr(self):
        r = C.c_int32()
        check(lib().rl_agent_q_repr(self.h, C.byref(r)))
        return QREPR[r.value]

    def set_q_mode(self, mode):
        """'auto' (the 2^-40 fixed point where its range is proven) or 'f64'"""
        check(lib().rl_agent_set_q_mode(self.h, QMODE[mode]))

    def ucb(self):
        if self.private:
            n = np.zeros(self.L * self.S * self.A, np.uint64)
            t = np.zeros(self.L, np.uint64)
            check(lib().rl_agent_get_ucb(self.h, n.ctypes.data, n.size, t.ctypes.data, t.size))
            return n.reshape(self.L, self.S, self.A), t
        n = np.zeros(self.S * self.A, np.uint64)
        t = np.zeros(1, np.uint64)
        check(lib().rl_agent_get_ucb(self.h, n.ctypes.data, n.size, t.ctypes.data, 1))
        return n.reshape(self.S, self.A), int(t[0])

    def set_ucb(self, counts, t):
        """UCB counters (shared [S][A] + t, private [L][S][A] + t[L], u64)"""
        counts = np.ascontiguousarray(counts, np.uint64).reshape(-1)
        t = np.ascontiguousarray(np.atleast_1d(t), np.uint64)
        check(lib().rl_agent_set_ucb(self.h, counts.ctypes.data, counts.size, t.ctypes.data, t.size))

    def epsilon(self):
        out = np.zeros(self.L, np.float64)
        check(lib().rl_agent_get_epsilon(self.h, out.ctypes.data, self.L))
        return out

    def set_recording(self, on=True):
        check(lib().rl_agent_set_recording(self.h, int(on)))

    def records(self):
        """[n_steps, n_lanes] rl_step_record since the last call (clears)."""
        n = C.c_uint64()
        check(lib().rl_agent_take_records(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, RECORD_DTYPE)
        check(lib().rl_agent_take_records(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out.reshape(-1, self.L)

    def set_reset_step(self, on=True):
        """batched schedule: a resetting lane also steps in the same synchronous step
        (shared mode, eps-greedy; rl.h rl_agent_set_reset_step)"""
        check(lib().rl_agent_set_reset_step(self.h, int(on)))

    def set_planning(self, planning_steps):
        """InternalModelAgent + RandomModel (Dyna-Q); private mode only."""
        check(lib().rl_agent_set_planning(self.h, planning_steps))

    def set_episode_log(self, capacity_per_lane):
        check(lib().rl_agent_set_episode_log(self.h, capacity_per_lane))

    def episodes(self):
        """Finished episodes since the last call (clears): EPISODE_DTYPE records,
        lane by lane, each lane oldest first; also returns the overwritten count."""
        n, lost = C.c_uint64(), C.c_uint64()
        check(lib().rl_agent_take_episodes(self.h, None, 0, C.byref(n), C.byref(lost)))
        out = np.zeros(n.value, EPISODE_DTYPE)
        check(lib().rl_agent_take_episodes(self.h, out.ctypes.data, n.value, C.byref(n), C.byref(lost)))
        return out, lost.value

    # ---- NeuralPolicy parameters (Layer::get_weights / set_weights)
    def net_dims(self):
        n_in, hid, npar = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().rl_agent_net_dims(self.h, C.byref(n_in), C.byref(hid), C.byref(npar)))
        return n_in.value, hid.value, npar.value

    def weights(self):
        _, _, npar = self.net_dims()
        out = np.zeros(self.L * npar, np.float64)
        check(lib().rl_agent_get_weights(self.h, out.ctypes.data, out.size))
        return out.reshape(self.L, npar)

    def set_weights(self, w):
        w = np.ascontiguousarray(w, dtype=np.float64).reshape(-1)
        check(lib().rl_agent_set_weights(self.h, w.ctypes.data, w.size))

    def lane_state(self):
        core = np.zeros((self.L, 4), np.uint32)
        aux = np.zeros((self.L, 4), np.uint32)
        check(lib().rl_agent_lane_state(self.h, core.ctypes.data, aux.ctypes.data, self.L))
        return core, aux

    # ---- multi-GPU merge as an external collective:
    # launch_train -> all-reduce MAX of the first delta_max_words() words ->
    # launch_fold -> all-reduce SUM of the rest -> launch_apply
    def delta_words(self):
        n = C.c_uint64()
        check(lib().rl_agent_delta_words(self.h, C.byref(n)))
        return n.value

    def delta_max_words(self):
        n = C.c_uint64()
        check(lib().rl_agent_delta_max_words(self.h, C.byref(n)))
        return n.value

    def delta_cap_words(self):
        """the largest merge layout of either representation (size caller buffers by it)"""
        n = C.c_uint64()
        check(lib().rl_agent_delta_cap_words(self.h, C.byref(n)))
        return n.value

    def set_merge_groups(self, total_groups):
        check(lib().rl_agent_set_merge_groups(self.h, total_groups))

    def launch_fold(self):
        check(lib().rl_agent_launch_fold(self.h))

    def set_delta_buffer(self, ptr, n_words):
        check(lib().rl_agent_set_delta_buffer(self.h, C.c_void_p(ptr), n_words))

    def launch_train(self):
        check(lib().rl_agent_launch_train(self.h))

    def launch_apply(self):
        check(lib().rl_agent_launch_apply(self.h))

    def set_comm(self, comm):
        """all-reduce every merge over an RCCL communicator (None: detach)"""
        self._comm = comm                     # keep it alive while attached
        check(lib().rl_agent_set_comm(self.h, comm.h if comm is not None else None))

    def sync(self):
        """the merge after launch_train(): RCCL all-reduces (MAX, fold, SUM), then apply"""
        check(lib().rl_agent_sync(self.h))

    # ---- ABI 7: the one-shot peer-read merge (rl.h rl_agent_peer_handle / _attach)
    def peer_handle(self):
        """this rank's exchange-region IPC handle (RL_PEER_HANDLE_BYTES bytes)"""
        buf = (C.c_uint8 * PEER_HANDLE_BYTES)()
        check(lib().rl_agent_peer_handle(self.h, buf))
        return bytes(buf)

    def peer_attach(self, rank, world, handles):
        """every rank's handle, in rank order: from then on every merge reads the peers"""
        assert len(handles) == world and all(len(h) == PEER_HANDLE_BYTES for h in handles)
        buf = (C.c_uint8 * (PEER_HANDLE_BYTES * world)).from_buffer_copy(b"".join(handles))
        check(lib().rl_agent_peer_attach(self.h, rank, world, buf))

    def q_lanes(self, lane0, n_lanes):
        """private mode: Q of lanes [lane0, lane0 + n_lanes), [n][P][S][A] as q()'s"""
        q = np.zeros((n_lanes, self.P, self.S, self.A), np.float64)
        check(lib().rl_agent_get_q_lanes(self.h, lane0, n_lanes, q.ctypes.data, q.size))
        return q

    def weights_lanes(self, lane0, n_lanes):
        nin, hid, npar = self.net_dims()
        w = np.zeros((n_lanes, npar), np.float64)
        check(lib().rl_agent_get_weights_lanes(self.h, lane0, n_lanes, w.ctypes.data, w.size))
        return w

    def trace_items(self):
        v = C.c_uint64()
        check(lib().rl_agent_trace_items(self.h, C.byref(v)))
        return v.value

    def merge_path(self):
        v = C.c_int32()
        check(lib().rl_agent_merge_path(self.h, C.byref(v)))
        return MERGE_PATHS[v.value]

    def set_stream(self, stream_ptr):
        check(lib().rl_agent_set_stream(self.h, C.c_void_p(stream_ptr)))

    def occupancy(self):
        g, b, t = C.c_uint32(), C.c_uint64(), C.c_uint32()
        check(lib().rl_agent_occupancy(self.h, C.byref(g), C.byref(b), C.byref(t)))
        return {"groups_per_cu": g.value, "lds_bytes": b.value, "block_threads": t.value}

    def set_timing(self, on=True):
        check(lib().rl_agent_set_timing(self.h, int(on)))

    def timing(self):
        ms, n = C.c_double(), C.c_uint64()
        check(lib().rl_agent_get_timing(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value


def comm_unique_id():
    """RCCL unique id (bytes) made on rank 0; hand it to every rank"""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    check(lib().rl_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """rl_comm: one RCCL communicator per process (one GPU per rank)"""

    def __init__(self, rank, world, uid, device=0):
        assert len(uid) == COMM_ID_BYTES
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().rl_comm_init(rank, world, buf, device, C.byref(h)))
        self.h = h
        self.rank, self.world = rank, world

    def allreduce(self, vals, op="sum"):
        """host values all-reduced over the ranks (RCCL): op sum / max / min"""
        x = np.ascontiguousarray(np.atleast_1d(vals), np.float64).copy()
        check(lib().rl_comm_allreduce_f64(self.h, x.ctypes.data, x.size, {"sum": 0, "max": 1, "min": 2}[op]))
        return x

    def barrier(self):
        check(lib().rl_comm_allreduce_f64(self.h, None, 0, 0))

    def close(self):
        if getattr(self, "h", None):
            lib().rl_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def kat_log(x, device=0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    check(lib().rl_kat_log(device, x.ctypes.data, out.ctypes.data, x.size))
    return out


def kat_rng(seed, lane, n, device=0):
    out = np.zeros(n, np.uint32)
    check(lib().rl_kat_rng(device, seed, lane, n, out.ctypes.data))
    return out


def kat_act(act, x, device=0):
    x = np.ascontiguousarray(x, dtype=np.float64)
    f, fp = np.zeros_like(x), np.zeros_like(x)
    check(lib().rl_kat_act(device, ACT[act], x.ctypes.data, f.ctypes.data, fp.ctypes.data, x.size))
    return f, fp


def net_features(p):
    """input-adapter features of every dense state (no GPU needed)"""
    S, _ = env_dims(p)
    c = env_config(p)
    n_in = 6 if p.get("net_input", "scalar") == "fl_obs" else 1
    out = np.zeros(S * n_in, np.float64)
    check(lib().rl_net_features(C.byref(c), INPUT[p.get("net_input", "scalar")], out.ctypes.data, out.size))
    return out.reshape(S, n_in)


def kat_ucb(q, ncount, t, c, device=0):
    q = np.ascontiguousarray(q, dtype=np.float64)
    ncount = np.ascontiguousarray(ncount, dtype=np.float64)
    t = np.ascontiguousarray(t, dtype=np.uint64)
    out = np.zeros_like(q)
    check(lib().rl_kat_ucb(device, q.ctypes.data, ncount.ctypes.data, t.ctypes.data, float(c),
                           out.ctypes.data, q.size))
    return out
