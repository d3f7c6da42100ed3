"""Plain-Python restatement of the reference's single-env training loop
(TEST INFRASTRUCTURE ONLY), written from the reference source, independently
of oracle/rlref.c, for FrozenLake + OneStepAgent + TabularPolicy with
eps-greedy or UCB selection:

  Agent::train / evaluate        src/agent.rs:66-141
  sarsa / qlearning / e. sarsa   src/agent.rs:19-45
  OneStepAgent get_action/update src/agent/one_step_agent.rs:48-86
  TabularPolicy (dict of rows)   src/policy/tabular_policy.rs:27-38
  UniformEpsilonGreed            src/action_selection/uniform_epsilon_greed.rs:42-80
  UpperConfidenceBound           src/action_selection/upper_confidence_bound.rs:29-63
  argmax / categorical_sample    src/utils.rs:1-43
  FrozenLakeEnv new/reset/step   src/env/frozen_lake.rs:48-134

thread_rng() is replaced, at the same draw sites, by the build's per-lane
xoshiro128+ stream, with rand 0.8.5's Uniform<f64> and
Uniform<usize> mappings; the stream skips the draws whose values the reference
never looks at (the one-'S' reset, a deterministic map's step, the low word of
a power-of-two Uniform<usize>), and draws the eps test's high word first.  Python floats are IEEE binary64 and the loop does
the reference's operations in the reference's order, so its results are the
reference arithmetic bit for bit; ln() is CPython's math.log (the platform
libm, like Rust's f64::ln).
"""
import math
import struct

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
MAP4 = ["SFFF", "FHFH", "FFFH", "HFFG"]
MAP8 = ["SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF", "FFFHFFFF", "FHHFFFHF", "FHFFHFHF", "FFFHFFFG"]
MIN_POSITIVE = 2.2250738585072014e-308


class Xoshiro128p:
    def __init__(self, seed, lane):
        x = (seed + lane * 0x632BE59BD9B4E019) & M64
        words = []
        for _ in range(2):
            x = (x + 0x9E3779B97F4A7C15) & M64
            z = x
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            z ^= z >> 31
            words += [z & M32, z >> 32]
        self.s = words if any(words) else [1, 0, 0, 0]

    def u32(self):
        s = self.s
        res = (s[0] + s[3]) & M32
        t = (s[1] << 9) & M32
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = ((s[3] << 11) | (s[3] >> 21)) & M32
        return res

    def u64(self):
        lo = self.u32()
        return lo | (self.u32() << 32)

    def uniform01(self):                          # rand UniformFloat<f64>, 0..1
        return struct.unpack("<d", struct.pack("<Q", (self.u64() >> 12) | 0x3FF0000000000000))[0] - 1.0

    def eps_test(self, eps):                      # u < eps, m's top 32 bits drawn first
        h = self.u32()
        e32 = math.ldexp(eps, 32)
        if h + 1.0 <= e32:
            return True
        if not h < e32:
            return False
        m = ((h << 32) | self.u32()) >> 12
        return struct.unpack("<d", struct.pack("<Q", m | 0x3FF0000000000000))[0] - 1.0 < eps

    def uniform_usize(self, n):                   # rand UniformInt<usize>::sample
        if n >= 2 and n & (n - 1) == 0:           # the top bits of the u64's high word only
            return self.u32() >> (32 - (n.bit_length() - 1))
        zone = M64 - ((1 << 64) - n) % n      # u64::MAX - (u64::MAX - range + 1) % range
        while True:
            m = self.u64() * n
            if (m & M64) <= zone:
                return m >> 64


def argmax(v):
    m, r = v[0], 0
    for i, x in enumerate(v):
        if x > m:
            m, r = x, i
    return r


def categorical_sample(probs, u):
    b = 0.0
    flags = []
    for p in probs:
        b += p
        flags.append(b > u)
    return argmax(flags)


class FrozenLake:
    def __init__(self, map8x8=False, slippery=False, max_steps=100):
        self.slippery = slippery
        m = MAP8 if map8x8 else MAP4
        n = len(m)
        self.n = n
        starts = [i for i, c in enumerate("".join(m)) if c == "S"]
        self.start = [0.0] * (n * n)
        for i in starts:
            self.start[i] = 1.0 / len(starts)

        def move(r, c, a):
            if a == 0:
                c = max(c - 1, 0)
            elif a == 1:
                r = min(r + 1, n - 1)
            elif a == 2:
                c = min(c + 1, n - 1)
            elif a == 3:
                r = max(r - 1, 0)
            letter = m[r][c]
            return r * n + c, 1.0 if letter == "G" else 0.0, letter in "GH"

        self.probs = []
        for r in range(n):
            for c in range(n):
                s = r * n + c
                row = []
                for a in range(4):
                    li = [(0.0, 0, 0.0, False)] * 3
                    if m[r][c] in "GH":
                        li[0] = (1.0, s, 0.0, True)
                    elif slippery:
                        li = [(1.0 / 3.0,) + move(r, c, b) for b in ((a - 1) % 4, a, (a + 1) % 4)]
                    else:
                        li[0] = (1.0,) + move(r, c, a)
                    row.append(li)
                self.probs.append(row)
        self.max_steps = max_steps
        self.ready = False
        self.pos = 0
        self.curr_step = 0

    def reset(self, rng):
        fixed = sum(1 for x in self.start if x != 0.0) == 1   # one 'S': the same state for every u
        self.pos = categorical_sample(self.start, 0.0 if fixed else rng.uniform01())
        self.ready = True
        self.curr_step = 0
        return self.pos

    def step(self, a, rng):
        if not self.ready:
            raise RuntimeError("EnvNotReady")
        if self.curr_step >= self.max_steps:
            self.ready = False
            return 0, 0.0, True
        self.curr_step += 1
        tr = self.probs[self.pos][a]
        i = categorical_sample([t[0] for t in tr], rng.uniform01()) if self.slippery else 0
        _, s, r, t = tr[i]
        self.pos = s
        if t:
            self.ready = False
        return s, r, t


class Agent:
    def __init__(self, rng, selector="eps_greedy", algo="qlearning", n_episodes=100000, lr=0.05, gamma=0.95,
                 eps0=1.0, exploration_time=0.5, eps_final=0.0, c=0.5, A=4):
        self.rng, self.sel, self.algo, self.A = rng, selector, algo, A
        self.lr, self.gamma, self.eps0, self.eps_final, self.c = lr, gamma, eps0, eps_final, c
        self.decay = eps0 / (exploration_time * n_episodes)      # src/bin/frozen_lake.rs:84,146
        self.q, self.counts, self.t, self.eps = {}, {}, 1, eps0

    def values(self, s):
        return list(self.q.get(s, [0.0] * self.A))

    def _ucbs(self, s, v):
        cnt = self.counts.setdefault(s, [0] * self.A)
        lnt = math.log(float(self.t))
        return cnt, [v[i] + self.c * math.sqrt(lnt / (float(cnt[i]) + MIN_POSITIVE)) for i in range(self.A)]

    def get_action(self, s):
        v = self.values(s)
        if self.sel == "eps_greedy":
            if self.eps != 0.0 and self.rng.eps_test(self.eps):
                return self.rng.uniform_usize(self.A)
            return argmax(v)
        cnt, u = self._ucbs(s, v)
        a = argmax(u)
        cnt[a] += 1
        self.t += 1
        return a

    def probs(self, s, v):
        if self.sel == "eps_greedy":
            p = [self.eps / float(self.A)] * self.A
            p[argmax(v)] = 1.0 - self.eps
            return p
        _, u = self._ucbs(s, v)
        total = 0.0
        for x in u:
            total += x
        return [x / total for x in u]

    def update(self, s, a, r, term, s2, a2):
        nq = self.values(s2)
        p = self.probs(s2, nq)
        if self.algo == "sarsa":
            f = nq[a2]
        elif self.algo == "qlearning":
            f = nq[0]
            for x in nq:
                if x > f:
                    f = x
        else:
            f = 0.0
            for i in range(self.A):
                f += p[i] * nq[i]
        td = r + self.gamma * f - self.values(s)[a]
        row = self.q.setdefault(s, [0.0] * self.A)
        row[a] += self.lr * td
        if term and self.sel == "eps_greedy":
            nw = self.eps - self.decay
            self.eps = self.eps if self.eps_final > nw else nw
        return td


def evaluate(agent, env, n):
    rewards, lengths = [], []
    for _ in range(n):
        k, er = 0, 0.0
        a = agent.get_action(env.reset(agent.rng))
        while True:
            k += 1
            s2, r, term = env.step(a, agent.rng)
            a = agent.get_action(s2)
            er += r
            if term:
                rewards.append(er)
                break
        lengths.append(k)
    return rewards, lengths


def train(agent, env, n, eval_at):
    rewards, lengths, errors = [], [], []
    for ep in range(n):
        k, er = 0, 0.0
        s = env.reset(agent.rng)
        a = agent.get_action(s)
        while True:
            k += 1
            s2, r, term = env.step(a, agent.rng)
            a2 = agent.get_action(s2)
            errors.append(agent.update(s, a, r, term, s2, a2))
            s, a = s2, a2
            er += r
            if term:
                rewards.append(er)
                break
        if ep % eval_at == 0:
            evaluate(agent, env, 100)
        lengths.append(k)
    return rewards, lengths, errors


def run(map8x8=False, slippery=False, selector="eps_greedy", algo="qlearning", n=2000, eval_at=200, seed=0x5EED,
        lane=0):
    """train(n, eval_at) on a fresh agent; returns (Q[S][A] list, rewards, lengths, errors)"""
    rng = Xoshiro128p(seed, lane)
    env = FrozenLake(map8x8, slippery)
    ag = Agent(rng, selector, algo, n_episodes=n)
    rh, el, te = train(ag, env, n, eval_at)
    q = [ag.values(s) for s in range(env.n * env.n)]
    return q, rh, el, te
