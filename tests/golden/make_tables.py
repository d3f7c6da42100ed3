"""Generate tests/golden/tables.json: an INDEPENDENT Python restatement of the
reference's environment constructors (third restatement, next to the C oracle
and the product's C++ host code), plus hand-derived known answers.

Sources restated (paths in the reference repo):
  FrozenLakeEnv::new      src/env/frozen_lake.rs:23-28 (maps), :30-102
  FrozenLakeEditedEnv::new src/env/frozen_lake_edited.rs:18-28 (terrain values), :94-218
  Network::fit            src/network.rs:61-80, src/network/layers.rs:75-141, loss.rs (net_kat)
  CliffWalkingEnv::new    src/env/cliff_walking.rs:9-58
  TaxiEnv::new            src/env/taxi.rs:22-31 (map, locs), :57-131
  utils::inc / from_2d_to_1d / categorical_sample   src/utils.rs:33-76
Run: python tests/golden/make_tables.py   (writes tables.json next to this file)
"""
import json
import os

FL_MAPS = {
    "4x4": ["SFFF", "FHFH", "FFFH", "HFFG"],
    "8x8": ["SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF", "FFFHFFFF", "FHHFFFHF", "FHFFHFHF",
            "FFFHFFFG"],
}
TAXI_MAP = ["+---------+", "|R: | : :G|", "| : | : : |", "| : : : : |", "| | : | : |",
            "|Y| : |B: |", "+---------+"]
TAXI_LOCS = [(0, 0), (0, 4), (4, 0), (4, 3)]


def inc(nrow, ncol, row, col, a):
    if a == 0:
        return row, max(col - 1, 0)
    if a == 1:
        return min(row + 1, nrow - 1), col
    if a == 2:
        return row, min(col + 1, ncol - 1)
    if a == 3:
        return max(row - 1, 0), col
    return row, col


def frozen_lake(name, slippery):
    m = FL_MAPS[name]
    n = len(m)
    S = n * n
    table = []  # [s][a] -> list of 3 (p, s', r, term)
    for s in range(S):
        row, col = divmod(s, n)
        per_a = []
        for a in range(4):
            outs = [(0.0, 0, 0.0, False)] * 3
            if m[row][col] in "GH":
                outs = [(1.0, s, 0.0, True)] + outs[1:]
            else:
                bs = [(a - 1) % 4, a, (a + 1) % 4] if slippery else [a]
                new = []
                for b in bs:
                    nr, nc = inc(n, n, row, col, b)
                    ch = m[nr][nc]
                    new.append(((1.0 / 3.0) if slippery else 1.0, nr * n + nc,
                                1.0 if ch == "G" else 0.0, ch in "GH"))
                outs = new + outs[len(new):]
            per_a.append(outs)
        table.append(per_a)
    cnt = sum(ch == "S" for r in m for ch in r)
    start = [(1.0 / cnt) if m[i // n][i % n] == "S" else 0.0 for i in range(S)]
    return table, start


WALL, HOLE, START, GROUND, GOAL = "WALL", "HOLE", "START", "GROUND", "GOAL"
TERRAIN_VALUE = {HOLE: -1.0, WALL: -0.5, START: 0.0, GROUND: 0.5, GOAL: 1.0}


def fle_terrain(m, row, col):
    """get_terrain (frozen_lake_edited.rs:146-162); off-map -> WALL"""
    if row < 0 or col < 0 or row >= len(m) or col >= len(m[0]):
        return WALL
    return {"S": START, "F": GROUND, "G": GOAL, "H": HOLE}[m[row][col]]


def fle_obs(m, row, col):
    """get_obs (:115-144): terrains left, down, right, up + (x, y) = (row, col)"""
    return [fle_terrain(m, row, col - 1), fle_terrain(m, row + 1, col), fle_terrain(m, row, col + 1),
            fle_terrain(m, row - 1, col), row, col]


def frozen_lake_edited(name, slippery):
    m = FL_MAPS[name]
    n = len(m)
    table = []
    for s in range(n * n):
        row, col = divmod(s, n)
        per_a = []
        for a in range(4):
            outs = [(0.0, 0, 0.0, False)] * 3
            if m[row][col] in "GH":
                outs = [(1.0, s, 0.0, True)] + outs[1:]
            else:
                bs = [(a - 1) % 4, a, (a + 1) % 4] if slippery else [a]
                new = []
                for b in bs:
                    nxt = fle_obs(m, row, col)[b]          # terrain in the moved direction
                    nr, nc = inc(n, n, row, col, b)
                    win = nxt == GOAL
                    new.append(((1.0 / 3.0) if slippery else 1.0, nr * n + nc, 10.0 if win else -1.0,
                                win or nxt == HOLE))
                outs = new + outs[len(new):]
            per_a.append(outs)
        table.append(per_a)
    cnt = sum(ch == "S" for r in m for ch in r)
    start = [(1.0 / cnt) if m[i // n][i % n] == "S" else 0.0 for i in range(n * n)]
    features = [[TERRAIN_VALUE[t] for t in fle_obs(m, *divmod(s, n))[:4]] + [float(s // n), float(s % n)]
                for s in range(n * n)]
    return table, start, features


def net_kat():
    """One Network::fit step of the neural bin's shape (DenseLayer(1,H) -> leaky_relu6 ->
    DenseLayer(H,4) -> linear, mse) on fixed weights, in plain Python floats (IEEE
    double, no FMA): sums over k in order from 0.0 (ndarray dot), Dense backward
    input_error with the old W, W -= lr * input^T err, b -= lr * err."""
    H, A, lr = 3, 4, 0.05
    W1 = [[0.25, -0.5, 0.125]]
    b1 = [0.1, -0.2, 0.0]
    W2 = [[0.5, -0.25, 0.75, 0.1], [-0.3, 0.2, 0.4, -0.6], [0.05, 0.15, -0.35, 0.45]]
    b2 = [0.0, 0.1, -0.1, 0.2]
    x = [3.0]

    def lrelu6(v):
        return min(max(v, 0.1 * v), 6.0)

    def lrelu6p(v):
        return 1.0 if 0.0 < v < 6.0 else 0.01

    def forward():
        z = [0.0 + x[0] * W1[0][j] + b1[j] for j in range(H)]
        h = [lrelu6(v) for v in z]
        o = []
        for i in range(A):
            acc = 0.0
            for j in range(H):
                acc = acc + h[j] * W2[j][i]
            o.append(acc + b2[i])
        return z, h, o

    z, h, y = forward()
    target = list(y)
    target[2] += -0.7                                     # curr_values[action] += td
    err = [(2.0 * (y[i] - target[i])) / A for i in range(A)]
    e2 = [1.0 * err[i] for i in range(A)]                 # linear_prime * err
    ie = []
    for j in range(H):
        acc = 0.0
        for i in range(A):
            acc = acc + e2[i] * W2[j][i]
        ie.append(acc)
    for j in range(H):
        for i in range(A):
            W2[j][i] = W2[j][i] - lr * (0.0 + h[j] * e2[i])
    b2 = [b2[i] - lr * e2[i] for i in range(A)]
    e1 = [lrelu6p(z[j]) * ie[j] for j in range(H)]
    for j in range(H):
        W1[0][j] = W1[0][j] - lr * (0.0 + x[0] * e1[j])
    b1 = [b1[j] - lr * e1[j] for j in range(H)]
    flat = lambda W1, b1, W2, b2: [v for r in W1 for v in r] + list(b1) + [v for r in W2 for v in r] + list(b2)
    w0 = flat([[0.25, -0.5, 0.125]], [0.1, -0.2, 0.0],
              [[0.5, -0.25, 0.75, 0.1], [-0.3, 0.2, 0.4, -0.6], [0.05, 0.15, -0.35, 0.45]], [0.0, 0.1, -0.1, 0.2])
    return {"hidden": H, "lr": lr, "x": x, "w": w0, "y": y, "target": target,
            "w_after": flat(W1, b1, W2, b2)}


def cliff_walking():
    table = []
    for s in range(48):
        row, col = divmod(s, 12)
        per_a = []
        for a in range(4):
            nr, nc = inc(4, 12, row, col, a)
            ns = nr * 12 + nc
            lose = 37 <= ns <= 46
            win = ns == 47
            per_a.append([(1.0, ns, -100.0 if lose else -1.0, lose or win)] + [(0.0, 0, 0.0, False)] * 2)
        table.append(per_a)
    start = [1.0 if i == 36 else 0.0 for i in range(48)]
    return table, start


def taxi_encode(r, c, p, d):
    return ((r * 5 + c) * 5 + p) * 4 + d


def taxi():
    table = [[None] * 6 for _ in range(500)]
    start = [0.0] * 500
    total = 0.0
    for r in range(5):
        for c in range(5):
            for p in range(5):
                for d in range(4):
                    s = taxi_encode(r, c, p, d)
                    if p < 4 and p != d:
                        start[s] += 1.0
                        total += 1.0
                    for a in range(6):
                        nr, nc, np_ = r, c, p
                        rew, term = -1.0, False
                        if a == 0:
                            nr = min(r + 1, 4)
                        elif a == 1:
                            nr = max(r - 1, 0)
                        if a == 2 and TAXI_MAP[1 + r][2 * c + 2] == ":":
                            nc = min(c + 1, 4)
                        elif a == 3 and TAXI_MAP[1 + r][2 * c] == ":":
                            nc = max(c - 1, 0)
                        elif a == 4:
                            if p < 4 and (r, c) == TAXI_LOCS[p]:
                                np_ = 4
                            else:
                                rew = -10.0
                        elif a == 5:
                            if (r, c) == TAXI_LOCS[d] and p == 4:
                                np_, term, rew = d, True, 20.0
                            else:
                                rew = -10.0
                        table[s][a] = [(1.0, taxi_encode(nr, nc, np_, d), rew, term)] + \
                                      [(0.0, 0, 0.0, False)] * 2
    start = [v / total for v in start]
    return table, start


def cumsum(xs):
    out, b = [], 0.0
    for x in xs:
        b += x
        out.append(b)
    return out


def eps_stall(n_episodes, eps0=1.0, exploration_time=0.5, final=0.0):
    """uniform_epsilon_greed.rs:42-49 with the bins' `a - decay` closure."""
    d = eps0 / (exploration_time * n_episodes)
    eps, k = eps0, 0
    while True:
        nw = eps - d
        if final > nw:
            return eps, k
        eps, k = nw, k + 1


def pack(table):
    return {"prob": [[[o[0] for o in outs] for outs in per_a] for per_a in table],
            "next": [[[o[1] for o in outs] for outs in per_a] for per_a in table],
            "reward": [[[o[2] for o in outs] for outs in per_a] for per_a in table],
            "term": [[[int(o[3]) for o in outs] for outs in per_a] for per_a in table]}


def main():
    out = {"source": "independent Python restatement of /root/reference src/env/*.rs (see docstring)"}
    for name in ("4x4", "8x8"):
        for slip in (0, 1):
            t, st = frozen_lake(name, slip)
            out[f"frozen_lake_{name}_{'slippery' if slip else 'det'}"] = dict(pack(t), start=st)
    for name in ("4x4", "8x8"):
        for slip in (0, 1):
            t, st, feat = frozen_lake_edited(name, slip)
            out[f"frozen_lake_edited_{name}_{'slippery' if slip else 'det'}"] = dict(pack(t), start=st,
                                                                                   fl_obs=feat)
    t, st = cliff_walking()
    out["cliff_walking"] = dict(pack(t), start=st)
    t, st = taxi()
    out["taxi"] = dict(pack(t), start=st)
    kat = {
        # hand-derived from the reference source (SURVEY §8c iii)
        "fl4x4_path": {"actions": [1, 1, 2, 2, 1, 2], "states": [4, 8, 9, 10, 14, 15],
                       "final_reward": 1.0},
        "cliff_path": {"actions": [3] + [2] * 11 + [1], "total_reward": -13.0, "final_state": 47},
        "cliff_fall": {"actions": [2], "state": 37, "reward": -100.0},
        "taxi_encode_4_3_4_2": taxi_encode(4, 3, 4, 2),
        "taxi_start_cumsum_last": cumsum(taxi()[1])[-1],
        "fl_slippery_cumsum": cumsum([1.0 / 3.0] * 3),
        "eps_stall": {str(n): list(eps_stall(n)) for n in (1000, 10000, 100000)},
        "ucb_first_inf_t": next(t for t in range(2, 200) if __import__("math").log(t) / 2.2250738585072014e-308 == float("inf")),
        "uniform_int_reject_6": (2**64 - 6) % 6,
        "uniform_card_reject": (2**32 - 10) % 10,
        "net_fit_leaky_relu6": net_kat(),
    }
    out["kat"] = kat
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, {k: v for k, v in kat.items() if k != "eps_stall"}, kat["eps_stall"])


if __name__ == "__main__":
    main()
