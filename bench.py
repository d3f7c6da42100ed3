#!/usr/bin/env python3
"""bench.py — training env-steps/s of the MI355X hot path.

Workload (BASELINE.json configs[1] = SURVEY §8(d) cfg 2): FrozenLake-8x8
(deterministic), one-step Q-learning, eps-greedy, 2^20 lanes per GPU, learner
groups of 512 lanes (one workgroup, Q in LDS), merge every K=64 synchronous
steps.  One bench "step" = one launch = K synchronous env-steps of every lane +
the merge (and, for N>1 GPUs, the ΔQ all-reduce over RCCL).  Defaults follow
§8(d): warm-up 64 synchronous steps (1 launch), timed window 4,096 (64 launches).
--config 3/4/5 selects the other §8(d) workloads (per-GPU lane counts); 6 and 7
the §8(f) rows on private agents: frozen_lake_neural's NeuralPolicy and
cliffwalking_model's Dyna-Q (InternalModelAgent, 10 planning steps); 8 is cfg 3's
Taxi + UCB with Q-learning, where Q stays finite (UCB's ln / sqrt / divide timed).

  python bench.py [--gpus N --steps K --warmup W]
  N>1: bench.py --gpus N starts its N ranks itself, or runs as one of them under
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
  At N>1 the default is the metric's fixed global lane set (strong scaling,
  GLOBAL_LANES: 2^20 for cfg 2); --lanes L gives weak scaling at L lanes per GPU.

No PyTorch: the stream, the kernel timing (HIP events, rl_agent_get_timing) and,
for N>1, the communicator all come from librlamd.
Multi-GPU: one process per GPU, lanes partitioned by global id; the merge buffer
is all-reduced by librlamd itself (rl_comm_* / rl_agent_set_comm: RCCL int64
all-reduces over xGMI, the path's only collectives).  Rank 0's RCCL id reaches the
other ranks through a file (one node); the barriers around the timed region and
the max time over ranks are RCCL all-reduces too (rl_comm_allreduce_f64).
RLAMD_COLLECTIVE=torch swaps in a torch all_reduce of the merge buffer (a
rehearsal mode for ranks sharing one GPU, where RCCL cannot run; it imports torch).

Prints ONE JSON line on rank 0.  `roofline` names the dominant kernel's binding
ceiling from the PMC counters of this very build (profiles/counters.json, matched
by rl_build_id), see roofline(); `cpu_baseline` times C restatements of the
reference loop on the host cores (bounded samples).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))

METRIC = "env-steps/sec, FrozenLake-8x8 Q-learning, 2^20 envs, 1/2/4/8 GPUs"
BYTES_PER_STEP = 32          # 16-B lane record read + written per env-step
HBM_PEAK = 8.0e12            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks, one process per GPU). Under a launcher (WORLD_SIZE set) it must equal "
                         "WORLD_SIZE; without one, N > 1 starts the N ranks itself (self_launch)")
    ap.add_argument("--child-timeout", type=float, default=1500.0,
                    help="self-launch: seconds before every rank is killed and the run fails")
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5, 6, 7, 8],
                    help="SURVEY §8(d) workload preset (2 = the headline)")
    ap.add_argument("--lanes", type=int, default=None, help="env lanes per GPU (weak scaling: per-GPU work fixed)")
    ap.add_argument("--lanes-total", type=int, default=None,
                    help="env lanes over all GPUs (strong scaling: lanes per GPU = total / N); the north "
                         "star's '2^20 parallel envs at 8xMI355X' is --lanes-total 1048576 --gpus 8")
    ap.add_argument("--group", type=int, default=None, help="learner-group size (lanes per workgroup)")
    ap.add_argument("--sync", type=int, default=64, help="K: synchronous steps per launch")
    for k in ("env", "agent", "policy", "selector", "algo"):
        ap.add_argument("--" + k, default=None)
    ap.add_argument("--map8x8", type=int, default=1)
    ap.add_argument("--reset-step", type=int, default=None,
                    help="batched schedule: resetting lanes also step in the same synchronous step "
                         "(rl_agent_set_reset_step; eps-greedy)")
    ap.add_argument("--slippery", type=int, default=0)
    ap.add_argument("--q-mode", default="auto", choices=["auto", "f64"],
                    help="shared-Q representation: the proven fixed point where it applies, or f64 always")
    # HIP events around EVERY launch cost 3 % of the headline's throughput (measured in
    # the driver's shape, --steps 20 --warmup 5: 3.19e11 with, 3.30e11 without; events
    # on every 4th launch 3.26e11): the kernel's average duration is sampled instead
    ap.add_argument("--timing-every", type=int, default=None,
                    help="HIP events around every N-th timed launch (the kernel's average duration; 0: none); "
                         "default 8, 1 for the private rows (a 100-ms launch hides the events' cost)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--counters-file", default=os.path.join(ROOT, "profiles", "counters.json"),
                    help="PMC summaries per workload (scripts/collect_counters.py)")
    a = ap.parse_args()
    a.user_lanes = a.lanes is not None
    for k, v in PRESETS[a.config].items():
        if k not in ("reset_step", "extra") and getattr(a, k) is None:
            setattr(a, k, v)
    a.extra = dict(PRESETS[a.config].get("extra", {}))
    if "map8x8" in a.extra:
        a.map8x8 = a.extra.pop("map8x8")
    if a.reset_step is None:
        a.reset_step = PRESETS[a.config].get("reset_step", 0)
    if a.timing_every is None:
        a.timing_every = 1 if a.group == 1 else 8
    return a


# SURVEY §8(d) workloads; lanes are per GPU (cfg 4: 2^19 over 4 GPUs, cfg 5: 2^22 over 8)
PRESETS = {
    2: dict(env="frozen_lake", agent="one_step", policy="tabular", selector="eps_greedy",
            algo="qlearning", lanes=1 << 20, group=512),
    3: dict(env="taxi", agent="one_step", policy="tabular", selector="ucb", algo="expected_sarsa",
            lanes=1 << 20, group=512),
    # cfg 4 / 5: the reset-and-step schedule (short episodes: a reset no longer costs
    # a synchronous step; measured 7.03e9 -> 7.25e9 and 5.94e10 -> 8.68e10; on cfg 2,
    # where 3 % of lane-steps are resets, the second selection costs more: 0.84x)
    4: dict(env="cliff_walking", agent="traces", policy="tabular", selector="eps_greedy", algo="sarsa",
            lanes=1 << 17, group=256, reset_step=1),
    5: dict(env="blackjack", agent="one_step", policy="double", selector="eps_greedy", algo="qlearning",
            lanes=1 << 19, group=512, reset_step=1),
    # §8(f) rows, private agents (one agent per lane):
    # src/bin/frozen_lake_neural.rs (FrozenLake 4x4, DenseLayer(1,32) -> leaky_relu6 ->
    # DenseLayer(32,4), eps <- eps * 0.5) and src/bin/cliffwalking_model.rs (Dyna-Q)
    6: dict(env="frozen_lake", agent="one_step", policy="neural", selector="eps_greedy", algo="qlearning",
            lanes=1 << 20, group=1, extra=dict(map8x8=0, decay_kind=1, eps_decay=0.5, net_input="scalar",
                                                net_hidden=32, net_act1="leaky_relu6", net_act2="linear")),
    7: dict(env="cliff_walking", agent="one_step", policy="tabular", selector="eps_greedy", algo="qlearning",
            lanes=1 << 20, group=1, extra=dict(planning=10)),
    # cfg 3's env and selector in a regime where Q stays finite:
    # UCB + Q-learning takes max(q') as its target (src/agent.rs:27-32), so the
    # selection's ln / sqrt / divide (upper_confidence_bound.rs:29-42) run on finite
    # rows at every step; one-step tabular with a contracting target: the proven
    # fixed point
    8: dict(env="taxi", agent="one_step", policy="tabular", selector="ucb", algo="qlearning",
            lanes=1 << 20, group=512),
}


# BASELINE.json's global lane count per workload ("2^20 envs, 1/2/4/8 GPUs"; cfg 4 "2^19 envs,
# 4xMI355X"; cfg 5 "2^22 envs across 8xMI355X"): at N > 1 ranks the default is strong scaling over
# this fixed set (each rank 1/N of it); --lanes L makes it weak scaling at L lanes per GPU
GLOBAL_LANES = {2: 1 << 20, 3: 1 << 20, 4: 1 << 19, 5: 1 << 22, 6: 1 << 20, 7: 1 << 20, 8: 1 << 20}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n, timeout):
    """`bench.py --gpus N` with no launcher: start N ranks of this same command (one
    process per GPU: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run
    sets them), relay rank 0's JSON line, and fail (non-zero) when any rank fails or
    the run outlives `timeout`.  This process never touches the GPU (it imports
    neither rlamd nor torch): the ranks are fresh children, not an exec."""
    import tempfile
    port = _free_port()
    procs, outs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = tempfile.TemporaryFile(mode="w+")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out, cwd=ROOT))
    t0, rc = time.time(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            print(f"bench.py: a rank exited with {rc}; stopping the others", file=sys.stderr)
            break
        if all(c == 0 for c in codes):
            break
        if time.time() - t0 > timeout:
            rc = 124
            print(f"bench.py: ranks still running after {timeout:.0f} s; stopping them", file=sys.stderr)
            break
        time.sleep(0.05)
    for p in procs:                       # the exact children started above, nothing else
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    texts = []
    for out in outs:
        out.seek(0)
        texts.append(out.read())
    for r, text in enumerate(texts[1:], 1):
        if text:
            sys.stderr.write(f"[rank {r} stdout]\n{text}")
    if rc == 0 and not any(l.startswith("{") for l in texts[0].splitlines()):
        print("bench.py: rank 0 printed no JSON line", file=sys.stderr)
        rc = 1
    (sys.stdout if rc == 0 else sys.stderr).write(texts[0])
    sys.stdout.flush()
    return 0 if rc == 0 else (rc if rc > 0 else 1)


def workload_key(args):
    return (f"cfg{args.config}" + ("_slippery" if args.slippery else "") +
            (f"_{args.q_mode}" if args.q_mode != "auto" else "") + (f"_L{args.lanes}" if args.lanes != PRESETS[
                args.config]["lanes"] else ""))


GLOBAL_Q = os.path.join(ROOT, "tests", "golden", "global_q.json")


def q_fixture(args, world):
    """The oracle's one-process result for this run's GLOBAL lane set, if committed
    (tests/golden/global_q.json, tests/golden/make_global_q.py): integer merges make
    Q identical for any rank count at a fixed global lane set, so the
    SHA-256 of the merged raw Q words is a known answer for an N-rank run."""
    try:
        tab = json.load(open(GLOBAL_Q))["cases"]
    except (OSError, ValueError, KeyError):
        return None
    want = {"env": args.env, "agent": args.agent, "policy": args.policy, "selector": args.selector,
            "algo": args.algo, "map8x8": args.map8x8, "slippery": args.slippery, "reset_step": int(args.reset_step),
            "q_mode": args.q_mode, "global_lanes": world * args.lanes, "group": args.group, "sync": args.sync,
            "launches": args.warmup + args.steps}
    for name, c in tab.items():
        if all(c["key"].get(k) == v for k, v in want.items()):
            return name, c
    return None


PRIVATE_Q = os.path.join(ROOT, "tests", "golden", "private_q.json")
PRIV_WINDOW = 4096


def private_q_check(args, agent):
    """Private rows: the last 4096 lanes' Q (cfg 6 also their
    network parameters), read alone (rl_agent_get_q_lanes), hashed and compared with
    the oracle's answer for exactly those lanes (tests/golden/private_q.json,
    tests/golden/make_private_q.py: private lanes are independent and keyed by global
    lane id, so the oracle runs only the window)"""
    import numpy as np
    L = args.lanes
    def f64_sha(x):       # NaN canonical (make_private_q.f64_sha)
        x = np.ascontiguousarray(x, "<f8")
        return hashlib.sha256(np.where(np.isnan(x), np.nan, x).astype("<f8").tobytes()).hexdigest()
    qh = f64_sha(agent.q_lanes(L - PRIV_WINDOW, PRIV_WINDOW))
    wh = f64_sha(agent.weights_lanes(L - PRIV_WINDOW, PRIV_WINDOW)) if args.policy == "neural" else None
    fx = None
    try:
        tab = json.load(open(PRIVATE_Q))["cases"]
        want = {"config": args.config, "global_lanes": L, "lane0": L - PRIV_WINDOW, "window": PRIV_WINDOW,
                "sync": args.sync, "launches": args.warmup + args.steps}
        fx = next(((n, c) for n, c in tab.items() if all(c["key"].get(k) == v for k, v in want.items())), None)
    except (OSError, ValueError, KeyError):
        pass
    return {"lanes": [L - PRIV_WINDOW, L], "q_sha256": qh, "w_sha256": wh, "launches": args.warmup + args.steps,
            "fixture": fx[0] if fx else None,
            "match": (fx[1]["q_sha256"] == qh and fx[1].get("w_sha256") == wh) if fx else None}


def counters_for(args, build_id):
    """PMC summary of the dominant kernel for this exact workload, collected from
    this very library (rl_build_id's source hash equal), or None"""
    try:
        tab = json.load(open(args.counters_file))
    except (OSError, ValueError):
        return None
    c = tab.get(workload_key(args))
    if not c:
        return None
    want = {"env": args.env, "algo": args.algo, "lanes": args.lanes, "group": args.group, "sync": args.sync,
            "slippery": args.slippery, "reset_step": args.reset_step, "q_mode": args.q_mode}
    if not all(c.get(k, "auto" if k == "q_mode" else None) == v for k, v in want.items()):
        return None
    src = (c.get("build_id") or "").split(" ")[0]
    return c if src and src == build_id.split(" ")[0] else None


def cpu_baseline(args):
    """SURVEY §8(d) CPU reference timing, on this host's cores, bounded samples.

    value  — "ref_faithful" (oracle/ref_faithful.c): the reference's single-env
             loop with its own data structures (FxHashMap Q / double-Q maps / trace
             map / UCB counters, per-step TD Vec push, ChaCha12 draws, eval
             interleave every n/10 episodes, Blackjack's fxhash observation ids),
             for THIS workload's env / agent / policy / selector / algorithm at the
             CLI defaults (n_episodes 1e5, src/bin/*.rs), 1 core; whole training
             runs repeated (train -> reset, as the bins' sweep) until the sample
             lasts about `cpu_seconds`.
    multi_core — the same, one independent env per thread, on every core the
             process may use (len(os.sched_getaffinity(0)), recorded in `cores`).
    cfg1   — SURVEY cfg 1: FrozenLake 4x4 one-step Q-learning eps-greedy, 1 core.
    ref_dense — the oracle's dense-array restatement of the same loop, 1 core.
    Every number is a C restatement of the reference loop, not the Rust binary
    (no Rust toolchain here: SURVEY §8(c))."""
    odir = os.path.join(ROOT, "oracle", "_build")
    rf, dense = os.path.join(odir, "ref_faithful"), os.path.join(odir, "rlref_bench")
    if not (os.path.exists(rf) and os.path.exists(dense)):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    envk = {"frozen_lake": 0, "cliff_walking": 1, "taxi": 2, "blackjack": 3}[args.env]
    agentk = {"one_step": 0, "traces": 1}[args.agent]
    polk = {"tabular": 0, "double": 1, "neural": 2}[args.policy]
    planning = args.extra.get("planning", 0)
    map8 = args.map8x8
    selk = {"eps_greedy": 0, "ucb": 1}[args.selector]
    algok = {"sarsa": 0, "qlearning": 1, "expected_sarsa": 2}[args.algo]
    n, eval_at = 100000, 10000          # the bins: train(env, n_episodes, n_episodes / 10)

    def run_rf(env, map8, agent, pol, sel, algo, reps, threads):
        out = subprocess.run([rf, str(env), str(map8), str(args.slippery), str(agent), str(pol), str(sel), str(algo),
                              str(n), str(eval_at), str(reps), str(threads)],
                             check=True, capture_output=True, text=True).stdout
        return json.loads(out)

    def run_dense(reps, threads):
        out = subprocess.run([dense, str(envk), str(map8), str(args.slippery), str(agentk), str(polk),
                              str(selk), str(algok), str(n), str(eval_at), str(threads), str(reps), str(planning)],
                             check=True, capture_output=True, text=True).stdout
        return json.loads(out)

    def sized(fn, target):
        reps, r = 1, fn(1)
        while r["seconds"] < 0.6 * target and reps < 1 << 20:
            reps = max(reps + 1, int(reps * min(8.0, target / max(r["seconds"], 1e-3))))
            r = fn(reps)
        return reps, r

    def line(kind, what, reps, r, threads):
        return {"value": r["steps_per_sec"], "unit": "env-steps/s", "cores": threads, "kind": "port",
                "sample": f"{what}: {reps} x train({n} episodes, eval every {eval_at}) per core = "
                          f"{r['steps']} training env-steps in {r['seconds']:.2f} s"}

    # every core this process may run on (the box's share: sched_getaffinity, not
    # os.cpu_count(), which counts the whole machine)
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    desc = (f"{args.env}{' 8x8' if map8 and args.env == 'frozen_lake' else ''}"
            f"{' slippery' if args.slippery else ''} {args.agent} {args.policy} {args.algo} {args.selector}"
            f"{f' + Dyna {planning} planning steps' if planning else ''}")
    mine = (envk, map8, agentk, polk, selk, algok)
    if polk == 2 or planning:
        # NeuralPolicy / InternalModelAgent: ref_faithful.c does not restate them, so
        # the oracle's faithful loop (rlref.c rlo_faithful, bit-exact with the device
        # in these rows, tests/test_gpu_parity.py) is the baseline
        n = 10000 if polk == 2 else 2000
        eval_at = n // 10
        repd, d = sized(lambda k: run_dense(k, 1), args.cpu_seconds)
        res = line("port", f"ref_dense (oracle/rlref.c rlo_faithful) {desc}", repd, d, 1)
        reps_m, m = sized(lambda k: run_dense(k, threads), args.cpu_seconds / 2)
        res["multi_core"] = line("port", f"{threads} independent rlo_faithful loops (len(os.sched_getaffinity(0)))",
                                 reps_m, m, threads)
        res["host_threads_machine"] = os.cpu_count()
        return res
    reps, r = sized(lambda k: run_rf(*mine, k, 1), args.cpu_seconds)
    res = line("port", f"ref_faithful (oracle/ref_faithful.c: FxHashMap tables, ChaCha12, Vec histories) {desc}",
               reps, r, 1)
    reps_m, m = sized(lambda k: run_rf(*mine, k, threads), args.cpu_seconds / 2)
    res["multi_core"] = line("port", f"{threads} independent ref_faithful envs (len(os.sched_getaffinity(0)))",
                             reps_m, m, threads)
    reps1, c1 = sized(lambda k: run_rf(0, 0, 0, 0, 0, 1, k, 1), args.cpu_seconds / 4)
    res["cfg1"] = line("port", "SURVEY cfg 1: ref_faithful FrozenLake 4x4 one-step Q-learning eps-greedy",
                       reps1, c1, 1)
    repd, d = sized(lambda k: run_dense(k, 1), args.cpu_seconds / 4)
    res["ref_dense"] = line("port", f"ref_dense (oracle/rlref.c rlo_faithful: dense-array Q) {desc}", repd, d, 1)
    res["host_threads_machine"] = os.cpu_count()
    return res


def roofline(args, agent, steps_done, avg_kern_s, pmc):
    """The dominant kernel against its binding ceiling.

    Counters (profiles/counters.json) are attached only when they were collected
    from this very library (rl_build_id equal), else `counters` is null.  With
    them: the VALU pipe occupancy of the gfx950 model (2 cycles per wave64 VALU
    instruction, +2 for an f64 / int64 one, +6 for an f64 transcendental;
    MI355X_MICROARCH.md) against 1.0, and `bound` "latency" when waves wait more
    than 40 % of their cycles while the pipe is below 70 %,
    "valu" when the pipe is the closer ceiling, else "hbm".  The HBM side is
    reported as measured traffic (PMC) and as the fused kernel's algorithmic bytes
    (every lane record read and written once per launch), both <= 1 of the peak;
    when the measured traffic is the nearer ceiling (the private agents' own tables
    and weights in HBM) `frac` is the HBM fraction (`ceiling`: "hbm").
    SURVEY §8(d)'s 32 B/env-step price assumes a lane-record round trip per step,
    which the fused kernel does not make; it is kept under `hbm_priced` as a ratio,
    not a fraction."""
    n_act = {"frozen_lake": 4, "cliff_walking": 4, "taxi": 6, "blackjack": 2}[args.env]
    st = agent.stats()
    v_bar = st["trace_states"] / max(st["train_steps"], 1) if args.agent == "traces" else 0.0
    bytes_per_step = BYTES_PER_STEP + (16 * n_act + 2) * v_bar
    priced = bytes_per_step * steps_done / args.steps / avg_kern_s
    # fused kernel: core + rng + aux (16 B each) + episode reward (8 B), read and
    # written once per launch; f64 tables: the group's final Q into its slot
    lanes = args.lanes
    groups = (lanes + args.group - 1) // args.group
    rows = 484 if (args.env == "blackjack" and args.selector != "ucb") else agent.S   # LDS rows per group
    slot_bytes = 8 * agent.P * rows * agent.A * groups if agent.q_repr() == "f64" else 0
    fused_bytes = 2 * 56 * lanes + slot_bytes
    # traces (shared): the lanes' eligibility-trace sets outlive a launch as the lane
    # records do — read in and written out once per launch: 10 B per visited pair
    # (u16 id + f64 E; the whole-row layout of UCB + expected SARSA: A x 8 B + a
    # 2 B list entry per visited state); their count at the run's end
    # (rl_agent_trace_items) stands for the launch boundaries'
    trace_items = agent.trace_items() if (args.agent == "traces" and args.group != 1) else 0
    if trace_items:
        pairs = not (args.selector == "ucb" and args.algo == "expected_sarsa")
        fused_bytes += 2 * (10 if pairs else 8 * n_act + 2) * trace_items
    kname = "k_train_private" if args.group == 1 else "k_train_shared"
    basis_priv = ("private agents: 2 x 56 B lane record per lane per launch + per env-step the lane's own "
                  "table traffic (tabular: row s2, Q(s,a) read + written, x (1 + planning steps); neural: "
                  "weights read by two predicts and read + written by the fit)")
    if args.group == 1:
        # private agents: which kernel the library launches (rl_host.cpp
        # agent_select_kernel): the bin's network on FrozenLake one-step agents holds
        # its parameters in registers (k_train_private_net), small tables hold Q in
        # LDS (k_train_private_lds) — each moves its parameters / tables once in and
        # once out per launch; otherwise per env-step the TD reads row s2 and Q(s, a)
        # and writes Q(s, a) (tabular, + the same per Dyna planning step), or the two
        # predicts read the weights and the fit reads + writes them (NeuralPolicy)
        planning = args.extra.get("planning", 0)
        psa8 = 8 * agent.P * agent.S * agent.A
        if args.policy == "neural":
            n_in, hid, npar = agent.net_dims()
            if (args.env == "frozen_lake" and args.agent == "one_step" and n_in == 1 and hid == 32
                    and args.extra.get("net_act1", "leaky_relu6") == "leaky_relu6"
                    and args.extra.get("net_act2", "linear") == "linear"):
                kname = "k_train_private_net"
                fused_bytes = 2 * 56 * lanes + 2 * 8 * npar * lanes
                basis_priv = ("k_train_private_net: 2 x 56 B lane record + the lane's parameters read once and "
                              "written once per launch (held in registers for the K steps)")
            else:
                fused_bytes = 2 * 56 * lanes + 4 * 8 * npar * steps_done / args.steps
        elif args.env in ("frozen_lake", "cliff_walking", "frozen_lake_edited") and psa8 <= 4096:
            kname = "k_train_private_lds"
            # + one 16-byte model record per Dyna planning step
            fused_bytes = 2 * 56 * lanes + 2 * psa8 * lanes + 16 * planning * steps_done / args.steps
            basis_priv = ("k_train_private_lds: 2 x 56 B lane record + the lane's Q table read once and written "
                          "once per launch (held in LDS for the K steps) + a 16 B model record per Dyna "
                          "planning step")
        else:
            per_step = 8 * (n_act + 2) * (1 + planning)
            fused_bytes = 2 * 56 * lanes + per_step * steps_done / args.steps
    fused_frac = fused_bytes / avg_kern_s / HBM_PEAK
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    traffic_frac = (traffic / avg_kern_s / HBM_PEAK) if traffic else None
    pipe = pmc.get("valu_pipe_frac") if pmc else None
    wait = (pmc.get("wave_cycle_split") or {}).get("SQ_WAIT_ANY") if pmc else None
    out = {"kernel": kname, "kernel_avg_ms": avg_kern_s * 1e3,
           "hbm": {"fused_bytes_per_launch": fused_bytes, "fused_frac": fused_frac,
                   "fused_basis": ("2 x 56 B lane record per lane per launch (+ 8 B x LDS entries per group "
                                   "for f64 tables; traces: + 2 x 10 B per live trace pair, in and out once): the "
                                   "fused kernel keeps lanes in registers for K steps")
                   if args.group != 1 else basis_priv,
                   **({"trace_items": trace_items} if trace_items else {}),
                   "traffic_bytes_per_launch": traffic, "traffic_frac": traffic_frac,
                   "traffic_over_fused": (traffic / fused_bytes) if traffic else None,
                   "peak_GBps": HBM_PEAK / 1e9},
           "hbm_priced": {"bytes_per_env_step": bytes_per_step, "GBps_equiv": priced / 1e9,
                          "ratio_to_peak": priced / HBM_PEAK,
                          "basis": "SURVEY 8(d): 32 B/env-step (+ (16A+2) V-bar for traces) x env-steps per "
                                   "launch / kernel time; a price, not traffic (ratio may exceed 1)"},
           **({"trace_v_bar": v_bar} if args.agent == "traces" else {}),
           "counters": pmc.get("source") if pmc else None,
           "counters_build": pmc.get("build_id") if pmc else None}
    if pipe is not None:
        # the ceiling: whichever of the VALU pipe and HBM the kernel runs closer to
        ceiling = "hbm" if traffic_frac is not None and traffic_frac > pipe else "valu"
        top = traffic_frac if ceiling == "hbm" else pipe
        bound = "latency" if (wait is not None and wait > 0.4 and top < 0.7) else ceiling
        basis = ("'latency': SQ_WAIT_ANY > 0.4 of wave cycles with both the VALU pipe and HBM below 0.7 of "
                 "their peaks; frac is the nearer ceiling's (`ceiling`)")
        if ceiling == "hbm":
            out.update(bound=bound, ceiling="hbm", achieved=traffic / avg_kern_s / 1e9, peak=HBM_PEAK / 1e9,
                       unit="GB/s", frac=traffic_frac, traffic=traffic, wait_frac=wait, valu_pipe_frac=pipe,
                       basis="measured HBM bytes (PMC FETCH_SIZE x 2 + WRITE_SIZE) / kernel time; " + basis)
        else:
            out.update(bound=bound, ceiling="valu", achieved=pipe, peak=1.0, unit="VALU pipe occupancy (gfx950 model)",
                       frac=pipe, traffic=traffic, wait_frac=wait,
                       basis="(2 x SQ_INSTS_VALU + 2 x (f64 add/mul/fma + int64) + 6 x f64 trans) cycles / "
                             "(cycles x 1024 SIMDs); " + basis)
    else:
        out.update(bound="hbm", achieved=fused_bytes / avg_kern_s / 1e9, peak=HBM_PEAK / 1e9, unit="GB/s",
                   frac=fused_frac, traffic=None,
                   basis="no counters from this build: the fused kernel's algorithmic bytes (hbm.fused_basis)")
    return out


def collective_name(collective, merge_path):
    if collective == "torch":
        return "torch all_reduce (rehearsal)"
    how = {"peer": "one-shot peer-read reduce of the merge buffer over IPC-mapped exchange regions (librlamd)",
           "rccl": "rccl int64 all-reduces of the merge buffer (librlamd)",
           "local": "none (one rank)"}[merge_path]
    return how + ("; rccl control plane" if collective == "rccl" else "; gloo control plane")


def rccl_bootstrap(rank, world, dev):
    """RCCL communicator without a torch control plane: rank 0's unique id is handed
    to the other ranks through a file (one node: every rank shares /tmp), keyed by
    the launcher's pid and MASTER_PORT so concurrent jobs never mix."""
    import rlamd
    path = f"/tmp/rlamd_commid_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
    if rank == 0:
        uid = rlamd.comm_unique_id()
        with open(path + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(path + ".tmp", path)
    else:
        t0 = time.time()
        while not os.path.exists(path):
            if time.time() - t0 > 300:
                raise RuntimeError(f"rank {rank}: no RCCL id from rank 0 at {path}")
            time.sleep(0.01)
        uid = open(path, "rb").read()
    comm = rlamd.Comm(rank, world, uid, dev)     # collective: every rank has read the id
    comm.barrier()
    if rank == 0:
        os.remove(path)
    return comm


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(self_launch(args.gpus, args.child_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    if world > 1 and args.lanes_total is None and not args.user_lanes:
        # the metric's fixed global lane set (BASELINE.json: "2^20 envs, 1/2/4/8 GPUs")
        args.lanes_total = GLOBAL_LANES[args.config]
    # RLAMD_FORCE_COMM=1 (tests): take the multi-GPU code path (librlamd's RCCL
    # communicator attached) even with one rank
    dist_on = world > 1 or os.environ.get("RLAMD_FORCE_COMM") == "1"
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    scaling = "weak"
    if args.lanes_total is not None:     # strong scaling: the global lane set is fixed
        if args.lanes_total % world or (args.lanes_total // world) % args.group:
            raise SystemExit(f"--lanes-total {args.lanes_total}: not {world} equal shards of whole "
                             f"learner groups of {args.group}")
        args.lanes = args.lanes_total // world
        scaling = "strong"
    # collective "rccl" (default): librlamd's own communicator — the merges by the
    # peer-read reduce (or RCCL all-reduces), the barriers and the max-over-ranks
    # time by RCCL — no PyTorch anywhere.  "peer": the peer-read merge with a gloo
    # control plane, for ranks sharing one GPU (RCCL refuses them).  "torch": a
    # torch.distributed all_reduce of the merge buffer, the same rehearsal.
    collective = os.environ.get("RLAMD_COLLECTIVE", "rccl")
    torch = dist = None
    if dist_on and collective != "rccl":
        import torch
        import torch.distributed as dist
        dev = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        dist.init_process_group(os.environ.get("RLAMD_DIST_BACKEND", "gloo"))
    else:
        dev = local_rank
    import rlamd

    kw = dict(env=args.env, map8x8=args.map8x8, slippery=args.slippery,
              agent=args.agent, policy=args.policy, selector=args.selector,
              algo=args.algo, n_lanes=args.lanes, group_size=args.group,
              sync_every=args.sync, lane_offset=rank * args.lanes, device=dev)
    kw.update({k: v for k, v in args.extra.items() if k != "planning"})
    p = rlamd.default_params(**kw)
    agent = rlamd.Agent(p)
    if args.extra.get("planning"):
        agent.set_planning(args.extra["planning"])
    if args.reset_step:
        agent.set_reset_step(True)
    if args.q_mode != "auto":
        agent.set_q_mode(args.q_mode)
    occ = agent.occupancy()   # resident learner groups per CU (LDS / VGPR limited)
    delta, comm = None, None
    if dist_on and collective == "rccl":
        comm = rccl_bootstrap(rank, world, dev)
        # every merge: the one-shot peer-read reduce over xGMI (rl.h ABI 7, set up by
        # set_comm at world > 1 after a self-test agreed by every rank), or RCCL
        # all-reduces (RLAMD_MERGE=rccl, or when the self-test fails); then apply
        agent.set_comm(comm)
    elif dist_on and collective == "peer":
        # ranks sharing one GPU (RCCL refuses them): the peer-read merge with the
        # exchange regions' handles all-gathered over gloo, the control plane gloo
        hs = [None] * world
        dist.all_gather_object(hs, agent.peer_handle())
        agent.peer_attach(rank, world, hs)
        agent.set_merge_groups(world * ((args.lanes + args.group - 1) // args.group))
    elif dist_on:
        # rehearsal: torch's HIP runtime (its wheel's own) and librlamd's are not one
        # runtime, so their streams do not order each other: every hand-over below is
        # an explicit synchronize on both sides
        delta = torch.zeros(agent.delta_words(), dtype=torch.int64, device=f"cuda:{dev}")
        torch.cuda.synchronize()
        agent.set_delta_buffer(delta.data_ptr(), delta.numel())
        agent.set_merge_groups(world * ((args.lanes + args.group - 1) // args.group))
    mw = agent.delta_max_words()
    merge_path = agent.merge_path() if delta is None else "torch"

    def step():
        if delta is None:                   # launch + merge (librlamd: RCCL all-reduces when world > 1)
            agent.run(1)
            return
        agent.launch_train()                # rehearsal: torch all_reduces of the merge buffer
        agent.synchronize()
        dist.all_reduce(delta[:mw], op=dist.ReduceOp.MAX)
        torch.cuda.synchronize()
        agent.launch_fold()
        agent.synchronize()
        dist.all_reduce(delta[mw:])
        torch.cuda.synchronize()
        agent.launch_apply()

    def barrier():
        agent.synchronize()
        if comm is not None:
            comm.barrier()
        elif dist is not None:
            dist.barrier()
        agent.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    st0 = agent.stats()
    every = max(args.timing_every, 0)       # HIP events around the train kernels, on its stream
    t0 = time.perf_counter()
    for i in range(args.steps):
        if every:
            agent.set_timing(i % every == 0)
        step()
    barrier()
    wall = time.perf_counter() - t0
    agent.set_timing(False)
    kern_ms, n_kern = agent.timing()
    st1 = agent.stats()
    # every Env::step inside train (truncation included) counted on the device;
    # RESET steps (env.reset + first get_action) are not env steps
    steps_done = st1["train_steps"] - st0["train_steps"]
    assert 0 < steps_done <= args.steps * args.sync * args.lanes, steps_done
    if comm is not None:                  # control plane over RCCL (librlamd)
        wall = float(comm.allreduce([wall], "max")[0])
        total_steps = int(comm.allreduce([float(steps_done)], "sum")[0])
    elif dist is not None:                # rehearsal: gloo, host tensors
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        ts = torch.tensor([steps_done], dtype=torch.int64)
        dist.all_reduce(ts)
        total_steps = int(ts.item())
    else:
        total_steps = steps_done
    value = total_steps / wall
    avg_kern_s = kern_ms / n_kern / 1e3 if n_kern else wall / args.steps
    # the merged Q after the run (untimed): SHA-256 of its raw int64 words, every
    # rank's digest compared, and the committed one-process answer for this global
    # lane set when there is one (a self-checking N-rank run)
    q_check = None
    if args.group != 1:
        qh = hashlib.sha256(agent.q_raw().astype("<i8").tobytes()).hexdigest()
        agree = True
        if comm is not None:              # 48 bits of the digest are exact in an f64
            h48 = float(int(qh[:12], 16))
            agree = bool(comm.allreduce([h48], "max")[0] == comm.allreduce([h48], "min")[0])
        elif dist is not None:
            t = torch.tensor([int(qh[:12], 16)], dtype=torch.int64)
            t2 = t.clone()
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(t2, op=dist.ReduceOp.MIN)
            agree = bool(t.item() == t2.item())
        fx = q_fixture(args, world)
        st_all = st1["train_steps"]
        if comm is not None:
            st_all = int(comm.allreduce([float(st_all)], "sum")[0])
        elif dist is not None:
            ts = torch.tensor([st_all], dtype=torch.int64)
            dist.all_reduce(ts)
            st_all = int(ts.item())
        q_check = {"q_sha256": qh, "ranks_agree": agree, "launches": args.warmup + args.steps,
                   "global_lanes": world * args.lanes, "train_steps_all_ranks": st_all,
                   "fixture": fx[0] if fx else None,
                   "match": (fx[1]["q_sha256"] == qh and fx[1]["train_steps"] == st_all) if fx else None}
    elif world == 1 and args.lanes >= PRIV_WINDOW:
        q_check = private_q_check(args, agent)
    bid = rlamd.build_id()
    pmc = counters_for(args, bid)
    q_repr = agent.q_repr()
    out = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": ("f64 TD arithmetic; shared Q int64 fixed point 2^-40 (range proven, |Q| <= 2048, no clamp)"
                  if q_repr == "fixed40" else f"f64 TD arithmetic; shared Q f64 ({q_repr}: the reference's full range)"),
        "data": "synthetic (env lanes seeded per global lane id; no dataset)",
        "config": {"workload": f"run mode (rl_agent_run: lanes train continuously, eval interleave off) "
                               f"{args.env}{(' 8x8' if args.map8x8 else ' 4x4') if args.env == 'frozen_lake' else ''}"
                               f"{' slippery' if args.slippery else ''} {args.agent} {args.policy} "
                               f"{args.algo} {args.selector}, {args.lanes} lanes/GPU"
                               f"{f' ({world * args.lanes} in total, fixed)' if scaling == 'strong' else ''}",
                   "survey_cfg": args.config,
                   "schedule": "reset-and-step" if args.reset_step else "one action per synchronous step",
                   "lanes_per_gpu": args.lanes, "lanes_total": world * args.lanes,
                   "group_size": args.group, "sync_every": args.sync,
                   "env_steps_per_launch": steps_done / args.steps,
                   "sync_steps_per_launch": args.sync, "parallelism": f"dp{world}",
                   "collective": collective_name(collective, merge_path) if dist_on else "none",
                   "merge_path": merge_path,
                   "groups_per_cu": occ["groups_per_cu"], "lds_bytes_per_group": occ["lds_bytes"],
                   "q_repr": q_repr, "q_mode": args.q_mode},
        "q_check": q_check,
        "build": rlamd.lib().rl_build_info().decode(),
        "build_id": bid,
        "roofline": roofline(args, agent, steps_done, avg_kern_s, pmc),
        "timing": {"wall_s": wall, "kernel_launches_timed": n_kern,
                   "kernel_ms_total": kern_ms, "host": "time.perf_counter between barriers; kernels: HIP "
                                                       "events on the agent's stream (rl_agent_get_timing) around "
                                                       f"every {args.timing_every}-th timed launch"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    agent.close()
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
