"""N>1 rehearsal on the one-GPU box (gloo, 2 ranks sharing the device).

The driver runs bench.py at N = 2/4/8 over RCCL (librlamd's rl_comm) on a whole node; these tests
exercise the same per-rank code path on real hardware:
  - the per-rank merge (launch_train -> all_reduce MAX -> launch_fold ->
    all_reduce SUM -> launch_apply) gives raw Q / UCB counters bit-identical to
    one process holding every lane, in both Q representations (the fixed point
    for FrozenLake Q-learning, f64 for the rest);
  - `python -m torch.distributed.run ... bench.py --gpus 2` prints one valid
    JSON line on rank 0 (whole-job value, max-over-ranks wall time).
Both run as child processes launched before this process touches the GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _torchrun(args, n=2, timeout=240):
    # two ranks share the one GPU, so the merge goes through torch's all_reduce
    # (bench.py RLAMD_COLLECTIVE=torch); RCCL itself is exercised by test_gpu_rccl.py
    env = dict(os.environ, RLAMD_DIST_BACKEND="gloo", RLAMD_COLLECTIVE="torch", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


CASES = {
    "fl8x8-qlearning": dict(env="frozen_lake", map8x8=1, algo="qlearning", group_size=256),
    "taxi-ucb-esarsa": dict(env="taxi", selector="ucb", algo="expected_sarsa", group_size=512),
    "cliff-traces-sarsa": dict(env="cliff_walking", agent="traces", algo="sarsa", group_size=256),
    "blackjack-double-q": dict(env="blackjack", policy="double", algo="qlearning", group_size=512),
    # UCB in the fixed point (cfg 8's regime): the fused peer merge also sums and
    # applies the visit counts N and t
    "taxi-ucb-qlearning": dict(env="taxi", selector="ucb", algo="qlearning", group_size=256),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_two_rank_device_merge_equals_one_process(tmp_path, name):
    case = dict(CASES[name], sync_every=32, n_launch=4, lanes_per_rank=8192)
    out = tmp_path / "res.json"
    r = _torchrun([os.path.join("tests", "dist_gpu_worker.py"), str(out), json.dumps(case)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert res["steps_ranks"] == res["steps_one"] > 0, res
    assert res["q_nonzero"] + res["q_nonfinite"] > 0, res   # UCB+E-SARSA: all-NaN/inf is legal (F7)
    assert res["q_equal"] and res["qf_equal"], res
    assert res["q_repr"][0] == res["q_repr"][1] == (
        "fixed40" if name in ("fl8x8-qlearning", "taxi-ucb-qlearning") else "f64"), res
    if "ucb_equal" in res:
        assert res["ucb_equal"], res


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_two_rank_peer_merge_equals_one_process(tmp_path, name):
    """VERDICT r05 item 2 / SURVEY §8(e): the one-shot peer-read merge (rl.h ABI 7:
    IPC-exported exchange regions, epoch flags, one kernel reading both ranks' words
    in rank order) — two processes sharing the GPU — ends every merge of run() and
    of train() (its control word too) with the raw Q, UCB counters and step counts of
    ONE process holding all lanes, in both representations"""
    case = dict(CASES[name], sync_every=32, n_launch=4, lanes_per_rank=8192, merge="peer", train_episodes=3)
    out = tmp_path / "res.json"
    r = _torchrun([os.path.join("tests", "dist_gpu_worker.py"), str(out), json.dumps(case)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert res["merge_path"] == "peer", res
    assert res["steps_ranks"] == res["steps_one"] > 0, res
    assert res["q_nonzero"] + res["q_nonfinite"] > 0, res
    assert res["q_equal"] and res["qf_equal"], res
    assert res["q_repr"][0] == res["q_repr"][1] == (
        "fixed40" if name in ("fl8x8-qlearning", "taxi-ucb-qlearning") else "f64"), res
    if "ucb_equal" in res:
        assert res["ucb_equal"], res


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_four_rank_peer_merge_equals_one_process(tmp_path, name):
    """The peer-read merge with four ranks (four processes sharing the GPU): every
    rank waits for three peers' flags and sums four regions in rank order — the
    N > 2 logic the driver's 8-GPU runs take — and still ends with one process's Q"""
    case = dict(CASES[name], sync_every=32, n_launch=3, lanes_per_rank=4096, merge="peer", train_episodes=2)
    out = tmp_path / "res.json"
    r = _torchrun([os.path.join("tests", "dist_gpu_worker.py"), str(out), json.dumps(case)], n=4, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert res["merge_path"] == "peer", res
    assert res["steps_ranks"] == res["steps_one"] > 0, res
    assert res["q_equal"] and res["qf_equal"], res
    if "ucb_equal" in res:
        assert res["ucb_equal"], res


@pytest.mark.gpu
def test_bench_two_ranks_prints_one_line():
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "4", "--warmup", "1", "--lanes", str(1 << 16),
                   "--no-cpu-baseline"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["scaling"] == "weak"
    # whole-job value: both ranks' env-steps over the max-over-ranks wall time
    assert d["value"] > 0 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["env_steps_per_launch"] <= 64 * (1 << 16)


@pytest.mark.gpu
def test_bench_rccl_path_one_rank():
    """bench.py's multi-GPU code path with librlamd's own RCCL merge (the one the
    driver's N = 2/4/8 runs take: gloo bootstrap of the RCCL id, rl_comm_init,
    rl_agent_set_comm, the all-reduce inside every launch), run with one rank —
    the box has one GPU and RCCL refuses two ranks on one device."""
    env = dict(os.environ, RLAMD_FORCE_COMM="1", MASTER_ADDR="127.0.0.1")
    env.pop("RLAMD_COLLECTIVE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--steps", "3",
           "--warmup", "1", "--lanes", str(1 << 16), "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["config"]["collective"].startswith("rccl") and d["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("extra,fixture,scaling", [(["--lanes", str(1 << 20)], "cfg2_L2M_25", "weak"),
                                                    ([], "cfg2_L1M_25", "strong")],
                         ids=["weak-2x2^20", "strong-2^20-default"])
def test_bench_two_ranks_q_check_matches_one_process(extra, fixture, scaling):
    """a 2-rank bench run in the driver's shape (--steps 20
    --warmup 5) ends with the merged Q of ONE process over its global lane set:
    every rank holds the same digest and it equals the oracle's for that set
    (tests/golden/global_q.json) — weak (--lanes: 2 x 2^20 lanes) and the
    default at N > 1, the metric's fixed 2^20 lanes split over the ranks (strong)"""
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--no-cpu-baseline"] + extra)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    qc = d["q_check"]
    assert d["scaling"] == scaling and qc["global_lanes"] == (2 << 20 if scaling == "weak" else 1 << 20)
    assert qc["ranks_agree"] is True and qc["fixture"] == fixture and qc["match"] is True, json.dumps(qc)


@pytest.mark.gpu
def test_bench_gpus2_self_launch_strong_default():
    """`bench.py --gpus 2` with NO launcher starts its two ranks
    itself and, by default, splits BASELINE's fixed 2^20 lanes over them (strong
    scaling): one JSON line, n_gpus 2, the merged Q equal to the oracle's one-process
    answer for 2^20 lanes over the driver's 25 launches (cfg2_L1M_25)"""
    env = dict(os.environ, RLAMD_DIST_BACKEND="gloo", RLAMD_COLLECTIVE="torch")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    qc = d["q_check"]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["lanes_total"] == 1 << 20, d["config"]
    assert d["config"]["lanes_per_gpu"] == 1 << 19 and d["config"]["parallelism"] == "dp2"
    assert qc["ranks_agree"] is True and qc["fixture"] == "cfg2_L1M_25" and qc["match"] is True, json.dumps(qc)


@pytest.mark.gpu
@pytest.mark.parametrize("config,fixture,n", [(2, "cfg2_L1M_25", 2), (4, "cfg4_L512K_25", 2),
                                              (4, "cfg4_L512K_25", 4), (2, "cfg2_L1M_25", 8),
                                              (5, "cfg5_L4M_25", 8)],
                         ids=["cfg2", "cfg4", "cfg4-4ranks", "cfg2-8ranks", "cfg5-8ranks"])
def test_bench_gpus2_peer_merge_q_check(config, fixture, n):
    """`bench.py --gpus N` (self-launched ranks sharing the
    GPU) with the one-shot peer-read merge in every launch: the default strong split
    of BASELINE's global lane set (cfg 2: 2^20; cfg 4: 2^19, "2^19 envs, 4xMI355X" —
    also at its 4 ranks; cfg 2 and cfg 5's "2^22 envs across 8xMI355X" at 8 ranks,
    every rank waiting for seven flags) ends with the oracle's one-process Q for that
    set over the driver's 25 launches"""
    env = dict(os.environ, RLAMD_DIST_BACKEND="gloo", RLAMD_COLLECTIVE="peer")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--config", str(config), "--gpus", str(n), "--steps", "20",
                        "--warmup", "5", "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    qc = d["q_check"]
    assert d["n_gpus"] == n and d["scaling"] == "strong" and d["config"]["merge_path"] == "peer", d["config"]
    assert qc["ranks_agree"] is True and qc["fixture"] == fixture and qc["match"] is True, json.dumps(qc)


@pytest.mark.gpu
def test_bench_rccl_peer_setup_one_rank():
    """bench.py's driver path at N > 1 — librlamd's RCCL communicator, then the
    peer-read setup inside rl_agent_set_comm (handles all-gathered over RCCL,
    agreement, self-test) — run at one rank (RLAMD_PEER_WORLD1: the box has one
    GPU): every merge through the peer kernels, and the driver-shape run's merged Q
    the oracle's (q_check cfg2_L1M_25)"""
    env = dict(os.environ, RLAMD_FORCE_COMM="1", RLAMD_PEER_WORLD1="1", MASTER_ADDR="127.0.0.1")
    env.pop("RLAMD_COLLECTIVE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--steps", "20",
           "--warmup", "5", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert d["config"]["merge_path"] == "peer", d["config"]
    assert d["q_check"]["fixture"] == "cfg2_L1M_25" and d["q_check"]["match"] is True, d["q_check"]
