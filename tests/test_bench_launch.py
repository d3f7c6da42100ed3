"""bench.py's rank handling, on the CPU (no GPU is touched):
  - under a launcher, --gpus must equal WORLD_SIZE;
  - `bench.py --gpus N` with no launcher starts N ranks itself and fails when a
    rank fails (here every rank fails: no HIP device in this container, and the
    product path has no CPU fallback)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "RLAMD_COLLECTIVE"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_gpus_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--no-cpu-baseline"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
    assert not any(l.startswith("{") for l in r.stdout.splitlines())


def test_self_launch_fails_when_a_rank_fails():
    t0 = time.time()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--lanes", "4096", "--child-timeout", "120"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "a rank exited with" in r.stderr, r.stderr[-3000:]
    assert not any(l.startswith("{") for l in r.stdout.splitlines())
    assert time.time() - t0 < 150


def test_self_launch_sets_rank_env(tmp_path):
    """the ranks get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as
    torch.distributed.run sets them (bench.self_launch run over a stub script in
    place of bench.py: each child reports its environment and exits 0)"""
    import json
    stub = tmp_path / "stub.py"
    stub.write_text("import json, os\nif os.environ['RANK'] == '0':\n"
                    "    print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', "
                    "'MASTER_ADDR', 'MASTER_PORT')}))\n")
    code = ("import sys, importlib.util as u\n"
            f"s = u.spec_from_file_location('b', {os.path.join(ROOT, 'bench.py')!r})\n"
            "b = u.module_from_spec(s)\ns.loader.exec_module(b)\n"
            f"b.__file__ = {str(stub)!r}\n"
            "sys.argv = ['bench.py']\nsys.exit(b.self_launch(3, 60))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=90)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["RANK"] == "0" and d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "3"
    assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
