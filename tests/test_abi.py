"""CPU: the C ABI library (no GPU compute).

* librlamd.so loads and exports every function include/rl.h declares
* the product's host-built transition tables (decoded through rl_env_table)
  equal the independent Python restatement and the oracle's
* Blackjack observation ids (fxhash 0.2.1) agree with the oracle
* without a GPU, compute entry points fail loudly (no CPU fallback)
"""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "tables.json")))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "rl.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rl_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol(rl):
    names = declared_functions()
    assert len(names) >= 40
    out = subprocess.run(["nm", "-D", "--defined-only", rl.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (rl_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # and the Python binding covers the whole header
    assert set(names) <= set(rl.SIGNATURES), set(names) - set(rl.SIGNATURES)
    assert rl.lib().rl_abi_version() == 7
    info = rl.lib().rl_build_info().decode()
    assert "gfx950" in info and "RLAMD_EXP=0" in info and "-ffp-contract=off" in info, info


def test_header_is_plain_c_and_links(rl, tmp_path):
    """The drop-in boundary is a C ABI: include/rl.h compiles as ISO C11 with
    -pedantic -Werror (what cgo / bindgen / any FFI would parse), a C program that
    takes the address of every declared function links against librlamd.so, and
    its GPU-free calls answer (no compute: this container has no GPU)"""
    names = declared_functions()
    prog = tmp_path / "abi.c"
    prog.write_text(
        "#include <stdio.h>\n#include \"rl.h\"\n"
        "typedef void (*fp)(void);\n"
        "static const fp every[] = {\n" + ",\n".join(f"    (fp){n}" for n in names) + "\n};\n"
        "int main(void) {\n"
        "    printf(\"%d %u %s\\n\", rl_abi_version(), (unsigned)(sizeof every / sizeof every[0]), rl_build_id());\n"
        "    return rl_abi_version() == RL_ABI_VERSION ? 0 : 1;\n}\n")
    exe = tmp_path / "abi"
    libdir = os.path.dirname(rl.LIB_PATH)
    cc = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I",
                         os.path.join(ROOT, "include"), str(prog), "-L", libdir, "-lrlamd",
                         f"-Wl,-rpath,{libdir}", "-o", str(exe)], capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-3000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert run.returncode == 0, run.stderr
    abi, n, bid = run.stdout.split()[:3]
    assert int(abi) == 7 and int(n) == len(names) and bid.startswith("src:")


def test_loaded_library_was_built_from_this_checkout(rl):
    """rl_build_id's source hash == the hash of the sources in this tree, so a stale
    librlamd.so (built from other sources) fails here instead of being benched or
    profiled unnoticed"""
    bid = rl.build_id()
    assert bid.startswith("src:") and " git:" in bid, bid
    assert bid.split()[0] == rl.source_id(), (bid, rl.source_id(), "rebuild: make -C rl-rust_amd")
    assert bid in rl.lib().rl_build_info().decode()


def test_obs_from_reference_inverts_obs_to_reference(rl):
    L = rl.lib()
    d = ctypes.c_uint32()
    for s in range(2048):
        assert L.rl_obs_from_reference(3, L.rl_obs_to_reference(3, s), ctypes.byref(d)) == 0 and d.value == s
    assert L.rl_obs_from_reference(3, 12345, ctypes.byref(d)) == 2
    assert L.rl_obs_from_reference(2, 499, ctypes.byref(d)) == 0 and d.value == 499


ENV_CASES = [("frozen_lake_4x4_det", dict(env="frozen_lake", map8x8=0, slippery=0)),
             ("frozen_lake_4x4_slippery", dict(env="frozen_lake", map8x8=0, slippery=1)),
             ("frozen_lake_8x8_det", dict(env="frozen_lake", map8x8=1, slippery=0)),
             ("frozen_lake_8x8_slippery", dict(env="frozen_lake", map8x8=1, slippery=1)),
             ("cliff_walking", dict(env="cliff_walking")),
             ("taxi", dict(env="taxi")),
             ("frozen_lake_edited_4x4_det", dict(env="frozen_lake_edited", map8x8=0, slippery=0)),
             ("frozen_lake_edited_4x4_slippery", dict(env="frozen_lake_edited", map8x8=0, slippery=1)),
             ("frozen_lake_edited_8x8_det", dict(env="frozen_lake_edited", map8x8=1, slippery=0)),
             ("frozen_lake_edited_8x8_slippery", dict(env="frozen_lake_edited", map8x8=1, slippery=1))]


@pytest.mark.parametrize("name,kw", ENV_CASES, ids=[c[0] for c in ENV_CASES])
def test_device_tables_match_fixtures_and_oracle(rl, oracle, name, kw):
    t = rl.env_table(rl.default_params(**kw))
    g = GOLD[name]
    o = oracle.env_table(oracle.default_params(**kw))
    for f in ("prob", "next", "reward", "term"):
        assert np.array_equal(t[f], np.array(g[f], dtype=t[f].dtype)), f
        assert np.array_equal(t[f], o[f]), f
    assert np.array_equal(t["start"], np.array(g["start"]))


def test_env_dims(rl):
    assert rl.env_dims(rl.default_params(env="frozen_lake", map8x8=1)) == (64, 4)
    assert rl.env_dims(rl.default_params(env="cliff_walking")) == (48, 4)
    assert rl.env_dims(rl.default_params(env="taxi")) == (500, 6)
    assert rl.env_dims(rl.default_params(env="blackjack")) == (32 * 32 * 2, 2)


def test_blackjack_ids(rl, oracle):
    L, O = rl.lib(), oracle.lib()
    for p in range(32):
        for d in range(27):
            for a in range(2):
                assert L.rl_blackjack_obs_id(p, d, a) == O.rlo_blackjack_obs_id(p, d, a)
                s = (p * 32 + d) * 2 + a
                assert L.rl_obs_to_reference(3, s) == O.rlo_blackjack_obs_id(p, d, a)
    assert L.rl_obs_to_reference(0, 17) == 17


def test_bad_arguments_are_reported(rl):
    c = rl.agent_config(rl.default_params(n_lanes=0))
    h = ctypes.c_void_p()
    rc = rl.lib().rl_agent_create(ctypes.byref(c), ctypes.byref(h))
    assert rc == 2 and b"n_lanes" in rl.lib().rl_last_error()


def _gpu_visible(rl):
    n = ctypes.c_int(0)
    return rl.lib().rl_device_count(ctypes.byref(n)) == 0 and n.value > 0


def test_no_cpu_fallback_without_gpu(rl):
    """The product path fails loudly when no HIP device is present."""
    if _gpu_visible(rl):
        pytest.skip("a GPU is visible")
    with pytest.raises(rl.RLError) as e:
        rl.Agent(rl.default_params())
    assert e.value.code == 3          # RL_E_HIP


@pytest.mark.parametrize("map8", [0, 1])
def test_fl_obs_features_match_fixture(rl, oracle, map8):
    """FrozenLakeObs input adapter (frozen_lake_neural.rs:136-145): host table ==
    independent restatement == oracle"""
    name = f"frozen_lake_edited_{'8x8' if map8 else '4x4'}_det"
    g = np.array(GOLD[name]["fl_obs"])
    for env in ("frozen_lake_edited", "frozen_lake"):
        p = dict(env=env, map8x8=map8, net_input="fl_obs", policy="neural")
        assert np.array_equal(rl.net_features(rl.default_params(**p)), g)
        assert np.array_equal(oracle.net_features(oracle.default_params(**p)), g)


def test_scalar_features_are_reference_obs_ids(rl):
    f = rl.net_features(rl.default_params(env="blackjack", net_input="scalar"))
    ids = [rl.lib().rl_obs_to_reference(3, s) for s in range(f.shape[0])]
    assert np.array_equal(f[:, 0], np.array(ids, dtype=np.uint64).astype(np.float64))
    f = rl.net_features(rl.default_params(env="taxi", net_input="scalar"))
    assert np.array_equal(f[:, 0], np.arange(500, dtype=np.float64))
    with pytest.raises(rl.RLError):   # FrozenLakeObs is a struct: no [[obs as f64]]
        rl.net_features(rl.default_params(env="frozen_lake_edited", net_input="scalar"))
    with pytest.raises(rl.RLError):
        rl.net_features(rl.default_params(env="taxi", net_input="fl_obs"))


def test_neural_config_validation(rl):
    """bad network configs fail with RL_E_ARG before any GPU work"""
    for kw in (dict(group_size=2), dict(net_hidden=0), dict(net_hidden=4096), dict(net_act1="softmax")):
        p = rl.default_params(policy="neural", n_lanes=4, **kw)
        with pytest.raises(rl.RLError) as e:
            rl.Agent(p)
        assert e.value.code == 2, (kw, e.value)
