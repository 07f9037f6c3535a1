"""CPU checks of the drop-in boundary: libmzgo.so loads, exports every symbol
include/mzgo.h declares, its ctypes mirror matches the C struct layout, and
the host-side record logic reproduces the reference's types.  No GPU needed
(and no compute call is made)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mzgo.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mzgo_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from mzgo import _lib
    names = declared_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(_lib.lib, n), f"{n} declared in mzgo.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with mzgo.h"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (mzgo_\w+)", out))
    assert set(names) <= exported


def test_config_struct_layout_matches_header(tmp_path):
    from mzgo._lib import Config
    src = tmp_path / "layout.c"
    fields = [f for f, _ in Config._fields_]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mzgo.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(mzgo_config, {f}));\n' for f in fields)
                   + 'printf("%zu\\n", sizeof(mzgo_config));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [getattr(Config, f).offset for f in fields] + [ctypes.sizeof(Config)]
    assert got == want


def test_default_config_is_the_reference_config():
    from mzgo import _lib
    c = _lib.Config()
    _lib.lib.mzgo_default_config(ctypes.byref(c), 9)
    assert (c.board_size, c.latent_dim, c.num_simulations, c.max_moves) == (9, 96, 128, 81)
    assert (c.c_puct, c.discount, c.dirichlet_alpha, c.dirichlet_epsilon, c.pass_epsilon) == \
        (2.5, 0.99, 0.15, 0.02, 0.01)
    assert (c.temperature, c.temperature_moves, c.komi, c.compat) == (1.0, 15, 0.0, 0)


def test_unsupported_config_fails_loudly():
    from mzgo import _lib
    c = _lib.Config()
    _lib.lib.mzgo_default_config(ctypes.byref(c), 7)        # no 7x7 build
    h = ctypes.c_void_p()
    rc = _lib.lib.mzgo_engine_create(ctypes.byref(c), ctypes.byref(h))
    assert rc == _lib.MZGO_EINVAL and not h.value
    assert b"unsupported board_size" in _lib.lib.mzgo_last_error()


def test_product_weights_match_oracle_generator():
    from mzgo.weights import deterministic_state_dict as product
    from oracle.weights import deterministic_state_dict as oracle
    for C, A, seed in ((96, 82, 0), (96, 26, 5), (64, 362, 1)):
        a, b = product(C, A, seed), oracle(C, A, seed)
        assert list(a) == list(b)
        for k in b:
            np.testing.assert_array_equal(a[k].numpy(), b[k])


def _fake_record(N, actions, final, reward_last):
    L = len(actions)
    A = N * N + 1
    return dict(length=L, status=1, stones=np.zeros((L, N * N), np.int8),
                invd=np.zeros((L, N * N), np.uint8), flags=np.zeros(L, np.uint8),
                action=np.array(actions, np.int32), value=np.linspace(0, 1, L),
                policy=np.full((L, A), 1.0 / A), reward=np.array([0.0] * (L - 1) + [reward_last]),
                final_reward=final)


def test_history_types_follow_the_reference():
    from mzgo.selfplay import history_from_device
    N = 5
    ended = history_from_device(_fake_record(N, [3, 25, 25], -1.0, -1.0), N, 0.99)
    rec = ended.to_record()
    assert [type(r).__name__ for r in rec["rewards"]] == ["int", "int", "float64"]
    assert type(rec["final_reward"]).__name__ == "float64"
    assert [type(r).__name__ for r in rec["returns"]] == ["float64"] * 3
    assert rec["returns"][-1] == -1.0 + 0.99 * -1.0          # outcome counted twice (Appendix C.4)
    cut = history_from_device(_fake_record(N, [3, 4, 25], 0.0, 0.0), N, 0.99).to_record()
    assert [type(r).__name__ for r in cut["rewards"]] == ["int"] * 3
    assert type(cut["final_reward"]).__name__ == "int"
    assert [type(r).__name__ for r in cut["returns"]] == ["float"] * 3
    assert all(type(v).__name__ == "float" for v in cut["values"])
    assert all(o.dtype == np.float64 and o.shape == (6, N, N) for o in cut["observations"])


def test_save_batches_slice_quirk(tmp_path):
    import pickle

    from mzgo.selfplay import GameHistory, save_batches
    hs = []
    for i in range(13):
        h = GameHistory(5, 0.99)
        h.actions.append(i)
        h.rewards.append(0)
        h.observations.append(np.zeros((6, 5, 5)))
        h.policies.append(np.zeros(26))
        h.values.append(0.0)
        hs.append(h)
    paths = save_batches(hs, str(tmp_path), save_interval=10)
    assert [os.path.basename(p) for p in paths] == ["self_play_batch_10.pkl", "self_play_batch_13.pkl"]
    with open(paths[1], "rb") as f:
        last = pickle.load(f)
    assert [r["actions"][0] for r in last] == list(range(3, 13))   # games 4..13 (duplicates 4..10)
