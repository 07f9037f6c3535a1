"""bench.py's host-side logic (no GPU): the CPU share the cpu_baseline leg
uses, and config 5's roofline arithmetic."""
import os

import pytest

import bench


def test_cpu_share_prefers_the_cgroup_quota(tmp_path, monkeypatch):
    f = tmp_path / "cpu.max"
    f.write_text("1600000 100000\n")
    monkeypatch.setenv("OMP_NUM_THREADS", "4")
    assert bench.cpu_share(str(f)) == (16, "cgroup cpu.max 1600000 100000")


def test_cpu_share_without_quota(tmp_path, monkeypatch):
    f = tmp_path / "cpu.max"
    f.write_text("max 100000\n")
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    n, src = bench.cpu_share(str(f))
    assert n == 1 and src.startswith("OMP_NUM_THREADS=1")
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_share(str(tmp_path / "absent")) == (aff, f"affinity mask ({aff} cpus)")
    # an OMP_NUM_THREADS beyond the affinity mask is not a share
    monkeypatch.setenv("OMP_NUM_THREADS", str(aff + 1))
    assert bench.cpu_share(str(f))[0] == aff


@pytest.mark.parametrize("batched", ["0", "1"])
def test_tower_roofline_arithmetic(batched, monkeypatch):
    """achieved = boards x L x 2 N^2 9 C^2 / time; per-launch values for G boards."""
    monkeypatch.setenv("MZGO_TOWER_BATCH", batched)
    N, C, B, G = 19, 256, 20, 64
    L = 2 * B + 1
    board_towers = 6400                      # e.g. 100 timed one-leaf towers of 64 boards
    ms = 6400 * L * 0.35e-3                  # 0.35 us per board-conv
    r = bench.tower_roofline(N, C, B, G, 102400, ms, board_towers, 110000)
    flop = 2 * N * N * 9 * C * C
    assert r["flops_per_board_conv"] == flop
    assert abs(r["achieved"] - flop / 0.35e-6 / 1e12) < 1e-6 * r["achieved"]
    assert abs(r["avg_launch_ms"] - 0.35e-3 * G) < 1e-12
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert abs(r["towers_per_simulation"] - 110000 / 102400) < 1e-12
    assert r["kernel"] == ("k_tconv_chain<19>" if batched == "0" else "k_tconv_ks<19>")


def test_selfplay_roofline_names_the_timed_kernel(tmp_path, monkeypatch):
    """The move-parallel epoch's roofline is k_search_queue's: its avg launch
    time is the one passed in, MFMA work per launch is the convs + the
    representation per move, and a PMC profile is attached only when it is
    of the same kernel (summarize_pmc stores the full demangled name)."""
    import json
    N, C, S, G = 9, 96, 200, 256
    counts = dict(launches=2, sims=2 * 4.0e6, moves=2 * 20000.0, convs=2 * 150000.0, rows=2 * 140000.0)
    prof = tmp_path / "profiles"
    prof.mkdir()
    wl = "9x9 Go self-play, 256 parallel games/GPU, 200 sims/move"
    pmc = {"tag": "t", "workload": wl, "dynamics": "factored", "moves_per_launch": 0, "n_gpus": 1,
           "kernel": "void mzgo::k_search_queue<9, 96>(mzgo::NetParams, ...)", "avg_duration_ms": 30.0,
           "counters": {"GRBM_GUI_ACTIVE": 8 * 2.4e9 * 0.030, "SQ_INSTS_VALU": 1.0e9, "SQ_LDS_IDX_ACTIVE": 4.0e9},
           "hbm_bytes_per_launch": 1.5e10}
    (prof / "latest_pmc.json").write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = bench.roofline(N, C, S, G, counts, 0.030, "factored", wl, 0, 1, "k_search_queue")
    assert r["kernel"] == "k_search_queue" and r["traffic"] == 1.5e10
    assert abs(r["avg_launch_ms"] - 30.0) < 1e-9
    per = 2048 * (150000 * bench.mfma_per_conv(N, C, C) + 20000 * (
        9 * 2 * 4 * 6 + bench.mfma_per_conv(N, 64, 64) + bench.mfma_per_conv(N, 64, C)))
    assert abs(r["units"]["mfma"]["per_launch"] - per) < 1e-6 * per
    assert r["units"]["pmc_source"] == "profiles/t_pmc.json"
    # a profile of the game-per-workgroup kernel is not this kernel's
    r2 = bench.roofline(N, C, S, G, counts, 0.030, "factored", wl, 0, 1, "k_selfplay_move")
    assert r2["traffic"] is None and "pmc_source" not in r2["units"]
