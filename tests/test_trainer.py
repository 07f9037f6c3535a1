"""Trainer ingestion (mzgo.trainer) on the CPU.

The reference-mode step is pinned by ``tests/golden/train_5x5_c32.npz``:
main.py's own ``MuZeroAgent.train`` (main.py:381-522) run twice on synthetic
trajectories with fixed start indices (oracle/make_golden.py: make_train).
Here the same step runs through ``mzgo.trainer.MuZeroTrainer`` with torch on
the CPU (same ops, one thread) and must reproduce the reference's losses,
priorities, learning rate and weights.
"""
import numpy as np
import pytest
import torch


def _unpack(g):
    lens = g["traj_len"]
    trajs, o, a, r, p = [], 0, 0, 0, 0
    for T in lens:
        T = int(T)
        trajs.append(dict(observations=list(g["traj_obs"][o:o + T + 2]),
                          actions=[int(x) for x in g["traj_actions"][a:a + T]],
                          rewards=[float(x) for x in g["traj_rewards"][r:r + T + 1]],
                          policies=list(g["traj_policies"][p:p + T])))
        o += T + 2
        a += T
        r += T + 1
        p += T
    return trajs


class _Buf:
    def __init__(self, trajs):
        self.trajs, self.prios = trajs, []

    def sample(self, bs):
        return self.trajs, list(range(bs))

    def update_priorities(self, idx, p):
        self.prios.append(list(p))


def _net(g, device="cpu"):
    import mzgo
    N, C = int(g["N"]), int(g["C"])
    net = mzgo.MuZeroNet(C, N * N + 1)
    net.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in _initial(g).items()})
    return net.to(device)


def _initial(g):
    from oracle.weights import deterministic_state_dict
    N, C, seed = int(g["N"]), int(g["C"]), int(g["seed"])
    return {"w_" + k: v for k, v in deterministic_state_dict(C, N * N + 1, seed).items()}


def run_reference_step(g, device="cpu"):
    from mzgo.trainer import MuZeroTrainer
    trajs = _unpack(g)
    starts = iter(int(s) for s in g["starts"])
    net = _net(g, device)
    tr = MuZeroTrainer(net, mode="reference", start_index=lambda T: next(starts))
    buf = _Buf(trajs)
    losses = [tr.train(buf, int(g["B"])) for _ in range(len(g["losses"]))]
    return net, tr, buf, losses


def test_reference_mode_matches_main_py_training_step(golden_dir):
    g = np.load(f"{golden_dir}/train_5x5_c32.npz")
    net, tr, buf, losses = run_reference_step(g)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-6)
    np.testing.assert_allclose(np.array(buf.prios), g["priorities"], rtol=1e-6)
    assert tr.optimizer.param_groups[0]["lr"] == float(g["lr"])
    sd = net.state_dict()
    for k in sd:
        np.testing.assert_allclose(sd[k].detach().numpy(), g["w_" + k], rtol=1e-5, atol=1e-7, err_msg=k)


def test_batched_mode_with_one_trajectory_is_the_reference_step(golden_dir):
    """With B = 1 both modes take one optimizer step on one trajectory's loss."""
    from mzgo.trainer import MuZeroTrainer
    g = np.load(f"{golden_dir}/train_5x5_c32.npz")
    trajs = _unpack(g)[:1]
    nets = {}
    for mode in ("reference", "batched"):
        starts = iter([int(g["starts"][0])] * 4)
        net = _net(g)
        tr = MuZeroTrainer(net, mode=mode, start_index=lambda T: next(starts))
        loss = tr.train(_Buf(trajs), 1)
        nets[mode] = (net, loss)
    assert nets["batched"][1] == pytest.approx(nets["reference"][1], rel=1e-5)
    a, b = nets["reference"][0].state_dict(), nets["batched"][0].state_dict()
    for k in a:
        np.testing.assert_allclose(a[k].numpy(), b[k].numpy(), rtol=1e-4, atol=1e-6, err_msg=k)


def test_trajectory_from_record_is_main_py_format():
    from mzgo.trainer import trajectory_from_record
    N, A, L = 3, 10, 4
    rec = dict(length=L, action=np.array([0, 9, 4, 9]), stones=np.zeros((L, 9), np.int8),
               invd=np.zeros((L, 9), np.uint8), flags=np.array([0, 1, 0, 1], np.uint8),
               reward=np.zeros(L), policy=np.full((L, A), 0.1), final_reward=np.array(1.0))
    fin = np.zeros((6, N, N))
    t = trajectory_from_record(rec, fin, N, max_moves=L)           # not ended, hit the cap
    assert len(t["observations"]) == L + 2 and len(t["actions"]) == L
    assert len(t["policies"]) == L and len(t["rewards"]) == L + 1
    assert t["rewards"][-2] == -0.5 and t["rewards"][-1] == 0.0    # main.py:699-702, winner() 0
    assert t["observations"][-1] is t["observations"][-2]
    fin[5] = 1.0                                                   # DONE plane: ended by double pass
    t = trajectory_from_record(rec, fin, N, max_moves=L)
    assert t["rewards"][-2] == 0.0 and t["rewards"][-1] == 1.0


def test_replay_buffers_follow_main_py():
    from mzgo.trainer import MultiVersionReplayBuffer, PrioritizedReplayBuffer
    b = PrioritizedReplayBuffer(3)
    for i in range(5):
        b.add({"id": i})
    assert [t["id"] for t in b.buffer] == [2, 3, 4] and b.priorities == [1.0] * 3
    np.random.seed(0)
    s, idx = b.sample(3)
    assert sorted(t["id"] for t in s) == [2, 3, 4]
    b.update_priorities(idx, [5.0, 5.0, 5.0])
    assert b.priorities == [5.0] * 3
    m = MultiVersionReplayBuffer(4, num_versions=2)
    m.add({"id": 0})
    m.add_version()
    m.add({"id": 1})
    assert m.sample(3) == ([], [])
    s, mapping = m.sample(2)
    assert sorted(mapping) == [(0, 0), (1, 0)]
    m.update_priorities(mapping, [2.0, 3.0])
    assert sorted([m.buffers[0].priorities[0], m.buffers[1].priorities[0]]) == [2.0, 3.0]
