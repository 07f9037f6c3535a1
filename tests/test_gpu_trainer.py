"""Trainer ingestion on the GPU (mzgo.trainer).

* main.py's training step (reference mode) on the GPU vs the step recorded
  from the reference (tests/golden/train_5x5_c32.npz), to GPU-conv tolerance;
* main.py-format trajectories from the device self-play (MainSelfPlay, main.py's
  6x6 / latent_dim 128 configuration): lengths, legal replay on the oracle
  board (bit-exact planes), policies, winners;
* batched mode: its bootstrap values come from one HIP initial_inference
  launch and must equal the torch forward's; with B = 1 it is the reference
  step.
"""
import numpy as np
import pytest
import torch

from test_trainer import _Buf, _unpack, run_reference_step

pytestmark = pytest.mark.gpu


def test_reference_step_on_gpu_matches_main_py(golden_dir):
    g = np.load(f"{golden_dir}/train_5x5_c32.npz")
    net, tr, buf, losses = run_reference_step(g, device="cuda")
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-4)
    np.testing.assert_allclose(np.array(buf.prios), g["priorities"], rtol=1e-4)
    sd = net.state_dict()
    for k in sd:
        np.testing.assert_allclose(sd[k].detach().cpu().numpy(), g["w_" + k], rtol=1e-3, atol=2e-5, err_msg=k)


def test_main_selfplay_trajectories_replay_on_the_oracle_board():
    import mzgo
    from mzgo.trainer import MainSelfPlay
    from oracle import gogame
    N, C, G, S = 6, 128, 8, 32                     # main.py's Config (main.py:27-53)
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda().eval()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 3))
    trajs = MainSelfPlay(net, G, S, seed=21).play()
    assert len(trajs) == G
    for t in trajs:
        T = len(t["actions"])
        assert 1 <= T <= int(1.5 * N * N)
        assert len(t["observations"]) == T + 2 and len(t["rewards"]) == T + 1 and len(t["policies"]) == T
        st = gogame.init_state(N)
        for k in range(T):
            np.testing.assert_array_equal(t["observations"][k], st)
            p = t["policies"][k]
            assert p.shape == (A,) and abs(p.sum() - 1.0) < 1e-9
            st = gogame.next_state(st, t["actions"][k])
        np.testing.assert_array_equal(t["observations"][T], st)
        np.testing.assert_array_equal(t["observations"][T + 1], st)
        ended = gogame.game_ended(st)
        winner = float(gogame.winning(st)) if ended else 0.0
        assert t["rewards"][-1] == winner
        if not ended:
            assert T == int(1.5 * N * N) and t["rewards"][-2] == -0.5


def test_batched_bootstrap_on_hip_equals_torch():
    import mzgo
    from mzgo.trainer import MuZeroTrainer, initial_inference_torch
    from oracle.make_golden import synthetic_trajectories
    N, C = 5, 96
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 4))
    trajs = synthetic_trajectories(N, 6, seed=9)
    obs = torch.as_tensor(np.stack([o for t in trajs for o in t["observations"]]), dtype=torch.float32).cuda()
    with torch.no_grad():
        _, v_hip, _ = net.initial_inference(obs)
        _, v_t, _ = initial_inference_torch(net, obs)
    np.testing.assert_allclose(v_hip.cpu().numpy(), v_t.cpu().numpy(), rtol=0, atol=1e-5)
    # B = 1: one optimizer step on one trajectory either way
    res = {}
    for mode in ("reference", "batched"):
        net2 = mzgo.MuZeroNet(C, A).cuda()
        net2.load_state_dict(mzgo.deterministic_state_dict(C, A, 4))
        tr = MuZeroTrainer(net2, mode=mode, start_index=lambda T: 0)
        res[mode] = (tr.train(_Buf(trajs[:1]), 1), net2.state_dict())
    assert res["batched"][0] == pytest.approx(res["reference"][0], rel=1e-4)
    for k in res["reference"][1]:
        np.testing.assert_allclose(res["batched"][1][k].cpu().numpy(), res["reference"][1][k].cpu().numpy(),
                                   rtol=1e-3, atol=1e-5, err_msg=k)


def test_batched_mode_trains_on_selfplay_output():
    import mzgo
    from mzgo.trainer import MainSelfPlay, MultiVersionReplayBuffer, MuZeroTrainer
    N, C, G, S = 6, 128, 8, 16
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 5))
    buf = MultiVersionReplayBuffer(100)
    for t in MainSelfPlay(net, G, S, seed=3).play():
        buf.add(t)
    np.random.seed(0)
    tr = MuZeroTrainer(net, mode="batched")
    before = {k: v.clone() for k, v in net.state_dict().items()}
    loss = tr.train(buf, 4)
    assert np.isfinite(loss)
    assert any(not torch.equal(before[k], v) for k, v in net.state_dict().items())
    # the engine picks up the new weights for the next self-play round
    trajs = MainSelfPlay(net, 2, S, seed=4).play()
    assert len(trajs) == 2


def test_hip_forward_autograd_matches_torch():
    """The unroll's HIP forward (k_initial_inference / k_recurrent_inference)
    with the HIP dynamics-conv backward (mzgo_dyn_conv_backward) and torch's
    for the rest: outputs and every parameter / input gradient equal the
    all-torch graph's to fp32-conv tolerance."""
    import mzgo
    from mzgo.trainer import (initial_inference_hip, initial_inference_torch, recurrent_inference_hip,
                              recurrent_inference_torch)
    from oracle.positions import random_position
    N, C, B = 5, 96, 7
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 2))
    obs = torch.as_tensor(np.stack([random_position(N, 3 * b, b) for b in range(B)]), dtype=torch.float32).cuda()
    act = torch.tensor([0, 3, A - 1, 7, 12, 1, 24]).cuda()
    outs = {}
    for name, f0, f in (("hip", initial_inference_hip, recurrent_inference_hip),
                        ("torch", initial_inference_torch, recurrent_inference_torch)):
        net.zero_grad()
        lat, v0, lg0 = f0(net, obs)
        x = lat
        loss = (v0 ** 2).sum() + lg0.logsumexp(1).sum()
        for k in range(3):
            x, r, v, lg = f(net, x, act.roll(k))
            loss = loss + (r ** 2).sum() + (v * 0.5).sum() + lg.logsumexp(1).sum() + 1e-3 * (x ** 2).sum()
        loss.backward()
        outs[name] = (loss.item(), {k: p.grad.detach().clone() for k, p in net.named_parameters()})
    assert outs["hip"][0] == pytest.approx(outs["torch"][0], rel=1e-5)
    for k, g in outs["torch"][1].items():
        np.testing.assert_allclose(outs["hip"][1][k].cpu().numpy(), g.cpu().numpy(), rtol=1e-3,
                                   atol=1e-5 * max(1.0, g.abs().max().item()), err_msg=k)


def test_batched_step_hip_forward_equals_torch_forward():
    import mzgo
    from mzgo.trainer import MuZeroTrainer
    from oracle.make_golden import synthetic_trajectories
    N, C = 5, 96
    A = N * N + 1
    trajs = synthetic_trajectories(N, 6, seed=9)
    res = {}
    for hip in (True, False):
        net = mzgo.MuZeroNet(C, A).cuda()
        net.load_state_dict(mzgo.deterministic_state_dict(C, A, 4))
        tr = MuZeroTrainer(net, mode="batched", start_index=lambda T: T // 3, hip_forward=hip)
        res[hip] = (tr.train(_Buf(trajs), len(trajs)), dict(tr.last))
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-5)
    for k in ("value_loss", "policy_loss", "reward_loss"):
        assert res[True][1][k] == pytest.approx(res[False][1][k], rel=1e-5, abs=1e-7)


@pytest.mark.parametrize("N,C,B", [(6, 128, 40), (5, 96, 7), (9, 96, 3), (6, 64, 1), (19, 96, 2)])
def test_dyn_conv_backward_hip_matches_torch(N, C, B):
    """The dynamics conv's input / weight / bias gradients on the HIP MFMA
    kernels (mzgo_dyn_conv_backward) against torch.nn.grad.conv2d_input /
    conv2d_weight on the same saved tensors (the backward main.py:478-482
    runs through main.py:97-103).  fp32 with a different summation order:
    |diff| <= 1e-5 + 1e-4 |ref| (gx, summed over 9C terms) and
    <= 1e-4 + 1e-4 |ref| for gw / gb (summed over B N^2 terms)."""
    from mzgo.trainer import dyn_conv_backward_hip
    A = N * N + 1
    gen = torch.Generator().manual_seed(N * 1000 + C + B)
    latent = torch.randn(B, C, N, N, generator=gen).relu().cuda()
    emb = torch.randn(A, C, generator=gen).cuda()
    w = (torch.randn(C, C, 3, 3, generator=gen) / (3 * C ** 0.5)).cuda()
    bias = (torch.randn(C, generator=gen) * 0.1).cuda()
    action = torch.randint(0, A, (B,), generator=gen).cuda()
    x = latent + emb[action][:, :, None, None]
    nxt = torch.relu(torch.nn.functional.conv2d(x, w, bias, padding=1))
    g = torch.randn(B, C, N, N, generator=gen).cuda()
    gx, gw, gb = dyn_conv_backward_hip(g, nxt, latent, action, emb, w)
    gp = g * (nxt > 0).float()
    rx = torch.nn.grad.conv2d_input(x.shape, w, gp, padding=1)
    rw = torch.nn.grad.conv2d_weight(x, w.shape, gp, padding=1)
    rb = gp.sum(dim=(0, 2, 3))
    torch.testing.assert_close(gx, rx, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(gw, rw, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gb, rb, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("N,Cin,Cout,B", [(5, 6, 64, 7), (9, 64, 64, 3), (6, 64, 96, 17), (19, 6, 64, 2),
                                          (9, 64, 128, 9)])
def test_conv3x3_layer_hip_matches_torch(N, Cin, Cout, B):
    """The representation's conv layers on the HIP kernels
    (mzgo_conv3x3_relu_forward: the activation recomputation;
    mzgo_conv3x3_backward: input / weight / bias gradients) against torch at
    the shapes of main.py:72-84 (conv1 6 -> 64, conv2 64 -> 64, conv3 64 ->
    C).  fp32, different summation order: forward |diff| <= 1e-5 + 1e-5 |ref|;
    gx <= 1e-5 + 1e-4 |ref|, gw / gb <= 1e-4 + 1e-4 |ref|."""
    from mzgo.trainer import conv3x3_backward_hip, conv3x3_forward_hip
    gen = torch.Generator().manual_seed(N * 1000 + Cin * 7 + Cout + B)
    x = torch.randn(B, Cin, N, N, generator=gen).relu().cuda()
    w = (torch.randn(Cout, Cin, 3, 3, generator=gen) / (3 * Cin ** 0.5)).cuda()
    bias = (torch.randn(Cout, generator=gen) * 0.1).cuda()
    y = conv3x3_forward_hip(x, w, bias)
    ref = torch.relu(torch.nn.functional.conv2d(x, w, bias, padding=1))
    torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn(B, Cout, N, N, generator=gen).cuda()
    gx, gw, gb = conv3x3_backward_hip(g, ref, x, w)
    gp = g * (ref > 0).float()
    torch.testing.assert_close(gx, torch.nn.grad.conv2d_input(x.shape, w, gp, padding=1), atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(gw, torch.nn.grad.conv2d_weight(x, w.shape, gp, padding=1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gb, gp.sum(dim=(0, 2, 3)), atol=1e-4, rtol=1e-4)
    none, gw2, gb2 = conv3x3_backward_hip(g, ref, x, w, need_input_grad=False)
    assert none is None
    assert torch.equal(gw2, gw) and torch.equal(gb2, gb)          # deterministic


def test_representation_backward_is_hip():
    """initial_inference_hip's backward runs the HIP conv kernels, not torch:
    its parameter gradients equal those assembled from conv3x3_backward_hip
    directly, bit for bit."""
    import mzgo
    from mzgo.trainer import conv3x3_backward_hip, conv3x3_forward_hip, initial_inference_hip
    N, C, B = 9, 96, 5
    A = N * N + 1
    net = mzgo.MuZeroNet(C, A).cuda()
    net.load_state_dict(mzgo.deterministic_state_dict(C, A, 3))
    gen = torch.Generator().manual_seed(5)
    obs = (torch.rand(B, 6, N, N, generator=gen) > 0.6).float().cuda()
    lat, _, _ = initial_inference_hip(net, obs)
    g = torch.randn(lat.shape, generator=gen).cuda()
    net.zero_grad()
    lat.backward(g)
    r = net.representation
    x1 = conv3x3_forward_hip(obs, r.conv1.weight, r.conv1.bias)
    x2 = conv3x3_forward_hip(x1, r.conv2.weight, r.conv2.bias)
    g2, gw3, _ = conv3x3_backward_hip(g, lat.detach(), x2, r.conv3.weight)
    g1, gw2, _ = conv3x3_backward_hip(g2, x2, x1, r.conv2.weight)
    _, gw1, _ = conv3x3_backward_hip(g1, x1, obs, r.conv1.weight, need_input_grad=False)
    for got, want in ((r.conv3.weight.grad, gw3), (r.conv2.weight.grad, gw2), (r.conv1.weight.grad, gw1)):
        assert torch.equal(got, want)
