"""GPU parity: the fused MFMA network kernels vs the reference network.

Golden vectors: reference MuZeroNet (self_play.py:115-128) in torch fp32 on
the CPU, plus its fp64 evaluation (tests/golden/net_N*.npz).  Tolerance: the
HIP kernels compute in fp32 with a different summation order (k-ordered fmaf
chains on v_mfma_f32_16x16x4_f32), so we require |gpu - ref32| <= 5e-5
absolute AND that the GPU's distance to the fp64 truth is within 4x (+1e-6)
of torch fp32's own distance to it.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("latent", "value0", "logits0", "next_latent", "reward1", "value1", "logits1")


def _net(N, C=96, seed=0):
    import mzgo
    from oracle.weights import deterministic_state_dict
    sd = deterministic_state_dict(C, N * N + 1, seed)
    net = mzgo.MuZeroNet(C, N * N + 1).to("cuda").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net, sd


@pytest.mark.parametrize("N", [5, 9, 19])
def test_inference_matches_reference_golden(golden_dir, N):
    g = np.load(f"{golden_dir}/net_N{N}.npz")
    net, _ = _net(N)
    lat, v0, lg0 = net.initial_inference(torch.from_numpy(g["obs"]).float().cuda())
    nl, r1, v1, lg1 = net.recurrent_inference(torch.from_numpy(g["latent"]).cuda(),
                                              torch.from_numpy(g["action"]).cuda())
    got = dict(zip(KEYS, (lat, v0, lg0, nl, r1, v1, lg1)))
    for k in KEYS:
        x = got[k].cpu().numpy()
        ref32, ref64 = g[k], g[k + "_f64"]
        assert x.shape == ref32.shape, k
        err32 = np.abs(x - ref32).max()
        assert err32 <= 5e-5, f"{k}: |gpu-ref32| = {err32}"
        e_gpu = np.abs(x - ref64).max()
        e_ref = np.abs(ref32 - ref64).max()
        assert e_gpu <= 4 * e_ref + 1e-6, f"{k}: gpu err {e_gpu} vs torch-fp32 err {e_ref}"


@pytest.mark.parametrize("N,B,C", [(5, 33, 96), (6, 7, 96), (9, 256, 96), (19, 9, 96), (6, 16, 128)])
def test_batched_inference_matches_oracle(N, B, C):
    """C=128 at 6x6 is main.py's training configuration (main.py:27-30)."""
    from oracle.net import OracleNet
    net, sd = _net(N, seed=3, C=C)
    ref = OracleNet(sd)
    gen = torch.Generator().manual_seed(N * 100 + B)
    obs = (torch.rand(B, 6, N, N, generator=gen) < 0.3).float()
    lat_in = torch.rand(B, C, N, N, generator=gen) * 2
    act = torch.randint(0, N * N + 1, (B,), generator=gen)
    lat, v0, lg0 = net.initial_inference(obs.cuda())
    nl, r1, v1, lg1 = net.recurrent_inference(lat_in.cuda(), act.cuda())
    with torch.no_grad():
        want = ref.initial_inference(obs) + ref.recurrent_inference(lat_in, act)
    for name, x, y in zip(KEYS, (lat, v0, lg0, nl, r1, v1, lg1), want):
        err = (x.cpu() - y).abs().max().item()
        tol = 5e-5 * max(1.0, y.abs().max().item())
        assert err <= tol, f"{name} N={N} B={B}: {err} > {tol}"


def test_out_of_range_action_raises():
    net, _ = _net(5)
    eng = net.engine()
    lat = torch.zeros(2, 96, 5, 5, device="cuda")
    with pytest.raises(IndexError):
        eng.recurrent_inference(lat, torch.tensor([0, 26], device="cuda"), check_range=True)


def test_weights_follow_parameter_updates():
    """load_state_dict after a call must re-pack the weights (MuZeroNet drop-in)."""
    net, sd = _net(5)
    obs = torch.zeros(1, 6, 5, 5, device="cuda")
    _, v_a, _ = net.initial_inference(obs)
    with torch.no_grad():
        net.prediction.value_fc.bias.add_(1.0)
    _, v_b, _ = net.initial_inference(obs)
    assert abs((v_b - v_a).item() - 1.0) < 1e-5
