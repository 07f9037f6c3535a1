"""CPU checks of the residual-tower network's host side (BASELINE config 5):
the product module's state_dict matches the weight generator and the C ABI's
key list, and the two oracle modes (fp32 definition, bf16 rounding points)
agree to bf16 precision."""
import numpy as np
import torch


def test_state_dict_keys_match_generator():
    import mzgo
    for C, N, blocks in ((64, 5, 0), (64, 9, 2), (256, 19, 3)):
        A = N * N + 1
        net = mzgo.ResMuZeroNet(C, A, blocks)
        sd = mzgo.deterministic_res_state_dict(C, A, blocks, 0)
        assert list(net.state_dict()) == list(sd)
        for k, v in net.state_dict().items():
            assert tuple(v.shape) == tuple(sd[k].shape), k
        net.load_state_dict(sd)


def test_generator_is_deterministic_and_seeded():
    import mzgo
    a = mzgo.deterministic_res_state_dict(64, 26, 1, 0)
    b = mzgo.deterministic_res_state_dict(64, 26, 1, 0)
    c = mzgo.deterministic_res_state_dict(64, 26, 1, 1)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert not torch.equal(a["dynamics.conv_in.weight"], c["dynamics.conv_in.weight"])
    w = a["representation.blocks.0.conv1.weight"]
    assert w.abs().max().item() <= 1 / np.sqrt(64 * 9) + 1e-7


def test_oracle_bf16_rounding_points_track_fp32():
    import mzgo
    from oracle.positions import random_position
    from oracle.resnet import OracleResNet
    N, C, blocks = 5, 64, 2
    A = N * N + 1
    sd = mzgo.deterministic_res_state_dict(C, A, blocks, 0)
    emu, f32 = OracleResNet(sd, blocks, bf16=True), OracleResNet(sd, blocks, bf16=False)
    obs = torch.from_numpy(np.stack([random_position(N, m, m) for m in (0, 5, 11)]).astype(np.float32))
    with torch.no_grad():
        l1, v1, g1 = emu.initial_inference(obs)
        l2, v2, g2 = f32.initial_inference(obs)
        # bf16-stored latents are exactly representable in bf16
        assert torch.equal(l1, l1.to(torch.bfloat16).float())
        np.testing.assert_allclose(l1.numpy(), l2.numpy(), atol=0.05, rtol=0.05)
        np.testing.assert_allclose(g1.numpy(), g2.numpy(), atol=0.05, rtol=0.05)
        a = torch.tensor([0, A - 1, 7])
        n1, r1, w1, h1 = emu.recurrent_inference(l1, a)
        n2, r2, w2, h2 = f32.recurrent_inference(l1, a)
        np.testing.assert_allclose(n1.numpy(), n2.numpy(), atol=0.05, rtol=0.05)
        np.testing.assert_allclose(r1.numpy(), r2.numpy(), atol=0.05, rtol=0.05)
