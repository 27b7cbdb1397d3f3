"""Single-kernel numerics on the GPU vs plain torch fp32 (the op as the graph states it)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,cout,T,k,dil,act", [
    (192, 576, 37, 1, 1, False), (192, 768, 45, 3, 1, False), (256, 256, 160, 11, 5, True),
    (16, 16, 300, 7, 3, True), (128, 256, 265, 5, 1, False), (16, 1, 200, 7, 1, True),
    (512, 512, 1, 1, 1, False), (96, 192, 70, 1, 1, False), (192, 384, 100, 5, 1, False)])
@pytest.mark.parametrize("splitk", [False, True])
def test_conv1d(cin, cout, T, k, dil, act, splitk):
    from genie_tts_amd.engine import debug_conv1d
    g = torch.Generator().manual_seed(cin * 7 + k)
    x = torch.randn(cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / np.sqrt(cin * k)
    b = torch.randn(cout, generator=g) * 0.1
    pad = dil * (k - 1) // 2
    xa = F.leaky_relu(x, 0.1) if act else x
    ref = F.conv1d(xa[None], w, b, padding=pad, dilation=dil)[0]
    ws = torch.empty(2 << 20, device="cuda") if splitk else None   # split-K slabs for small grids
    out = debug_conv1d(x.cuda(), w.cuda(), b.cuda(), dil=dil, pad=pad, in_act=act, splitk_ws=ws).cpu()
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=2e-5 * np.sqrt(cin * k), rtol=1e-4)


# The MRF convs on the f16-split MFMA path: the V2 channel widths 256..16 and the
# V2ProPlus ones (384..24; Cin % 32 != 0 -> 8-channel chunks), every kernel
# size / dilation of dec.resblocks, ragged T.  Weights are fp16-valued weight_v
# with a weight-norm scale, as the character files hold them.
@pytest.mark.parametrize("c,T,k,dil", [
    (256, 160, 11, 5), (256, 1600, 3, 1), (128, 1000, 7, 3), (64, 2050, 11, 1), (32, 4099, 3, 5),
    (16, 8000, 7, 1), (384, 300, 3, 3), (192, 777, 11, 5), (96, 500, 7, 1), (48, 1500, 3, 1), (24, 3001, 11, 3)])
def test_conv1d_f16split(c, T, k, dil):
    from genie_tts_amd.engine import debug_conv1d_h
    g = torch.Generator().manual_seed(c * 13 + k * 3 + dil)
    x = torch.randn(c, T, generator=g) * 3.0
    v = (torch.randn(c, c, k, generator=g) / np.sqrt(c * k)).half().float()       # fp16-valued weight_v
    wg = torch.rand(c, generator=g) + 0.5                                          # weight_g
    nrm = torch.sqrt((v.double() ** 2).sum(dim=(1, 2))).float()
    w = (v / nrm[:, None, None]) * wg[:, None, None]                               # graph order: v/||v|| * g
    b = torch.randn(c, generator=g) * 0.1
    pad = dil * (k - 1) // 2
    ref = F.conv1d(F.leaky_relu(x, 0.1)[None], w, b, padding=pad, dilation=dil)[0]
    out, ovf = debug_conv1d_h(x.cuda(), v, wg / nrm, b.cuda(), dil=dil, pad=pad, in_act=True)
    assert ovf == 0
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), atol=2e-5 * np.sqrt(c * k), rtol=1e-4)


def test_conv1d_f16split_overflow_flag():
    from genie_tts_amd.engine import debug_conv1d_h
    x = torch.randn(32, 200)
    x[5, 17] = 1e6                                   # no fp16 hi part
    v = torch.randn(32, 32, 3).half().float()
    _, ovf = debug_conv1d_h(x.cuda(), v, torch.ones(32), None, dil=1, pad=1)
    assert ovf == 1


def test_hbm_copy_probe_copies_and_times():
    """gsv_debug_hbm_copy: the destination equals the source after the copies, and the rate is
    plausible for HBM3E (bench.py's roofline.achievable_hbm)."""
    import torch
    from genie_tts_amd.engine import hbm_copy_ms
    src = torch.randn(1 << 24, device="cuda")
    dst = torch.zeros_like(src)
    ms = hbm_copy_ms(src, dst, 3)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    gbs = 2 * src.numel() * 4 / (ms * 1e-3) / 1e9
    assert 500 < gbs < 9000, gbs
