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
