import sys, numpy as np, torch
sys.path.insert(0, '.')
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine
from oracle import restate as R
from tests.common import character
ver = sys.argv[1] if len(sys.argv) > 1 else 'v2'
w = character(ver)
e = Engine({k: w[k] for k in w}, ver)
vm = R.VitsModel(w['vits'], ver)
G, S = 8, 10
txt = synth.synth_phones(S, 'vt10'); sem = ((np.arange(G) * 37 + 11) % 1024).reshape(1, 1, G)
kw = dict(ref_audio=synth.synth_ref_audio(32000 * 2 + 1234)) if ver == 'v2' else dict(ge=synth.synth_ge(1024), ge_advanced=synth.synth_ge(512, 'adv'))
ref = vm(txt, sem, **kw).numpy()
out = e.vits_decode(txt, sem, **kw).cpu().numpy()
torch.cuda.synchronize()
T = 2 * G
def cmp(name, a, b):
    a = np.asarray(a).ravel(); b = np.asarray(b).ravel()
    print(f"{name:8s} maxdiff {np.abs(a-b).max():.3e} ref_absmax {np.abs(b).max():.3e} got_absmax {np.abs(a).max():.3e}")
if ver == 'v2':
    cmp('ge', e.debug_copy('ge', 512).cpu().numpy(), vm.last['ge'].numpy())
cmp('stats_m', e.debug_copy('stats', 384 * T).cpu().numpy()[:192 * T], vm.last['m_p'].numpy())
cmp('stats_l', e.debug_copy('stats', 384 * T).cpu().numpy()[192 * T:], vm.last['logs_p'].numpy())
cmp('z', e.debug_copy('z', 192 * T).cpu().numpy(), vm.last['z'].numpy())
cmp('audio', out, ref)
# generator intermediates
import torch.nn.functional as F
wv = vm.w; c = vm.cfg; d = "vq_model.dec."
z = vm.last['z']; ge = vm.last['ge']
x = F.conv1d(z, wv[d + "conv_pre.weight"], wv[d + "conv_pre.bias"], padding=3) + F.conv1d(ge, wv[d + "cond.weight"], wv[d + "cond.bias"])
stages = []
for i, (u, k) in enumerate(zip(c.up_rates, c.up_kernels)):
    xu = F.conv_transpose1d(F.leaky_relu(x, 0.1), wv[d + f"ups.{i}.weight"], wv[d + f"ups.{i}.bias"], stride=u, padding=(k - u) // 2)
    xs = None
    for j, kk in enumerate(c.rb_kernels):
        rb = d + f"resblocks.{i * 3 + j}."; r = xu
        for m_, dil in enumerate(c.rb_dilations):
            xt = F.conv1d(F.leaky_relu(r, 0.1), wv[rb + f"convs1.{m_}.weight"], wv[rb + f"convs1.{m_}.bias"], padding=(kk * dil - dil) // 2, dilation=dil)
            xt = F.conv1d(F.leaky_relu(xt, 0.1), wv[rb + f"convs2.{m_}.weight"], wv[rb + f"convs2.{m_}.bias"], padding=(kk - 1) // 2)
            r = xt + r
        xs = r if xs is None else xs + r
    x = xs / 3.0
    stages.append((xu, x))
n = stages[-1][1].numel()
cmp('g0_final', e.debug_copy('g0', n).cpu().numpy(), stages[-1][1].numpy())
cmp('g1_convT4', e.debug_copy('g1', stages[-1][0].numel()).cpu().numpy(), stages[-1][0].numpy())
from genie_tts_amd.engine import debug_conv1d
g0 = e.debug_copy('g0', n).reshape(16, -1)
wpost = wv[d + "conv_post.weight"].cuda()
o1 = debug_conv1d(g0, wpost, None, dil=1, pad=3, in_act=True, slope=0.01).cpu()
o_ref = F.conv1d(F.leaky_relu(stages[-1][1], 0.01), wv[d + "conv_post.weight"], None, padding=3)[0]
cmp('post_dbg', o1.numpy(), o_ref.numpy())
cmp('post_tanh', np.tanh(o1.numpy()), ref)
print('audio head', out[:8], 'ref head', ref[:8])
