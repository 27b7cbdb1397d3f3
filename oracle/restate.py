"""CPU restatement of Genie's ONNX hot path in torch fp32 (oracle / CPU baseline).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Op-for-op restatement of
the reference graphs (op order and constants as in the templates; node
indices cite `file.onnx#N`), used
  * by tests, as the fp32 checker of the HIP engine at sizes the numpy graph
    executor (oracle/onnx_interp.py) is too slow for, and
  * by bench.py's `cpu_baseline` leg ("port": the reference's ONNX-CPU path
    restated on the host cores).
It is itself pinned to the graph executor by tests/test_oracle.py and by the
golden fixtures in tests/golden/.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

T = torch.Tensor


def _t(w: Dict[str, np.ndarray]) -> Dict[str, T]:
    return {k: torch.from_numpy(np.asarray(v, dtype=np.float32).copy()) for k, v in w.items()}


# ------------------------------------------------------------------ T2S
# div_term of the sinusoidal PE (`t2s_encoder_fp32.onnx#70`, `stage#21`): fp32
# exp(-2i ln(1e4)/512), as torch computes it at export.
def pe_div_term(d: int = 512) -> T:
    return torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))


_DIV_OVERRIDE = None


def set_div_term(div) -> None:
    """Use the exact div_term constant of a graph (e.g. tests/golden/pe_div_term.npy)."""
    global _DIV_OVERRIDE
    _DIV_OVERRIDE = None if div is None else torch.as_tensor(np.asarray(div, np.float32))


def sine_pe(positions: T, d: int = 512) -> T:
    """Interleaved sin/cos at 1-based positions (`stage#15-30`): pe[2i]=sin, pe[2i+1]=cos."""
    div = _DIV_OVERRIDE if _DIV_OVERRIDE is not None else pe_div_term(d)
    ang = positions.to(torch.float32).reshape(-1, 1) * div.reshape(1, -1)
    return torch.stack([torch.sin(ang), torch.cos(ang)], dim=-1).reshape(-1, d)


def t2s_encoder(w, ref_seq, text_seq, ref_bert, text_bert, ssl_content):
    """`t2s_encoder_fp32.onnx`: K1 (#49-83) and K2 (#2-48)."""
    w = _t(w) if not isinstance(next(iter(w.values())), torch.Tensor) else w
    ssl = torch.from_numpy(np.asarray(ssl_content, np.float32))
    h = F.conv1d(ssl, w["vits.ssl_proj.weight"], w["vits.ssl_proj.bias"], stride=2)  # #2
    h = h.transpose(1, 2).reshape(-1, 768)                                           # #3,#22
    cb = w["vits.quantizer.vq.layers.0._codebook.embed"]
    dist = (h.pow(2).sum(1, keepdim=True) - (h * 2.0) @ cb.t()) + cb.t().pow(2).sum(0, keepdim=True)
    prompts = torch.argmax(-dist, dim=-1).reshape(1, -1)                             # #35-36
    seq = torch.from_numpy(np.concatenate([ref_seq, text_seq], axis=1).astype(np.int64))
    bert = torch.from_numpy(np.concatenate([ref_bert, text_bert], axis=0).astype(np.float32))
    emb = w["encoder.ar_text_embedding.word_embeddings.weight"][seq[0]]
    x = emb + (w["encoder.bert_proj.bias"] + bert @ w["encoder.bert_proj.weight"].t())
    L = x.shape[0]
    pe = sine_pe(torch.arange(1, L + 1))
    x = x * 1.0 + w["encoder.ar_text_position.alpha"] * pe                            # #81-83
    return x.reshape(1, L, 512), prompts


@dataclass
class T2SLayer:
    w_in: T
    b_in: T
    w_out: T
    b_out: T
    w1: T
    b1: T
    w2: T
    b2: T
    n1w: T
    n1b: T
    n2w: T
    n2b: T


class T2SModel:
    """fp32 weights of `t2s_shared_fp16.bin` (upcast exactly as `g/ModelManager.py:75-76`)."""

    def __init__(self, w):
        w = _t(w)
        self.emb = w["ar_audio_embedding.word_embeddings.weight"]
        self.alpha = w["ar_audio_position.alpha"]
        self.pred = w["ar_predict_layer.weight"]
        self.layers = []
        for i in range(24):
            p = f"transformer_encoder.layers.{i}."
            self.layers.append(T2SLayer(
                w[p + "self_attn.in_proj_weight"], w[p + "self_attn.in_proj_bias"],
                w[p + "self_attn.out_proj.weight"], w[p + "self_attn.out_proj.bias"],
                w[p + "linear1.weight"], w[p + "linear1.bias"],
                w[p + "linear2.weight"], w[p + "linear2.bias"],
                w[p + "norm1.weight"], w[p + "norm1.bias"],
                w[p + "norm2.weight"], w[p + "norm2.bias"]))
        # scale applied to q and k^T separately (`stage#84-93`)
        self.qk_scale = torch.sqrt(torch.tensor(1.0, dtype=torch.float32) /
                                   torch.sqrt(torch.tensor(32.0, dtype=torch.float32)))


def _layer(lw: T2SLayer, h: T, k_all: T, v_all: T, mask: Optional[T], scale: T) -> T:
    """One post-norm layer for query rows h [M,512] over keys k_all/v_all [T,512]."""
    M = h.shape[0]
    Tn = k_all.shape[0]
    q = (h @ lw.w_in[:512].t()) + lw.b_in[:512]
    q = q.reshape(M, 16, 32).transpose(0, 1) * scale                    # [16,M,32]
    k = k_all.reshape(Tn, 16, 32).permute(1, 2, 0) * scale               # [16,32,T]
    v = v_all.reshape(Tn, 16, 32).transpose(0, 1)                        # [16,T,32]
    s = q @ k
    if mask is not None:
        s = s + mask
    p = torch.softmax(s, dim=-1)
    o = (p @ v).permute(1, 0, 2).reshape(M, 512)
    o = o @ lw.w_out.t() + lw.b_out                                      # Gemm #100
    h1 = F.layer_norm(h + o, (512,), lw.n1w, lw.n1b, eps=1e-5)
    f = torch.relu(lw.b1 + h1 @ lw.w1.t())
    f = lw.b2 + f @ lw.w2.t()
    return F.layer_norm(h1 + f, (512,), lw.n2w, lw.n2b, eps=1e-5)


def _kv(lw: T2SLayer, h: T) -> Tuple[T, T]:
    kv = (h @ lw.w_in[512:].t()) + lw.b_in[512:]
    return kv[:, :512], kv[:, 512:]


@dataclass
class SamplerCfg:
    top_k: int = 15
    temperature: float = 1.0
    repetition_penalty: float = 1.35
    eos: int = 1024


def sample(logits: T, history: T, q: T, cfg: SamplerCfg = SamplerCfg()) -> Tuple[int, int]:
    """K10 (`stage#1775-1806`): penalty on every history token, /T, top-k
    threshold, softmax, argmax(p/q).  Returns (token, argmax of raw logits)."""
    l = logits.clone()
    g = logits[history]
    pen = torch.where(g < 0, g * cfg.repetition_penalty, g / cfg.repetition_penalty)
    l[history] = pen
    l = l / cfg.temperature
    thr = torch.topk(l, cfg.top_k).values[-1]
    l = torch.where(l < thr, torch.tensor(float("-inf")), l)
    p = torch.softmax(l, dim=-1)
    tok = int(torch.argmax(p / q))
    return tok, int(torch.argmax(logits))


class T2SState:
    """KV cache + histories of one sequence (prefix x + prompts + generated)."""

    def __init__(self):
        self.k: List[T] = []
        self.v: List[T] = []
        self.y: List[int] = []
        self.y_emb: Optional[T] = None


def t2s_prefill(m: T2SModel, x: T, prompts: np.ndarray, q: T,
                cfg: SamplerCfg = SamplerCfg()) -> Tuple[T2SState, T]:
    """`t2s_first_stage_decoder_fp32.onnx`."""
    x = x.reshape(-1, 512)
    L = x.shape[0]
    pr = torch.from_numpy(np.asarray(prompts, np.int64).reshape(-1))
    P = pr.shape[0]
    y_emb = m.emb[pr]                                                     # #5
    ypos = y_emb + m.alpha * sine_pe(torch.arange(1, P + 1))             # #6-24
    h = torch.cat([x, ypos], 0)
    N = L + P
    mask = torch.zeros(N, N)
    mask[:L, L:] = float("-inf")                                          # #29-56
    mask[L:, L:] = torch.triu(torch.full((P, P), float("-inf")), diagonal=1)
    st = T2SState()
    for lw in m.layers:
        k, v = _kv(lw, h)
        st.k.append(k)
        st.v.append(v)
        h = _layer(lw, h, k, v, mask, m.qk_scale)
    logits = h[-1] @ m.pred.t()
    tok, _ = sample(logits, pr, q, cfg)
    st.y = pr.tolist() + [tok]
    st.y_emb = y_emb
    return st, logits


def t2s_step(m: T2SModel, st: T2SState, q: T, cfg: SamplerCfg = SamplerCfg()) -> Tuple[bool, T]:
    """`t2s_stage_decoder_fp32.onnx`: embed y[-1], PE at position len(y), 24 layers, K10."""
    last = st.y[-1]
    e = m.emb[last].reshape(1, 512)
    st.y_emb = torch.cat([st.y_emb, e], 0)
    n = st.y_emb.shape[0]
    h = e + m.alpha * sine_pe(torch.tensor([n]))
    for i, lw in enumerate(m.layers):
        k, v = _kv(lw, h)
        st.k[i] = torch.cat([st.k[i], k], 0)
        st.v[i] = torch.cat([st.v[i], v], 0)
        h = _layer(lw, h, st.k[i], st.v[i], None, m.qk_scale)
    logits = h[0] @ m.pred.t()
    hist = torch.tensor(st.y, dtype=torch.int64)
    tok, raw_arg = sample(logits, hist, q, cfg)
    st.y.append(tok)
    stop = raw_arg == cfg.eos or tok == cfg.eos
    return stop, logits


def trim_tokens(y: List[int], idx: int) -> np.ndarray:
    """`g/Core/Inference.py:108-109` then `:41-44` (EOS filter)."""
    arr = np.asarray(y, dtype=np.int64).reshape(1, -1).copy()
    arr[0, -1] = 0
    sem = np.expand_dims(arr[:, -idx:], axis=0)
    eos = np.where(sem >= 1024)
    if len(eos[0]) > 0:
        sem = sem[..., :eos[-1][0]]
    return sem


def t2s_generate(w_enc, m: T2SModel, ref_seq, ref_bert, text_seq, text_bert, ssl_content,
                 cfg: SamplerCfg = SamplerCfg(), max_steps: int = 500,
                 force_steps: Optional[int] = None, q_fn=None):
    """`GENIE.t2s_cpu` (`g/Core/Inference.py:63-109`) + EOS filter; greedy when q_fn is None."""
    x, prompts = t2s_encoder(w_enc, ref_seq, text_seq, ref_bert, text_bert, ssl_content)
    ones = torch.ones(1025)
    st, _ = t2s_prefill(m, x, prompts.numpy(), ones if q_fn is None else q_fn(-1), cfg)
    idx = 0
    n_iter = max_steps if force_steps is None else force_steps
    for idx in range(n_iter):
        stop, _ = t2s_step(m, st, ones if q_fn is None else q_fn(idx), cfg)
        if force_steps is None and stop:
            break
    return trim_tokens(st.y, idx), st, prompts


# ------------------------------------------------------------------ VITS
def fold_weight_norm(w: Dict[str, T]) -> Dict[str, T]:
    """w = (v / ||v||_2 over dims 1..) * g (`vits_fp32.onnx` ReduceL2 -> Div -> Mul)."""
    out = dict(w)
    for k in list(w):
        if k.endswith(".weight_v"):
            base = k[: -len("weight_v")]
            v = w[k]
            g = w[base + "weight_g"]
            nrm = torch.sqrt((v.double() ** 2).sum(dim=(1, 2), keepdim=True)).float()
            out[base + "weight"] = (v / nrm) * g
    return out


def _ln_ch(x: T, g: T, b: T) -> T:
    return F.layer_norm(x.transpose(1, -1), (x.shape[1],), g, b, 1e-5).transpose(1, -1)


def _conv(x, w, b=None, pad=0, dil=1, stride=1):
    return F.conv1d(x, w, b, stride=stride, padding=pad, dilation=dil)


def _rel_attn(x: T, w: Dict[str, T], pre: str, heads: int, window: int) -> T:
    """attentions.MultiHeadAttention with relative keys/values (window 4)."""
    q = _conv(x, w[pre + "conv_q.weight"], w[pre + "conv_q.bias"])
    k = _conv(x, w[pre + "conv_k.weight"], w[pre + "conv_k.bias"])
    v = _conv(x, w[pre + "conv_v.weight"], w[pre + "conv_v.bias"])
    b, d, t = q.shape
    dk = d // heads
    q = q.view(b, heads, dk, t).transpose(2, 3)
    k = k.view(b, heads, dk, t).transpose(2, 3)
    v = v.view(b, heads, dk, t).transpose(2, 3)
    qs = q / math.sqrt(dk)
    scores = qs @ k.transpose(-2, -1)
    ek = w[pre + "emb_rel_k"][0]          # [2W+1, dk]
    ev = w[pre + "emb_rel_v"][0]
    # scores_local[i, j] = qs_i . ek[j - i + W] for |j-i| <= W
    rel = qs @ ek.t()                     # [b,h,t,2W+1]
    loc = torch.zeros_like(scores)
    for r in range(-window, window + 1):
        n = t - abs(r)
        if n <= 0:
            continue
        i = torch.arange(max(0, -r), max(0, -r) + n)
        loc[:, :, i, i + r] = rel[:, :, i, r + window]
    scores = scores + loc
    p = torch.softmax(scores, dim=-1)
    o = p @ v
    for r in range(-window, window + 1):
        n = t - abs(r)
        if n <= 0:
            continue
        i = torch.arange(max(0, -r), max(0, -r) + n)
        o[:, :, i, :] += p[:, :, i, i + r].unsqueeze(-1) * ev[r + window]
    o = o.transpose(2, 3).contiguous().view(b, d, t)
    return _conv(o, w[pre + "conv_o.weight"], w[pre + "conv_o.bias"])


def _attn_encoder(x: T, w, pre: str, n: int) -> T:
    for i in range(n):
        y = _rel_attn(x, w, f"{pre}.attn_layers.{i}.", 2, 4)
        x = _ln_ch(x + y, w[f"{pre}.norm_layers_1.{i}.gamma"], w[f"{pre}.norm_layers_1.{i}.beta"])
        f = _conv(x, w[f"{pre}.ffn_layers.{i}.conv_1.weight"], w[f"{pre}.ffn_layers.{i}.conv_1.bias"], pad=1)
        f = torch.relu(f)
        f = _conv(f, w[f"{pre}.ffn_layers.{i}.conv_2.weight"], w[f"{pre}.ffn_layers.{i}.conv_2.bias"], pad=1)
        x = _ln_ch(x + f, w[f"{pre}.norm_layers_2.{i}.gamma"], w[f"{pre}.norm_layers_2.{i}.beta"])
    return x


def _mha_plain(xq: T, xkv: T, w, pre: str, heads: int) -> T:
    q = _conv(xq, w[pre + "conv_q.weight"], w[pre + "conv_q.bias"])
    k = _conv(xkv, w[pre + "conv_k.weight"], w[pre + "conv_k.bias"])
    v = _conv(xkv, w[pre + "conv_v.weight"], w[pre + "conv_v.bias"])
    b, d, tq = q.shape
    tk = k.shape[2]
    dk = d // heads
    q = q.view(b, heads, dk, tq).transpose(2, 3)
    k = k.view(b, heads, dk, tk).transpose(2, 3)
    v = v.view(b, heads, dk, tk).transpose(2, 3)
    p = torch.softmax((q / math.sqrt(dk)) @ k.transpose(-2, -1), dim=-1)
    o = (p @ v).transpose(2, 3).contiguous().view(b, d, tq)
    return _conv(o, w[pre + "conv_o.weight"], w[pre + "conv_o.bias"])


def mish(x: T) -> T:
    return x * torch.tanh(F.softplus(x))


def spectrogram(audio: T) -> T:
    """`vits_fp32.onnx(v2)#26-55`: reflect pad 704, STFT(2048, hop 640, hann), |.|."""
    y = F.pad(audio.reshape(1, 1, -1), (704, 704), mode="reflect").reshape(1, -1)
    win = torch.hann_window(2048, periodic=True, dtype=torch.float32)
    s = torch.stft(y, 2048, hop_length=640, win_length=2048, window=win, center=False,
                   onesided=True, return_complex=True)
    s = torch.view_as_real(s)
    return torch.sqrt(s.pow(2).sum(-1) + 1e-6)       # [1, 1025, frames]


def ref_encoder(spec: T, w, pre: str) -> T:
    """MelStyleEncoder (`vits_fp32.onnx(v2)#79-271`): -> ge [1, out, 1]."""
    x = spec[:, :704].transpose(1, 2)                 # [1, T, 704]
    x = mish(x @ w[pre + "spectral.0.fc.weight"].t() + w[pre + "spectral.0.fc.bias"])
    x = mish(x @ w[pre + "spectral.3.fc.weight"].t() + w[pre + "spectral.3.fc.bias"])
    x = x.transpose(1, 2)
    for i in range(2):
        r = x
        h = _conv(x, w[pre + f"temporal.{i}.conv1.conv.weight"],
                  w[pre + f"temporal.{i}.conv1.conv.bias"], pad=2)
        a, g = h[:, :128], h[:, 128:]
        x = r + a * torch.sigmoid(g)
    x = x.transpose(1, 2)                              # [1, T, 128]
    res = x
    B, Tn, _ = x.shape
    q = (x @ w[pre + "slf_attn.w_qs.weight"].t() + w[pre + "slf_attn.w_qs.bias"]).view(B, Tn, 2, 64)
    k = (x @ w[pre + "slf_attn.w_ks.weight"].t() + w[pre + "slf_attn.w_ks.bias"]).view(B, Tn, 2, 64)
    v = (x @ w[pre + "slf_attn.w_vs.weight"].t() + w[pre + "slf_attn.w_vs.bias"]).view(B, Tn, 2, 64)
    q = q.permute(2, 0, 1, 3).reshape(-1, Tn, 64)
    k = k.permute(2, 0, 1, 3).reshape(-1, Tn, 64)
    v = v.permute(2, 0, 1, 3).reshape(-1, Tn, 64)
    a = torch.bmm(q, k.transpose(1, 2)) / math.sqrt(128.0)
    a = torch.softmax(a, dim=2)
    o = torch.bmm(a, v).view(2, B, Tn, 64).permute(1, 2, 0, 3).reshape(B, Tn, 128)
    o = o @ w[pre + "slf_attn.fc.weight"].t() + w[pre + "slf_attn.fc.bias"]
    x = o + res
    x = x @ w[pre + "fc.fc.weight"].t() + w[pre + "fc.fc.bias"]
    return (x.sum(dim=1) / float(Tn)).unsqueeze(-1)


class VitsModel:
    def __init__(self, w, version: str):
        from genie_tts_amd.weights import vits_config
        self.cfg = vits_config(version)
        self.version = version
        self.w = fold_weight_norm(_t(w))

    def text_encoder(self, sem: np.ndarray, text_seq: np.ndarray, ge_mrte: T):
        """enc_p (`(v2)#273-6489`) -> (m_p, logs_p) [1,192,2G]."""
        w = self.w
        p = "vq_model.enc_p."
        codes = torch.from_numpy(np.asarray(sem, np.int64)).reshape(-1)
        q = w["vq_model.quantizer.vq.layers.0._codebook.embed"][codes].t().unsqueeze(0)  # [1,768,G]
        q = torch.repeat_interleave(q, 2, dim=2)                                          # x2
        y = _conv(q, w[p + "ssl_proj.weight"], w[p + "ssl_proj.bias"])
        y = _attn_encoder(y, w, p + "encoder_ssl", self.cfg.n_ssl_layers)
        t = torch.from_numpy(np.asarray(text_seq, np.int64)).reshape(-1)
        te = w[p + "text_embedding.weight"][t].t().unsqueeze(0)
        te = _attn_encoder(te, w, p + "encoder_text", self.cfg.n_text_layers)
        m = p + "mrte."
        ssl_enc = _conv(y, w[m + "c_pre.weight"], w[m + "c_pre.bias"])
        text_enc = _conv(te, w[m + "text_pre.weight"], w[m + "text_pre.bias"])
        x = _mha_plain(ssl_enc, text_enc, w, m + "cross_attention.", 4) + ssl_enc + ge_mrte
        y = _conv(x, w[m + "c_post.weight"], w[m + "c_post.bias"])
        y = _attn_encoder(y, w, p + "encoder2", self.cfg.n_enc2_layers)
        stats = _conv(y, w[p + "proj.weight"], w[p + "proj.bias"])
        return stats[:, :192], stats[:, 192:]

    def flow_reverse(self, z: T, ge: T) -> T:
        w = self.w
        for f in (6, 4, 2, 0):
            z = torch.flip(z, [1])                     # Flip layers 7,5,3,1
            fp = f"vq_model.flow.flows.{f}."
            x0, x1 = z[:, :96], z[:, 96:]
            h = _conv(x0, w[fp + "pre.weight"], w[fp + "pre.bias"])
            g = _conv(ge, w[fp + "enc.cond_layer.weight"], w[fp + "enc.cond_layer.bias"])
            out = torch.zeros_like(h)
            for l in range(4):
                xin = _conv(h, w[fp + f"enc.in_layers.{l}.weight"], w[fp + f"enc.in_layers.{l}.bias"], pad=2)
                a = xin + g[:, l * 384:(l + 1) * 384]
                acts = torch.tanh(a[:, :192]) * torch.sigmoid(a[:, 192:])
                rs = _conv(acts, w[fp + f"enc.res_skip_layers.{l}.weight"], w[fp + f"enc.res_skip_layers.{l}.bias"])
                if l < 3:
                    h = h + rs[:, :192]
                    out = out + rs[:, 192:]
                else:
                    out = out + rs
            mstat = _conv(out, w[fp + "post.weight"], w[fp + "post.bias"])
            x1 = (x1 - mstat)
            z = torch.cat([x0, x1], 1)
        return z

    def generator(self, z: T, ge: T) -> T:
        w = self.w
        c = self.cfg
        d = "vq_model.dec."
        x = _conv(z, w[d + "conv_pre.weight"], w[d + "conv_pre.bias"], pad=3)
        x = x + _conv(ge, w[d + "cond.weight"], w[d + "cond.bias"])
        nk = len(c.rb_kernels)
        for i, (u, k) in enumerate(zip(c.up_rates, c.up_kernels)):
            x = F.leaky_relu(x, 0.1)
            x = F.conv_transpose1d(x, w[d + f"ups.{i}.weight"], w[d + f"ups.{i}.bias"],
                                   stride=u, padding=(k - u) // 2)
            xs = None
            for j, kk in enumerate(c.rb_kernels):
                rb = d + f"resblocks.{i * nk + j}."
                r = x
                for m_, dil in enumerate(c.rb_dilations):
                    xt = F.leaky_relu(r, 0.1)
                    xt = _conv(xt, w[rb + f"convs1.{m_}.weight"], w[rb + f"convs1.{m_}.bias"],
                               pad=(kk * dil - dil) // 2, dil=dil)
                    xt = F.leaky_relu(xt, 0.1)
                    xt = _conv(xt, w[rb + f"convs2.{m_}.weight"], w[rb + f"convs2.{m_}.bias"],
                               pad=(kk - 1) // 2)
                    r = xt + r
                xs = r if xs is None else xs + r
            x = xs / float(nk)
        x = F.leaky_relu(x, 0.01)
        x = _conv(x, w[d + "conv_post.weight"], None, pad=3)
        return torch.tanh(x)

    def __call__(self, text_seq, pred_semantic, ref_audio=None, ge=None, ge_advanced=None,
                 eps: Optional[np.ndarray] = None, noise_scale: float = 0.5):
        if self.version == "v2":
            spec = spectrogram(torch.from_numpy(np.asarray(ref_audio, np.float32)))
            ge_t = ref_encoder(spec, self.w, "vq_model.ref_enc.")
            ge_m = ge_t
        else:
            ge_t = torch.from_numpy(np.asarray(ge, np.float32))
            ge_m = torch.from_numpy(np.asarray(ge_advanced, np.float32))
        m_p, logs_p = self.text_encoder(pred_semantic, text_seq, ge_m)
        e = torch.zeros_like(m_p) if eps is None else torch.from_numpy(np.asarray(eps, np.float32))
        z_p = m_p + (e * torch.exp(logs_p)) * noise_scale
        z = self.flow_reverse(z_p, ge_t)
        o = self.generator(z, ge_t)
        self.last = dict(ge=ge_t, m_p=m_p, logs_p=logs_p, z=z)
        return o[0, 0]


def prompt_encoder(w, ref_audio, sv_emb):
    """`prompt_encoder_fp32.onnx`: ref_enc(->1024) + sv_emb Gemm, PReLU, ge_to512."""
    w = _t(w)
    spec = spectrogram(torch.from_numpy(np.asarray(ref_audio, np.float32)))
    ge = ref_encoder(spec, w, "ref_enc.")
    sv = torch.from_numpy(np.asarray(sv_emb, np.float32))
    ge = ge + (sv @ w["sv_emb.weight"].t() + w["sv_emb.bias"]).unsqueeze(-1)
    ge = torch.where(ge >= 0, ge, ge * w["prelu.weight"].reshape(1, -1, 1))
    adv = (ge.transpose(2, 1) @ w["ge_to512.weight"].t() + w["ge_to512.bias"]).transpose(2, 1)
    return ge, adv
