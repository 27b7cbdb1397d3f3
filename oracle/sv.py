"""Speaker-verification (SV) oracle (TEST INFRASTRUCTURE ONLY: imported by tests/ and nothing else).

The reference runs, once per V2ProPlus reference clip,
    sv_emb = model_manager.speaker_verification_model.run(None, {'waveform': audio_16k})[0]
(`g/Audio/ReferenceAudio.py:68-76`, session loaded at `g/ModelManager.py:155-170`),
and feeds the [1, 20480] result to the prompt encoder's `sv_emb` input
(`prompt_encoder_fp32.onnx#269`).  `speaker_encoder.onnx` is a GenieData download
that is absent here, and so is its source.  It is GPT-SoVITS's v2Pro speaker
model, `SV.compute_embedding3` (GPT_SoVITS/sv.py) over 3D-Speaker's ERes2NetV2:

    feat   = Kaldi.fbank(wav, num_mel_bins=80, sample_frequency=16000, dither=0)   [T, 80]
    sv_emb = ERes2NetV2(baseWidth=24, scale=4, expansion=4).forward3(feat[None])    [1, 20480]

This module restates both from their published definitions (torchaudio's
compliance.kaldi.fbank defaults; ERes2NetV2 with m_channels=64, blocks [3,4,6,3],
Res2Net-style split convs with AFF fusion in stages 3-4, layer3_ds + fuse34, and
forward3's flatten(1, 2).mean(-1) over time), in torch fp32 with BatchNorm in
eval mode.  Parity at the ONNX level is UNPINNED: no graph, no weights and no
fixture of the real model exist offline, and torchaudio is not installed here.
The engine (`genie_tts_amd/csrc/sv.hip`) is checked against this restatement.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

SAMPLE_RATE = 16000
N_MELS = 80
FRAME_LEN = 400        # 25 ms
FRAME_SHIFT = 160      # 10 ms
N_FFT = 512            # round_to_power_of_two(400)
EPS = float(torch.finfo(torch.float32).eps)
BN_EPS = 1e-5

# (planes, blocks, first stride, AFF fusion) per stage; width = floor(planes * 24 / 64), scale 4, expansion 4
STAGES = ((64, 3, 1, False), (128, 4, 2, False), (256, 6, 2, True), (512, 3, 2, True))
BASE_WIDTH, SCALE, EXPANSION, M_CHANNELS = 24, 4, 4, 64


def n_frames(n_samples: int) -> int:
    """Kaldi frames with snip_edges=True."""
    return 0 if n_samples < FRAME_LEN else 1 + (n_samples - FRAME_LEN) // FRAME_SHIFT


def mel_banks() -> np.ndarray:
    """[80, 257] triangular Kaldi mel filters (low 20 Hz, high = Nyquist, no VTLN),
    torchaudio.compliance.kaldi.get_mel_banks + its zero Nyquist column."""
    def mel(f):
        return 1127.0 * np.log(1.0 + np.asarray(f, np.float64) / 700.0)
    lo, hi = mel(20.0), mel(SAMPLE_RATE / 2)
    delta = (hi - lo) / (N_MELS + 1)
    b = np.arange(N_MELS, dtype=np.float64)[:, None]
    left, center, right = lo + b * delta, lo + (b + 1) * delta, lo + (b + 2) * delta
    m = mel(np.arange(N_FFT // 2, dtype=np.float64) * (SAMPLE_RATE / N_FFT))[None, :]
    up = (m - left) / (center - left)
    down = (right - m) / (right - center)
    banks = np.maximum(0.0, np.minimum(up, down))
    return np.concatenate([banks, np.zeros((N_MELS, 1))], axis=1).astype(np.float32)


@torch.no_grad()
def fbank(wav: np.ndarray) -> torch.Tensor:
    """Kaldi.fbank(wav[None], num_mel_bins=80, sample_frequency=16000, dither=0):
    frames of 400 (shift 160, snip edges) -> remove DC -> pre-emphasis 0.97 (first
    sample against itself) -> povey window (hann(400, periodic=False)^0.85) -> zero
    pad to 512 -> |rfft|^2 -> mel banks -> log(max(., float32 eps)).  [T, 80] f32."""
    x = torch.from_numpy(np.asarray(wav, np.float32).reshape(-1))
    T = n_frames(x.numel())
    fr = x.as_strided((T, FRAME_LEN), (FRAME_SHIFT, 1))
    fr = fr - fr.mean(dim=1, keepdim=True)
    prev = torch.cat([fr[:, :1], fr[:, :-1]], dim=1)
    fr = fr - 0.97 * prev
    win = torch.hann_window(FRAME_LEN, periodic=False, dtype=torch.float32).pow(0.85)
    fr = F.pad(fr * win, (0, N_FFT - FRAME_LEN))
    power = torch.fft.rfft(fr).abs().pow(2.0)
    mel = power @ torch.from_numpy(mel_banks()).T
    return torch.clamp_min(mel, EPS).log()


def _bn(x, w, p):
    if p + ".weight" not in w:     # an export with BatchNorm folded into the conv (its bias)
        return x
    return F.batch_norm(x, w[p + ".running_mean"], w[p + ".running_var"], w[p + ".weight"], w[p + ".bias"],
                        training=False, eps=BN_EPS)


def _relu20(x):
    return torch.clamp(x, 0.0, 20.0)    # the blocks' ReLU is nn.Hardtanh(0, 20)


def _aff(w, p, x, y):
    """AFF(x, ds_y): att = 1 + tanh(BN(conv(SiLU(BN(conv(cat(x, y))))))), x att + y (2 - att)."""
    a = F.conv2d(torch.cat([x, y], 1), w[p + ".local_att.0.weight"], w[p + ".local_att.0.bias"])
    a = F.silu(_bn(a, w, p + ".local_att.1"))
    a = F.conv2d(a, w[p + ".local_att.3.weight"], w[p + ".local_att.3.bias"])
    a = 1.0 + torch.tanh(_bn(a, w, p + ".local_att.4"))
    return x * a + y * (2.0 - a)


def _block(w, p, x, planes, stride, aff):
    width = int(math.floor(planes * (BASE_WIDTH / 64.0)))
    out = _relu20(_bn(F.conv2d(x, w[p + ".conv1.weight"], w.get(p + ".conv1.bias"), stride=stride), w, p + ".bn1"))
    spx = torch.split(out, width, 1)
    outs = []
    sp = None
    for i in range(SCALE):
        if i == 0:
            sp = spx[0]
        elif aff:
            sp = _aff(w, f"{p}.fuse_models.{i - 1}", sp, spx[i])
        else:
            sp = sp + spx[i]
        sp = _relu20(_bn(F.conv2d(sp, w[f"{p}.convs.{i}.weight"], w.get(f"{p}.convs.{i}.bias"), padding=1), w, f"{p}.bns.{i}"))
        outs.append(sp)
    out = _bn(F.conv2d(torch.cat(outs, 1), w[p + ".conv3.weight"], w.get(p + ".conv3.bias")), w, p + ".bn3")
    if p + ".shortcut.0.weight" in w:
        res = _bn(F.conv2d(x, w[p + ".shortcut.0.weight"], w.get(p + ".shortcut.0.bias"), stride=stride), w, p + ".shortcut.1")
    else:
        res = x
    return _relu20(out + res)


@torch.no_grad()
def forward3(w: Dict[str, torch.Tensor], feat: torch.Tensor) -> torch.Tensor:
    """ERes2NetV2.forward3 on feat [T, 80] -> [1, 20480] (channel-major c * 10 + f)."""
    x = feat.T.contiguous()[None, None]                       # (B, 1, F=80, T)
    out = F.relu(_bn(F.conv2d(x, w["conv1.weight"], w.get("conv1.bias"), padding=1), w, "bn1"))
    outs = []
    for s, (planes, nb, stride, aff) in enumerate(STAGES, start=1):
        for b in range(nb):
            out = _block(w, f"layer{s}.{b}", out, planes, stride if b == 0 else 1, aff)
        outs.append(out)
    out3_ds = F.conv2d(outs[2], w["layer3_ds.weight"], w.get("layer3_ds.bias"), stride=2, padding=1)
    fuse = _aff(w, "fuse34", outs[3], out3_ds)
    return torch.flatten(fuse, start_dim=1, end_dim=2).mean(-1)


def torch_weights(w: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.asarray(v, np.float32).copy()) for k, v in w.items()}


def sv_embedding(w: Dict[str, np.ndarray], audio_16k: np.ndarray) -> np.ndarray:
    """speaker_encoder.run(None, {'waveform': audio_16k})[0]: [1, 20480] f32."""
    return forward3(torch_weights(w), fbank(audio_16k)).numpy()
