"""CPU: the SV oracle (oracle/sv.py) and the SV weight table (weights.sv_spec).

The Kaldi fbank restatement is checked against a second, independent one (numpy,
float64, direct DFT over the frame instead of torch.fft), and every sv_spec tensor
must be read by the ERes2NetV2 restatement (and nothing else).  Parity with the
absent speaker_encoder.onnx stays unpinned."""
import numpy as np
import pytest

from genie_tts_amd import synth, weights as W
from oracle import sv as S


def _fbank_f64(wav):
    x = np.asarray(wav, np.float64)
    T = 1 + (len(x) - 400) // 160
    out = np.empty((T, 80))
    n = np.arange(400)
    win = (0.5 - 0.5 * np.cos(2 * np.pi * n / 399)) ** 0.85
    k = np.arange(257)[:, None]
    basis = np.exp(-2j * np.pi * k * n[None, :] / 512)
    banks = S.mel_banks().astype(np.float64)
    for t in range(T):
        f = x[160 * t:160 * t + 400].copy()
        f -= f.mean()
        f = (f - 0.97 * np.concatenate([f[:1], f[:-1]])) * win
        p = np.abs(basis @ f) ** 2
        out[t] = np.log(np.maximum(banks @ p, np.finfo(np.float32).eps))
    return out


def test_fbank_matches_independent_restatement():
    r = synth.rng_for("sv-fb")
    a = (0.3 * np.sin(np.arange(8000) * 0.07) + 0.05 * r.standard_normal(8000)).astype(np.float32)
    got = S.fbank(a).numpy()
    want = _fbank_f64(a)
    assert got.shape == want.shape == (S.n_frames(8000), 80)
    assert np.abs(got - want).max() < 2e-3, np.abs(got - want).max()


def test_fbank_silence_is_log_eps():
    f = S.fbank(np.zeros(1200, np.float32)).numpy()
    assert np.allclose(f, np.log(np.finfo(np.float32).eps))


def test_mel_banks_shape_and_support():
    b = S.mel_banks()
    assert b.shape == (80, 257)
    assert np.all(b[:, 256] == 0) and np.all(b >= 0) and np.all(b <= 1)
    assert np.all(b.sum(axis=1) > 0)
    assert np.all(b[:, 0] == 0)          # 0 Hz is below the 20 Hz low edge


@pytest.mark.parametrize("n,T", [(399, 0), (400, 1), (559, 1), (560, 2), (89600, 558)])
def test_frame_count(n, T):
    assert S.n_frames(n) == T


class _Track(dict):
    def __init__(self, d):
        super().__init__(d)
        self.read = set()

    def __getitem__(self, k):
        self.read.add(k)
        return super().__getitem__(k)


def test_spec_is_exactly_what_the_model_reads():
    import torch
    w = synth.synth_sv_weights()
    spec = W.sv_spec()
    assert list(w) == list(spec)
    for k, shp in spec.items():
        assert w[k].shape == shp and w[k].dtype == np.float32
    tw = _Track(S.torch_weights(w))
    feat = torch.from_numpy(np.random.default_rng(0).standard_normal((17, 80)).astype(np.float32))
    out = S.forward3(tw, feat)
    assert out.shape == (1, 20480)
    assert tw.read == set(spec)
    assert np.all(w["layer1.0.bn1.running_var"] > 0)


def test_embedding_depends_on_audio():
    w = synth.synth_sv_weights()
    r = synth.rng_for("sv-dep")
    a = (0.1 * r.standard_normal(4000)).astype(np.float32)
    e1 = S.sv_embedding(w, a)
    e2 = S.sv_embedding(w, a * 0.5)
    assert e1.shape == (1, 20480) and np.isfinite(e1).all()
    assert np.abs(e1 - e2).max() > 1e-3


def test_sv_loader_reads_speaker_encoder_onnx(tmp_path):
    """load_sv_weights reads GenieData's speaker_encoder.onnx (inline fp32 initializers,
    ModelManager.py:155-170) by sv_spec names, from the file or its directory; tensors
    the model does not use are ignored (written here by tests/onnx_writer.py)."""
    from tests.onnx_writer import model_inline
    w = synth.synth_sv_weights()
    arrs = dict(w)
    arrs["seg_1.weight"] = np.zeros((192, 8), np.float32)       # the pooling head forward3 skips
    (tmp_path / "speaker_encoder.onnx").write_bytes(model_inline(arrs))
    for path in (str(tmp_path / "speaker_encoder.onnx"), str(tmp_path)):
        got = W.load_sv_weights(path)
        assert list(got) == list(W.sv_spec())
        for k in ("conv1.weight", "layer4.2.fuse_models.2.local_att.4.running_var", "fuse34.local_att.3.weight"):
            np.testing.assert_array_equal(np.asarray(got[k], np.float32), w[k])


def test_sv_loader_reads_renamed_exports(tmp_path):
    """speaker_encoder.onnx exports that renamed the initializers
    (onnx::Conv_N) are read by Conv node order: with BatchNormalization nodes the
    state-dict tensors come back exactly; with BatchNorm folded into the convs the
    oracle's forward over the loaded tensors equals the unfolded model's."""
    from tests.sv_export import export
    w = synth.synth_sv_weights()
    p = str(tmp_path / "bn.onnx")
    export(w, p, folded=False)
    got = W.load_sv_weights(p)
    assert set(got) == set(W.sv_spec()) and all(np.array_equal(got[k], w[k]) for k in got)
    p = str(tmp_path / "folded.onnx")
    export(w, p, folded=True)
    got = W.load_sv_weights(p)
    assert not any(k.endswith("running_var") for k in got) and "layer1.0.conv1.bias" in got
    a = (0.1 * synth.rng_for("sv-fold").standard_normal(16000)).astype(np.float32)
    ref, fol = S.sv_embedding(w, a), S.sv_embedding(got, a)
    # fp32 folding reorders the rounding; a wrong conv mapping would differ by O(1)
    rel = float(np.sqrt(np.mean((fol - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))
    assert rel <= 1e-4, rel


def test_sv_loader_names_what_is_missing(tmp_path):
    from tests.onnx_writer import model_graph
    p = str(tmp_path / "bad.onnx")
    with open(p, "wb") as f:
        f.write(model_graph({"onnx::Conv_0": np.zeros((64, 1, 3, 3), np.float32)},
                            [("Conv", ["x", "onnx::Conv_0"], ["y"], "/conv1/Conv")]))
    with pytest.raises(KeyError, match="conv1.weight|missing"):
        W.load_sv_weights(p)
