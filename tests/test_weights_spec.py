"""CPU: weight tables vs the reference templates, and the Genie on-disk format
(fp16 bins addressed through the relinked graph's fp32 offsets,
g/ModelManager.py:59-114) read back through genie_tts_amd.weights."""
import os

import numpy as np
import pytest

from genie_tts_amd import synth, weights as W
from tests.onnx_writer import model

REF = "/root/reference/src/genie_tts/Data"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference templates not present")
@pytest.mark.parametrize("rel,spec", [
    ("v2/Models/t2s_first_stage_decoder_fp32.onnx", W.t2s_spec),
    ("v2/Models/t2s_stage_decoder_fp32.onnx", W.t2s_spec),
    ("v2/Models/t2s_encoder_fp32.onnx", W.t2s_encoder_spec),
    ("v2/Models/vits_fp32.onnx", lambda: W.vits_spec("v2")),
    ("v2ProPlus/Models/vits_fp32.onnx", lambda: W.vits_spec("v2ProPlus")),
    ("v2ProPlus/Models/prompt_encoder_fp32.onnx", W.prompt_encoder_spec),
])
def test_spec_matches_template(rel, spec):
    from genie_tts_amd.onnx_table import read_initializer_table
    table = read_initializer_table(os.path.join(REF, rel))
    s = spec()
    assert set(table) == set(s)
    for name, shape in s.items():
        assert tuple(table[name][0]) == tuple(shape), name


def test_param_counts():
    assert W.spec_numel(W.t2s_spec()) == 76_706_817
    assert W.spec_numel(W.vits_spec("v2")) == 40_421_760
    assert W.spec_numel(W.vits_spec("v2ProPlus")) == 62_172_928
    assert W.spec_numel(W.prompt_encoder_spec()) == 22_131_456


def _write_char_dir(d, version, w):
    """Write a character directory in Genie's format from weight dicts."""
    def fp16_bin(fname, onnx_name, spec, arrays):
        lay = W.layout_offsets(spec, 4)          # offsets describe the fp32 upcast
        np.concatenate([np.asarray(arrays[n], np.float16).reshape(-1) for n in spec]).tofile(os.path.join(d, fname))
        inits = [(n, list(spec[n]), off, ln) for n, off, ln in lay]
        with open(os.path.join(d, onnx_name), "wb") as f:
            f.write(model(inits, fname))
    fp16_bin("t2s_shared_fp16.bin", "t2s_first_stage_decoder_fp32.onnx", W.t2s_spec(), w["t2s"])
    fp16_bin("t2s_shared_fp16.bin", "t2s_stage_decoder_fp32.onnx", W.t2s_spec(), w["t2s"])
    fp16_bin("vits_fp16.bin", "vits_fp32.onnx", W.vits_spec(version), w["vits"])
    es = W.t2s_encoder_spec()
    lay = W.layout_offsets(es, 4)
    np.concatenate([np.asarray(w["t2s_encoder"][n], np.float32).reshape(-1) for n in es]).tofile(
        os.path.join(d, "t2s_encoder_fp32.bin"))
    with open(os.path.join(d, "t2s_encoder_fp32.onnx"), "wb") as f:
        f.write(model([(n, list(es[n]), off, ln) for n, off, ln in lay], "t2s_encoder_fp32.bin"))
    if version != "v2":
        fp16_bin("prompt_encoder_fp16.bin", "prompt_encoder_fp32.onnx", W.prompt_encoder_spec(), w["prompt_encoder"])


@pytest.mark.parametrize("version", ["v2", "v2ProPlus"])
def test_character_dir_roundtrip(tmp_path, version):
    w = synth.synthetic_character(version)
    _write_char_dir(str(tmp_path), version, w)
    ver, got = W.load_character_weights(str(tmp_path))
    assert ver == version
    for group in w:
        for name, arr in w[group].items():
            np.testing.assert_array_equal(np.asarray(got[group][name], np.float32), np.asarray(arr, np.float32))


def test_missing_files_error(tmp_path):
    with pytest.raises(FileNotFoundError, match="missing base files"):
        W.load_character_weights(str(tmp_path))
