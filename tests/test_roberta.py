"""CPU: the RoBERTa weight layout against transformers' BertModel and the inline
initializer reader (RoBERTa.onnx keeps its weights in the graph file,
ModelManager.py:139)."""
import numpy as np

from genie_tts_amd import weights as W


def test_spec_matches_bert_model_state_dict():
    from transformers import BertConfig, BertModel
    m = BertModel(BertConfig(vocab_size=21128, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                             intermediate_size=4096, layer_norm_eps=1e-12), add_pooling_layer=False)
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    spec = W.roberta_spec()
    assert set(spec) == set(sd) - {"embeddings.position_ids", "embeddings.token_type_ids"} or set(spec) <= set(sd)
    for k, s in spec.items():
        assert sd[k] == s, k


def test_inline_initializer_reader(tmp_path):
    from genie_tts_amd.onnx_table import read_initializer_values
    from tests.onnx_writer import model_inline
    spec = {"a.weight": (3, 4), "b.bias": (5,)}
    arrs = {"a.weight": np.arange(12, dtype=np.float32).reshape(3, 4), "b.bias": np.ones(5, np.float16),
            "unused": np.zeros(2, np.float32)}
    p = tmp_path / "RoBERTa.onnx"
    p.write_bytes(model_inline(arrs))
    got = read_initializer_values(str(p), spec)
    np.testing.assert_array_equal(got["a.weight"], arrs["a.weight"])
    assert got["b.bias"].dtype == np.float16 and got["b.bias"].shape == (5,)
