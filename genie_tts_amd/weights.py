"""Weight tables for the GPT-SoVITS graphs Genie ships, and the Genie on-disk format.

The reference keeps model *structure* in ONNX templates and model *values* in
header-less fp16 bins written by its converter in key-file order
(`g/Converter/v2/T2SConverter.py:45-111`, `VITSConverter.py:44-112`,
`EncoderConverter.py:38-106`, `v2ProPlus/PromptEncoderConverter.py:43-123`);
at load time it upcasts the bin to fp32 and patches each EXTERNAL initializer
from its (offset, length) in the fp32 layout (`g/ModelManager.py:59-114`).

This module re-derives the name -> shape table of every graph from the model
hyper-parameters (no template needed at run time), and reads real character
directories through the same (offset, length) contract.  `tests/test_weights_spec.py`
checks the derived tables against the shipped templates name-for-name.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

Spec = "OrderedDict[str, Tuple[int, ...]]"

# --------------------------------------------------------------------- T2S
T2S_LAYERS = 24
T2S_D = 512
T2S_FF = 2048
T2S_HEADS = 16
T2S_VOCAB = 1025          # semantic tokens, EOS = 1024
T2S_EOS = 1024
TEXT_VOCAB = 732          # symbols_v2 (g/G2P/SymbolsV2.py:100-119)
BERT_DIM = 1024           # g/Utils/Language.py BERT_FEATURE_DIM


def t2s_spec() -> Spec:
    """`t2s_shared_fp16.bin` tensors (`Data/v2/Keys/t2s_onnx_keys.txt` order)."""
    s: Spec = OrderedDict()
    s["ar_audio_embedding.word_embeddings.weight"] = (T2S_VOCAB, T2S_D)
    s["ar_audio_position.alpha"] = (1,)
    for i in range(T2S_LAYERS):
        p = f"transformer_encoder.layers.{i}."
        s[p + "self_attn.in_proj_weight"] = (3 * T2S_D, T2S_D)
        s[p + "self_attn.in_proj_bias"] = (3 * T2S_D,)
        s[p + "self_attn.out_proj.weight"] = (T2S_D, T2S_D)
        s[p + "self_attn.out_proj.bias"] = (T2S_D,)
        s[p + "linear1.weight"] = (T2S_FF, T2S_D)
        s[p + "linear1.bias"] = (T2S_FF,)
        s[p + "linear2.weight"] = (T2S_D, T2S_FF)
        s[p + "linear2.bias"] = (T2S_D,)
        s[p + "norm1.weight"] = (T2S_D,)
        s[p + "norm1.bias"] = (T2S_D,)
        s[p + "norm2.weight"] = (T2S_D,)
        s[p + "norm2.bias"] = (T2S_D,)
    s["ar_predict_layer.weight"] = (T2S_VOCAB, T2S_D)
    return s


def t2s_encoder_spec() -> Spec:
    """`t2s_encoder_fp32.bin` (true fp32; order `EncoderConverter.py:40-48`)."""
    s: Spec = OrderedDict()
    s["encoder.ar_text_embedding.word_embeddings.weight"] = (TEXT_VOCAB, T2S_D)
    s["encoder.bert_proj.weight"] = (T2S_D, BERT_DIM)
    s["encoder.bert_proj.bias"] = (T2S_D,)
    s["encoder.ar_text_position.alpha"] = (1,)
    s["vits.ssl_proj.weight"] = (768, 768, 2)
    s["vits.ssl_proj.bias"] = (768,)
    s["vits.quantizer.vq.layers.0._codebook.embed"] = (1024, 768)
    return s


# -------------------------------------------------------------------- VITS
@dataclass(frozen=True)
class VitsConfig:
    version: str              # "v2" | "v2ProPlus"
    hidden: int = 192
    filter: int = 768
    heads: int = 2
    window: int = 4
    ssl_dim: int = 768
    mrte_dim: int = 512
    mrte_heads: int = 4
    n_ssl_layers: int = 3
    n_text_layers: int = 6
    n_enc2_layers: int = 3
    gin: int = 512            # ge channels into flow cond / dec.cond
    ge_adv: int = 512         # MRTE conditioning (ge, or ge_advanced for v2pp)
    upc: int = 512            # generator initial channels
    up_rates: Tuple[int, ...] = (10, 8, 2, 2, 2)
    up_kernels: Tuple[int, ...] = (16, 16, 8, 2, 2)
    rb_kernels: Tuple[int, ...] = (3, 7, 11)
    rb_dilations: Tuple[int, ...] = (1, 3, 5)
    flow_layers: int = 4      # WN layers per coupling
    flow_kernel: int = 5
    n_flows: int = 4
    spec_bins: int = 704      # ref STFT bins kept (n_fft 2048 -> 1025, sliced)
    ref_hidden: int = 128

    @property
    def has_ref_enc(self) -> bool:
        return self.version == "v2"

    @property
    def hop(self) -> int:
        return int(np.prod(self.up_rates)) * 2   # 640 per token after x2 codebook upsampling


V2 = VitsConfig("v2")
V2PP = VitsConfig("v2ProPlus", gin=1024, upc=768, up_kernels=(20, 16, 8, 2, 2))


def vits_config(version: str) -> VitsConfig:
    if version == "v2":
        return V2
    if version in ("v2ProPlus", "v2pp"):
        return V2PP
    raise ValueError(f"unknown VITS version {version!r}")


def _attn_encoder(s: Spec, pre: str, n: int, c: VitsConfig) -> None:
    h, hd = c.hidden, c.hidden // c.heads
    for i in range(n):
        s[f"{pre}.attn_layers.{i}.emb_rel_k"] = (1, 2 * c.window + 1, hd)
        s[f"{pre}.attn_layers.{i}.emb_rel_v"] = (1, 2 * c.window + 1, hd)
        for cv in ("conv_q", "conv_k", "conv_v", "conv_o"):
            s[f"{pre}.attn_layers.{i}.{cv}.weight"] = (h, h, 1)
            s[f"{pre}.attn_layers.{i}.{cv}.bias"] = (h,)
        s[f"{pre}.norm_layers_1.{i}.gamma"] = (h,)
        s[f"{pre}.norm_layers_1.{i}.beta"] = (h,)
        s[f"{pre}.ffn_layers.{i}.conv_1.weight"] = (c.filter, h, 3)
        s[f"{pre}.ffn_layers.{i}.conv_1.bias"] = (c.filter,)
        s[f"{pre}.ffn_layers.{i}.conv_2.weight"] = (h, c.filter, 3)
        s[f"{pre}.ffn_layers.{i}.conv_2.bias"] = (h,)
        s[f"{pre}.norm_layers_2.{i}.gamma"] = (h,)
        s[f"{pre}.norm_layers_2.{i}.beta"] = (h,)


def _wn(s: Spec, name: str, cout: int, cin: int, k: int, transposed=False) -> None:
    s[name + ".bias"] = (cout,)
    if transposed:   # ConvTranspose weight is [Cin, Cout, K]; weight norm over dim 0
        s[name + ".weight_g"] = (cin, 1, 1)
        s[name + ".weight_v"] = (cin, cout, k)
    else:
        s[name + ".weight_g"] = (cout, 1, 1)
        s[name + ".weight_v"] = (cout, cin, k)


def ref_enc_spec(s: Spec, pre: str, out_dim: int, c: VitsConfig) -> None:
    r = c.ref_hidden
    s[pre + "spectral.0.fc.weight"] = (r, c.spec_bins)
    s[pre + "spectral.0.fc.bias"] = (r,)
    s[pre + "spectral.3.fc.weight"] = (r, r)
    s[pre + "spectral.3.fc.bias"] = (r,)
    for i in range(2):
        s[pre + f"temporal.{i}.conv1.conv.weight"] = (2 * r, r, 5)
        s[pre + f"temporal.{i}.conv1.conv.bias"] = (2 * r,)
    for nm in ("w_qs", "w_ks", "w_vs", "fc"):
        s[pre + f"slf_attn.{nm}.weight"] = (r, r)
        s[pre + f"slf_attn.{nm}.bias"] = (r,)
    s[pre + "fc.fc.weight"] = (out_dim, r)
    s[pre + "fc.fc.bias"] = (out_dim,)


def vits_spec(version: str) -> Spec:
    c = vits_config(version)
    s: Spec = OrderedDict()
    p = "vq_model.enc_p."
    s[p + "ssl_proj.weight"] = (c.hidden, c.ssl_dim, 1)
    s[p + "ssl_proj.bias"] = (c.hidden,)
    _attn_encoder(s, p + "encoder_ssl", c.n_ssl_layers, c)
    _attn_encoder(s, p + "encoder_text", c.n_text_layers, c)
    s[p + "text_embedding.weight"] = (TEXT_VOCAB, c.hidden)
    m = p + "mrte."
    for cv in ("conv_q", "conv_k", "conv_v", "conv_o"):
        s[m + f"cross_attention.{cv}.weight"] = (c.mrte_dim, c.mrte_dim, 1)
        s[m + f"cross_attention.{cv}.bias"] = (c.mrte_dim,)
    s[m + "c_pre.weight"] = (c.mrte_dim, c.hidden, 1)
    s[m + "c_pre.bias"] = (c.mrte_dim,)
    s[m + "text_pre.weight"] = (c.mrte_dim, c.hidden, 1)
    s[m + "text_pre.bias"] = (c.mrte_dim,)
    s[m + "c_post.weight"] = (c.hidden, c.mrte_dim, 1)
    s[m + "c_post.bias"] = (c.hidden,)
    _attn_encoder(s, p + "encoder2", c.n_enc2_layers, c)
    s[p + "proj.weight"] = (2 * c.hidden, c.hidden, 1)
    s[p + "proj.bias"] = (2 * c.hidden,)
    d = "vq_model.dec."
    s[d + "conv_pre.weight"] = (c.upc, c.hidden, 7)
    s[d + "conv_pre.bias"] = (c.upc,)
    ch = c.upc
    for i, (u, k) in enumerate(zip(c.up_rates, c.up_kernels)):
        _wn(s, d + f"ups.{i}", ch // 2, ch, k, transposed=True)
        ch //= 2
    ch = c.upc
    for i in range(len(c.up_rates)):
        ch //= 2
        for j, k in enumerate(c.rb_kernels):
            rb = d + f"resblocks.{i * len(c.rb_kernels) + j}."
            for m_ in range(len(c.rb_dilations)):
                _wn(s, rb + f"convs1.{m_}", ch, ch, k)
            for m_ in range(len(c.rb_dilations)):
                _wn(s, rb + f"convs2.{m_}", ch, ch, k)
    s[d + "conv_post.weight"] = (1, ch, 7)
    s[d + "cond.weight"] = (c.upc, c.gin, 1)
    s[d + "cond.bias"] = (c.upc,)
    half = c.hidden // 2
    for f in range(0, 2 * c.n_flows, 2):
        fp = f"vq_model.flow.flows.{f}."
        s[fp + "pre.weight"] = (c.hidden, half, 1)
        s[fp + "pre.bias"] = (c.hidden,)
        for l in range(c.flow_layers):
            _wn(s, fp + f"enc.in_layers.{l}", 2 * c.hidden, c.hidden, c.flow_kernel)
        for l in range(c.flow_layers):
            out = 2 * c.hidden if l < c.flow_layers - 1 else c.hidden
            _wn(s, fp + f"enc.res_skip_layers.{l}", out, c.hidden, 1)
        _wn(s, fp + "enc.cond_layer", 2 * c.hidden * c.flow_layers, c.gin, 1)
        s[fp + "post.weight"] = (half, c.hidden, 1)
        s[fp + "post.bias"] = (half,)
    if c.has_ref_enc:
        ref_enc_spec(s, "vq_model.ref_enc.", c.gin, c)
    s["vq_model.quantizer.vq.layers.0._codebook.embed"] = (1024, c.ssl_dim)
    return s


def prompt_encoder_spec() -> Spec:
    c = V2PP
    s: Spec = OrderedDict()
    ref_enc_spec(s, "ref_enc.", 1024, c)
    s["sv_emb.weight"] = (1024, 20480)
    s["sv_emb.bias"] = (1024,)
    s["ge_to512.weight"] = (512, 1024)
    s["ge_to512.bias"] = (512,)
    s["prelu.weight"] = (1024,)
    return s


def hubert_spec() -> Spec:
    """CN-HuBERT (chinese-hubert-base, GenieData/chinese-hubert-base; loaded at
    `g/ModelManager.py:172-195`).  Names and shapes of transformers' HubertModel
    (conv_bias=False, feat_extract_norm="group"), the model GPT-SoVITS exports;
    the positional conv is stored weight-normed (g v / ||v||), as an exported
    graph folds it.  The graph file itself is absent here: this layout is not
    pinned to the real chinese-hubert-base.onnx initializer table."""
    s: Spec = OrderedDict()
    s["feature_extractor.conv_layers.0.conv.weight"] = (512, 1, 10)
    s["feature_extractor.conv_layers.0.layer_norm.weight"] = (512,)
    s["feature_extractor.conv_layers.0.layer_norm.bias"] = (512,)
    for i, k in enumerate((3, 3, 3, 3, 2, 2), start=1):
        s[f"feature_extractor.conv_layers.{i}.conv.weight"] = (512, 512, k)
    s["feature_projection.layer_norm.weight"] = (512,)
    s["feature_projection.layer_norm.bias"] = (512,)
    s["feature_projection.projection.weight"] = (768, 512)
    s["feature_projection.projection.bias"] = (768,)
    s["encoder.pos_conv_embed.conv.weight"] = (768, 48, 128)
    s["encoder.pos_conv_embed.conv.bias"] = (768,)
    s["encoder.layer_norm.weight"] = (768,)
    s["encoder.layer_norm.bias"] = (768,)
    for l in range(12):
        p = f"encoder.layers.{l}."
        for m in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s[p + f"attention.{m}.weight"] = (768, 768)
            s[p + f"attention.{m}.bias"] = (768,)
        s[p + "layer_norm.weight"] = (768,)
        s[p + "layer_norm.bias"] = (768,)
        s[p + "feed_forward.intermediate_dense.weight"] = (3072, 768)
        s[p + "feed_forward.intermediate_dense.bias"] = (3072,)
        s[p + "feed_forward.output_dense.weight"] = (768, 3072)
        s[p + "feed_forward.output_dense.bias"] = (768,)
        s[p + "final_layer_norm.weight"] = (768,)
        s[p + "final_layer_norm.bias"] = (768,)
    return s


def load_hubert_weights(model_dir: str) -> Dict[str, np.ndarray]:
    """GenieData/chinese-hubert-base: chinese-hubert-base.onnx + *_weights_fp16.bin
    (`g/ModelManager.py:41-42,177-182`), read through the initializer table like
    a character's bins.  Unverified against a real file (none offline)."""
    return load_fp16_bin(os.path.join(model_dir, "chinese-hubert-base.onnx"),
                         os.path.join(model_dir, "chinese-hubert-base_weights_fp16.bin"), hubert_spec())


def roberta_spec(n_layers: int = 24, vocab: int = 21128, max_pos: int = 512) -> Spec:
    """RoBERTa for Chinese BERT features (chinese-roberta-wwm-ext-large, GenieData
    RoBERTa.onnx, `g/ModelManager.py:44,132-150`): transformers BertModel names
    (hidden 1024, 16 heads, FFN 4096); the graph reads hidden_states[-3], so the
    last two layers are never run.  Not pinned to the real RoBERTa.onnx table."""
    s: Spec = OrderedDict()
    s["embeddings.word_embeddings.weight"] = (vocab, 1024)
    s["embeddings.position_embeddings.weight"] = (max_pos, 1024)
    s["embeddings.token_type_embeddings.weight"] = (2, 1024)
    s["embeddings.LayerNorm.weight"] = (1024,)
    s["embeddings.LayerNorm.bias"] = (1024,)
    for l in range(n_layers):
        p = f"encoder.layer.{l}."
        for m in ("query", "key", "value"):
            s[p + f"attention.self.{m}.weight"] = (1024, 1024)
            s[p + f"attention.self.{m}.bias"] = (1024,)
        s[p + "attention.output.dense.weight"] = (1024, 1024)
        s[p + "attention.output.dense.bias"] = (1024,)
        s[p + "attention.output.LayerNorm.weight"] = (1024,)
        s[p + "attention.output.LayerNorm.bias"] = (1024,)
        s[p + "intermediate.dense.weight"] = (4096, 1024)
        s[p + "intermediate.dense.bias"] = (4096,)
        s[p + "output.dense.weight"] = (1024, 4096)
        s[p + "output.dense.bias"] = (1024,)
        s[p + "output.LayerNorm.weight"] = (1024,)
        s[p + "output.LayerNorm.bias"] = (1024,)
    return s


def load_roberta_weights(model_dir: str) -> Dict[str, np.ndarray]:
    """GenieData RoBERTa/RoBERTa.onnx weights (`g/ModelManager.py:44,139`) through the
    initializer table; the reference loads that graph without an fp16 bin, so its
    initializers are read in place (fp32).  Unverified against a real file."""
    from .onnx_table import read_initializer_values
    return read_initializer_values(os.path.join(model_dir, "RoBERTa.onnx"), roberta_spec())


SV_STAGES = ((64, 3, 1, False), (128, 4, 2, False), (256, 6, 2, True), (512, 3, 2, True))


def sv_spec() -> Spec:
    """Speaker-verification model (GenieData speaker_encoder.onnx, V2ProPlus `sv_emb`;
    loaded at `g/ModelManager.py:155-170`, run at `g/Audio/ReferenceAudio.py:71-72`):
    GPT-SoVITS's ERes2NetV2(baseWidth=24, scale=4, expansion=4) state_dict names,
    BatchNorm unfolded (weight, bias, running_mean, running_var; eps 1e-5).  Stages
    (planes, blocks, stride, AFF) = SV_STAGES; width = floor(planes * 24 / 64).  The
    real graph is absent: this layout is not pinned to its initializer table."""
    s: Spec = OrderedDict()

    def bn(p, c):
        for leaf in ("weight", "bias", "running_mean", "running_var"):
            s[f"{p}.{leaf}"] = (c,)

    def aff(p, c):
        inter = c // 4
        s[p + ".local_att.0.weight"] = (inter, 2 * c, 1, 1)
        s[p + ".local_att.0.bias"] = (inter,)
        bn(p + ".local_att.1", inter)
        s[p + ".local_att.3.weight"] = (c, inter, 1, 1)
        s[p + ".local_att.3.bias"] = (c,)
        bn(p + ".local_att.4", c)

    s["conv1.weight"] = (64, 1, 3, 3)
    bn("bn1", 64)
    cin = 64
    for li, (planes, nb, stride, use_aff) in enumerate(SV_STAGES, start=1):
        width = planes * 24 // 64
        for b in range(nb):
            p = f"layer{li}.{b}"
            st = stride if b == 0 else 1
            s[p + ".conv1.weight"] = (width * 4, cin, 1, 1)
            bn(p + ".bn1", width * 4)
            for i in range(4):
                s[p + f".convs.{i}.weight"] = (width, width, 3, 3)
                bn(p + f".bns.{i}", width)
            if use_aff:
                for i in range(3):
                    aff(p + f".fuse_models.{i}", width)
            s[p + ".conv3.weight"] = (planes * 4, width * 4, 1, 1)
            bn(p + ".bn3", planes * 4)
            if st != 1 or cin != planes * 4:
                s[p + ".shortcut.0.weight"] = (planes * 4, cin, 1, 1)
                bn(p + ".shortcut.1", planes * 4)
            cin = planes * 4
    s["layer3_ds.weight"] = (2048, 1024, 3, 3)
    aff("fuse34", 2048)
    return s


def sv_conv_order() -> List[Tuple[str, Optional[str]]]:
    """The SV model's convs in forward3's execution order (the order torch.onnx.export
    writes their Conv nodes): (conv prefix, BatchNorm prefix applied to its output or
    None).  Stem; per block conv1, convs.0, [fuse_models.i-1 local_att.0 / .3,] convs.i,
    conv3, shortcut.0; then layer3_ds (computed after layer4) and fuse34."""
    order: List[Tuple[str, Optional[str]]] = [("conv1", "bn1")]
    cin = 64
    for li, (planes, nb, stride, use_aff) in enumerate(SV_STAGES, start=1):
        for b in range(nb):
            p = f"layer{li}.{b}"
            order.append((p + ".conv1", p + ".bn1"))
            for i in range(4):
                if i > 0 and use_aff:
                    order.append((p + f".fuse_models.{i - 1}.local_att.0", p + f".fuse_models.{i - 1}.local_att.1"))
                    order.append((p + f".fuse_models.{i - 1}.local_att.3", p + f".fuse_models.{i - 1}.local_att.4"))
                order.append((p + f".convs.{i}", p + f".bns.{i}"))
            order.append((p + ".conv3", p + ".bn3"))
            st = stride if b == 0 else 1
            if st != 1 or cin != planes * 4:
                order.append((p + ".shortcut.0", p + ".shortcut.1"))
            cin = planes * 4
    order.append(("layer3_ds", None))
    order.append(("fuse34.local_att.0", "fuse34.local_att.1"))
    order.append(("fuse34.local_att.3", "fuse34.local_att.4"))
    return order


def load_sv_weights(path: str) -> Dict[str, np.ndarray]:
    """GenieData speaker_encoder.onnx (`g/ModelManager.py:155-170`, plain ONNX with
    fp32 initializers, no fp16 bin).  Two layouts are read:

      * initializers under sv_spec's state-dict names (BatchNorm unfolded);
      * an export that renamed them (onnx::Conv_N ...), with or without BatchNorm
        folded into the convs: its Conv nodes, in the file's (topological) order, are
        mapped onto sv_conv_order() with every weight shape checked; a conv's own bias
        input becomes '<conv>.bias', and a BatchNormalization node reading a conv's
        output gives that conv's BatchNorm tensors (folded exports have none: the
        engine then takes the conv bias alone).

    Neither fits -> KeyError naming the missing tensors.  Unverified against the real
    file (none offline): SV parity at the ONNX level is unpinned."""
    from .onnx_table import read_graph, read_initializer_values
    if os.path.isdir(path):
        path = os.path.join(path, "speaker_encoder.onnx")
    spec = sv_spec()
    try:
        return read_initializer_values(path, spec)
    except KeyError:
        pass
    inits, nodes = read_graph(path)
    missing = [n for n in spec if n not in inits]
    convs = [nd for nd in nodes if nd[0] == "Conv"]
    order = sv_conv_order()
    if len(convs) != len(order):
        raise KeyError(f"{path}: {len(missing)} SV initializers missing by name (e.g. {missing[:4]}) and "
                       f"{len(convs)} Conv nodes where the renamed layout has {len(order)}")
    bn_of = {nd[1][0]: nd for nd in nodes if nd[0] == "BatchNormalization"}
    out: Dict[str, np.ndarray] = {}
    for k, ((conv, bn), nd) in enumerate(zip(order, convs)):
        w = inits.get(nd[1][1]) if len(nd[1]) > 1 else None
        want = spec[conv + ".weight"]
        if w is None or tuple(w.shape) != tuple(want):
            raise KeyError(f"{path}: Conv node {k} ({nd[3] or nd[1][1]}) has weight shape "
                           f"{None if w is None else tuple(w.shape)}, expected {conv}.weight {want}")
        out[conv + ".weight"] = np.asarray(w, np.float32)
        b = inits.get(nd[1][2]) if len(nd[1]) > 2 and nd[1][2] else None
        if b is not None:
            out[conv + ".bias"] = np.asarray(b, np.float32).reshape(-1)
        bnode = bn_of.get(nd[2][0]) if nd[2] else None
        if bn is not None and bnode is not None:
            for leaf, name in zip(("weight", "bias", "running_mean", "running_var"), bnode[1][1:5]):
                out[f"{bn}.{leaf}"] = np.asarray(inits[name], np.float32).reshape(-1)
        elif bn is not None and b is None:
            raise KeyError(f"{path}: {conv} has neither a bias (folded BatchNorm) nor a BatchNormalization node")
    return out


def spec_numel(spec: Spec) -> int:
    return int(sum(int(np.prod(v)) for v in spec.values()))


# ------------------------------------------------------- Genie file format
@dataclass
class CharacterFiles:
    """The files `check_onnx_model_dir` requires (`g/Internal.py:41-91`)."""
    model_dir: str

    def path(self, name: str) -> str:
        return os.path.join(self.model_dir, name)

    REQUIRED = (
        "t2s_encoder_fp32.bin", "t2s_encoder_fp32.onnx",
        "t2s_first_stage_decoder_fp32.onnx", "t2s_shared_fp16.bin",
        "t2s_stage_decoder_fp32.onnx", "vits_fp16.bin", "vits_fp32.onnx",
    )

    def check(self) -> None:
        if not os.path.isdir(self.model_dir):
            raise FileNotFoundError(
                f"The model directory '{self.model_dir}' does not exist or is not a directory.")
        missing = [f for f in self.REQUIRED if not os.path.exists(self.path(f))]
        if missing:
            raise FileNotFoundError(
                f"[Genie Error] Invalid ONNX model directory: '{self.model_dir}'; "
                f"missing base files: {', '.join(sorted(missing))}")

    @property
    def is_v2pp(self) -> bool:
        return os.path.exists(self.path("prompt_encoder_fp32.onnx")) and \
            os.path.exists(self.path("prompt_encoder_fp16.bin"))


def load_fp16_bin(onnx_path: str, bin_path: str, spec: Spec) -> Dict[str, np.ndarray]:
    """Read a Genie fp16 weight bin through the ONNX initializer table.

    Mirrors `load_session_with_fp16_conversion` (`g/ModelManager.py:59-114`):
    the relinked graph's EXTERNAL (offset, length) pairs address the fp32
    upcast of the bin, so the fp16 slice is elements [offset/4, (offset+length)/4).
    Values are returned as fp16 (lossless; the reference's upcast adds nothing).
    The fp16 element index of a tensor is offset/4 (fp32 byte offset / 4 B).
    """
    from .onnx_table import read_initializer_table
    table = read_initializer_table(onnx_path)
    raw = np.fromfile(bin_path, dtype=np.float16)
    out: Dict[str, np.ndarray] = {}
    for name, shape in spec.items():
        if name not in table:
            raise KeyError(f"{onnx_path}: initializer {name} not found")
        dims, offset, length = table[name]
        if tuple(dims) != tuple(shape):
            raise ValueError(f"{name}: shape {dims} in graph, expected {shape}")
        if offset is None:
            raise ValueError(f"{name}: not an external initializer")
        lo, n = offset // 4, length // 4
        if lo + n > raw.size:
            raise ValueError(f"{name}: range exceeds {bin_path}")
        out[name] = raw[lo: lo + n].reshape(shape)
    return out


def load_fp32_bin(onnx_path: str, bin_path: str, spec: Spec) -> Dict[str, np.ndarray]:
    """`t2s_encoder_fp32.bin` is plain fp32 external data of `t2s_encoder_fp32.onnx`."""
    from .onnx_table import read_initializer_table
    table = read_initializer_table(onnx_path)
    raw = np.fromfile(bin_path, dtype=np.float32)
    out: Dict[str, np.ndarray] = {}
    for name, shape in spec.items():
        dims, offset, length = table[name]
        if tuple(dims) != tuple(shape):
            raise ValueError(f"{name}: shape {dims} in graph, expected {shape}")
        lo, n = offset // 4, length // 4
        out[name] = raw[lo: lo + n].reshape(shape)
    return out


def load_character_weights(model_dir: str) -> Tuple[str, Dict[str, Dict[str, np.ndarray]]]:
    """Load every weight of a converted character directory.

    Returns (version, {"t2s_encoder", "t2s", "vits", ["prompt_encoder"]}).
    """
    files = CharacterFiles(model_dir)
    files.check()
    version = "v2ProPlus" if files.is_v2pp else "v2"
    w: Dict[str, Dict[str, np.ndarray]] = {}
    w["t2s_encoder"] = load_fp32_bin(files.path("t2s_encoder_fp32.onnx"),
                                     files.path("t2s_encoder_fp32.bin"), t2s_encoder_spec())
    w["t2s"] = load_fp16_bin(files.path("t2s_first_stage_decoder_fp32.onnx"),
                             files.path("t2s_shared_fp16.bin"), t2s_spec())
    w["vits"] = load_fp16_bin(files.path("vits_fp32.onnx"), files.path("vits_fp16.bin"),
                              vits_spec(version))
    if files.is_v2pp:
        w["prompt_encoder"] = load_fp16_bin(files.path("prompt_encoder_fp32.onnx"),
                                            files.path("prompt_encoder_fp16.bin"),
                                            prompt_encoder_spec())
    return version, w


def layout_offsets(spec: Spec, bytes_per_elem: int = 4) -> List[Tuple[str, int, int]]:
    """(name, offset, length) of a header-less concat of `spec` in order."""
    off = 0
    res = []
    for name, shape in spec.items():
        ln = int(np.prod(shape)) * bytes_per_elem
        res.append((name, off, ln))
        off += ln
    return res
