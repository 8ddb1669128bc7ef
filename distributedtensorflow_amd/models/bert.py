"""BERT (google-research/bert ``modeling.py`` architecture) for masked-LM pre-training.

North-star BASELINE.json config 5 ("BERT-base MLM MultiWorkerMirroredStrategy, MFMA GEMM path +
fused LAMB"); the reference itself has no sequence models, so semantics and
variable names follow google-research/bert so TF checkpoints line up:
``bert/embeddings/word_embeddings``, ``bert/encoder/layer_0/attention/self/query/kernel``,
``cls/predictions/transform/dense/kernel``, ``cls/predictions/output_bias`` ...

MI355X layout choices:
  * activations are token-major bf16 ``[B*S, 768]`` matrices end to end (no [B,H,S,D]
    transposes): Q/K/V come from ONE fused ``768 -> 2304`` GEMM whose output the MFMA attention
    kernel reads in place; its fp32 master ``[2304, 768]`` is exported to checkpoints as the
    three TF variables ``query|key|value`` (row slices, ``_dtf_splits``);
  * every GEMM runs on our persistent MFMA GEMM (csrc/kernels/gemm.hip gemm_pp2) and every
    weight gradient on our TN weight-gradient kernel, and everything around them is fused into
    our kernels: bias+GELU, bias+dropout+residual+LayerNorm, embedding gather+sum+LN+dropout,
    flash attention with in-kernel dropout, weighted MLM cross-entropy;
  * the MLM decoder is tied to the word embeddings (one fp32 master whose bf16 shadow feeds both
    the gather and the logits GEMM).  Its vocabulary is padded to a multiple of 64 (30522 ->
    30528 rows) so the decoder's forward, data gradient and weight gradient fit our GEMM tiles:
    the padding rows of the table and of the output bias are zero, never gathered, get an exact
    zero gradient (the loss leaves their logits out of the softmax), so training is exactly the
    unpadded model; checkpoints and SavedModels carry the TF shapes ``[30522, 768]`` /
    ``[30522]`` (row slices, ``_dtf_splits``).
"""
from __future__ import annotations

import dataclasses
import os

import torch
import torch.nn as nn

from .. import ops
from .layers import Layer, _tag, truncated_normal_


# BERT's dense layers take ops.dense(impl="library"): the bias rides in the GEMM epilogue or in
# the fused consumer kernel, and the GEMMs run on our persistent MFMA GEMM (ops/native.py _Dense;
# hipBLASLt only for shapes outside its tiles, none in BERT-base).  "native" selects the
# tf.layers.dense form (bias + ReLU epilogue, separate bias-gradient pass) instead.
BERT_GEMM = os.environ.get("DTF_BERT_GEMM", "library")
# the tied decoder's vocabulary rows are padded to a multiple of this (GEMM tile / 16-B rows)
VOCAB_ALIGN = 64


def padded_vocab(v: int) -> int:
    return -(-v // VOCAB_ALIGN) * VOCAB_ALIGN
# FFN: bias + GELU + second GEMM as one op whose data gradient carries the GELU derivative in our
# GEMM's epilogue (A/B knob)
FUSE_GELU_DGRAD = os.environ.get("DTF_BERT_FUSE_GELU_DGRAD", "1") == "1"


@dataclasses.dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12

    @staticmethod
    def base(**kw):
        return BertConfig(**kw)

    @staticmethod
    def large(**kw):
        d = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                 intermediate_size=4096)
        d.update(kw)
        return BertConfig(**d)


def _param(shape, name, std=None, layout=None, fill=None):
    p = nn.Parameter(torch.empty(*shape))
    if fill is not None:
        p.data.fill_(fill)
    else:
        truncated_normal_(p.data, std)
    return _tag(p, name, layout)


class _Dense(nn.Module):
    """y = x @ W^T (hipBLASLt) with the bias applied by the fused consumer kernel."""

    def __init__(self, n_in, n_out, name, std):
        super().__init__()
        self.kernel = _param((n_out, n_in), f"{name}/kernel", std, "OI")
        self.bias = _param((n_out,), f"{name}/bias", fill=0.0)

    def gemm(self, x):
        return ops.dense(x, self.kernel, None, impl=BERT_GEMM)


class _LayerNorm(nn.Module):
    def __init__(self, n, name):
        super().__init__()
        self.gamma = _param((n,), f"{name}/gamma", fill=1.0)
        self.beta = _param((n,), f"{name}/beta", fill=0.0)


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig, idx: int):
        super().__init__()
        H, std = cfg.hidden_size, cfg.initializer_range
        pre = f"bert/encoder/layer_{idx}"
        self.cfg = cfg
        # fused Q|K|V projection; checkpoint names split back into query / key / value
        self.qkv_kernel = _param((3 * H, H), f"{pre}/attention/self/qkv/kernel", std, "OI")
        self.qkv_kernel._dtf_splits = [
            (f"{pre}/attention/self/{n}/kernel", i * H, (i + 1) * H) for i, n in
            enumerate(("query", "key", "value"))]
        self.qkv_bias = _param((3 * H,), f"{pre}/attention/self/qkv/bias", fill=0.0)
        self.qkv_bias._dtf_splits = [
            (f"{pre}/attention/self/{n}/bias", i * H, (i + 1) * H) for i, n in
            enumerate(("query", "key", "value"))]
        self.attn_out = _Dense(H, H, f"{pre}/attention/output/dense", std)
        self.attn_ln = _LayerNorm(H, f"{pre}/attention/output/LayerNorm")
        self.inter = _Dense(H, cfg.intermediate_size, f"{pre}/intermediate/dense", std)
        self.out = _Dense(cfg.intermediate_size, H, f"{pre}/output/dense", std)
        self.out_ln = _LayerNorm(H, f"{pre}/output/LayerNorm")

    def forward(self, x, mask, B, S):
        cfg = self.cfg
        qkv = ops.dense(x, self.qkv_kernel, self.qkv_bias, impl=BERT_GEMM)
        ctx = ops.attention_qkv(qkv, mask, B, S, cfg.num_attention_heads,
                                cfg.attention_probs_dropout_prob, self.training)
        a = self.attn_out.gemm(ctx)
        # x feeds the QKV dense above and the residual here: its two gradients are summed by
        # that dense's dgrad GEMM (beta = 1), not by a separate add
        x = ops.bias_dropout_add_layer_norm(a, self.attn_out.bias, x, self.attn_ln.gamma,
                                            self.attn_ln.beta, cfg.hidden_dropout_prob,
                                            self.training, cfg.layer_norm_eps,
                                            residual_to_dense=True)
        if FUSE_GELU_DGRAD and BERT_GEMM == "library":
            # the whole FFN as one op: the first GEMM applies bias + GELU in its epilogue (our
            # MFMA GEMM); the backward forms d(pre-activation) in one GEMM pass with the GELU
            # derivative in the epilogue (ops.native.dense_gelu_dense / _BiasGeluDense)
            o = ops.dense_gelu_dense(x, self.inter.kernel, self.inter.bias, self.out.kernel)
        else:
            h = ops.bias_gelu(self.inter.gemm(x), self.inter.bias)
            o = self.out.gemm(h)
        return ops.bias_dropout_add_layer_norm(o, self.out.bias, x, self.out_ln.gamma,
                                               self.out_ln.beta, cfg.hidden_dropout_prob,
                                               self.training, cfg.layer_norm_eps,
                                               residual_to_dense=True)


class BertForPreTraining(Layer):
    """BERT encoder + masked-LM head (the NSP head of the original is omitted: config 5 is MLM)."""

    def __init__(self, cfg: BertConfig | None = None):
        super().__init__()
        cfg = cfg or BertConfig()
        self.cfg = cfg
        H, std = cfg.hidden_size, cfg.initializer_range
        if H % cfg.num_attention_heads or H // cfg.num_attention_heads != 64:
            raise ValueError("attention kernels are built for head_dim 64")
        V, Vp = cfg.vocab_size, padded_vocab(cfg.vocab_size)
        self.word_embeddings = _param((Vp, H), "bert/embeddings/word_embeddings", std)
        self.token_type_embeddings = _param((cfg.type_vocab_size, H),
                                            "bert/embeddings/token_type_embeddings", std)
        self.position_embeddings = _param((cfg.max_position_embeddings, H),
                                          "bert/embeddings/position_embeddings", std)
        self.emb_ln = _LayerNorm(H, "bert/embeddings/LayerNorm")
        self.layers = nn.ModuleList(BertLayer(cfg, i) for i in range(cfg.num_hidden_layers))
        self.mlm_transform = _Dense(H, H, "cls/predictions/transform/dense", std)
        self.mlm_ln = _LayerNorm(H, "cls/predictions/transform/LayerNorm")
        self.mlm_bias = _param((Vp,), "cls/predictions/output_bias", fill=0.0)
        if Vp != V:
            with torch.no_grad():
                self.word_embeddings[V:].zero_()
            # checkpoints / SavedModels carry the TF shapes (the first V rows)
            self.word_embeddings._dtf_splits = [("bert/embeddings/word_embeddings", 0, V)]
            self.mlm_bias._dtf_splits = [("cls/predictions/output_bias", 0, V)]

    def num_params_tf(self) -> int:
        """Parameters of the TF model (the padding rows of the tied vocabulary excluded)."""
        return sum(t.numel() for _, t, _ in self.variables_tf())

    def variables_tf(self):
        for p in self.parameters():
            if hasattr(p, "_dtf_name"):
                splits = getattr(p, "_dtf_splits", None)
                if splits:
                    for name, s, e in splits:
                        yield name, p[s:e], p._dtf_layout
                else:
                    yield p._dtf_name, p, p._dtf_layout

    def encode(self, input_ids, token_type_ids=None, attention_mask=None):
        """-> ([B*S, H] final hidden states, additive key mask)."""
        cfg = self.cfg
        B, S = input_ids.shape
        dtype = torch.bfloat16 if input_ids.is_cuda else torch.float32
        x = ops.embedding_layer_norm(input_ids, token_type_ids, self.word_embeddings,
                                     self.position_embeddings, self.token_type_embeddings,
                                     self.emb_ln.gamma, self.emb_ln.beta, cfg.hidden_dropout_prob,
                                     self.training, cfg.layer_norm_eps, dtype=dtype)
        mask = None
        if attention_mask is not None:
            mask = (1.0 - attention_mask.float()) * -10000.0
        for layer in self.layers:
            x = layer(x, mask, B, S)
        return x, mask

    def forward(self, input_ids, token_type_ids=None, attention_mask=None,
                masked_lm_positions=None, masked_lm_ids=None, masked_lm_weights=None):
        """Returns the MLM loss (sum(w * nll) / sum(w)) when labels are given, else logits of the
        masked positions ``[B*P, vocab]``."""
        cfg = self.cfg
        B, S = input_ids.shape
        x, _ = self.encode(input_ids, token_type_ids, attention_mask)
        if masked_lm_positions is None:
            masked_lm_positions = torch.arange(S, device=x.device).expand(B, S)
        flat = (masked_lm_positions + torch.arange(B, device=x.device).unsqueeze(1) * S).reshape(-1)
        h = x.index_select(0, flat)                                      # [B*P, H] gather
        h = ops.bias_gelu(self.mlm_transform.gemm(h), self.mlm_transform.bias)
        h = ops.bias_dropout_add_layer_norm(h, None, None, self.mlm_ln.gamma, self.mlm_ln.beta,
                                            0.0, self.training, cfg.layer_norm_eps)
        # tied decoder over the padded vocabulary [B*P, Vp]; the padding logits are exactly 0
        logits = ops.dense(h, self.word_embeddings, self.mlm_bias, impl=BERT_GEMM)
        V = cfg.vocab_size
        if masked_lm_ids is None:
            return logits if logits.shape[-1] == V else logits[:, :V]
        return ops.mlm_loss(logits, masked_lm_ids, masked_lm_weights, vocab=V)


def bert_base(**kw) -> BertForPreTraining:
    return BertForPreTraining(BertConfig.base(**kw))


def bert_large(**kw) -> BertForPreTraining:
    return BertForPreTraining(BertConfig.large(**kw))


def mlm_flops_per_token(cfg: BertConfig, seq_len: int, max_predictions: int) -> float:
    """Training FLOPs per input token (fwd + bwd = 3x fwd) for MFU accounting."""
    H, L, I = cfg.hidden_size, cfg.num_hidden_layers, cfg.intermediate_size
    gemm = 2 * (3 * H * H + H * H + 2 * H * I) * L
    attn = 2 * 2 * seq_len * H * L
    head = 2 * (H * H + H * cfg.vocab_size) * max_predictions / seq_len
    return 3.0 * (gemm + attn + head)


__all__ = ["BertConfig", "BertForPreTraining", "BertLayer", "bert_base", "bert_large",
           "mlm_flops_per_token"]
