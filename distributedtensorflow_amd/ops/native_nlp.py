"""Autograd wrappers for the transformer kernels in ``csrc/kernels/nlp.hip`` (BERT, config 5).

All activations are bf16 ``[T, H]`` token-major matrices (T = batch * seq); parameters are fp32
masters (LayerNorm gamma/beta and biases are read in fp32, embedding tables through their bf16
shadow).  Dropout masks are never stored: every op draws a 32-bit seed per call and the kernels
regenerate the same mask in the backward from a counter-based hash (see ``reference.keep_mask``
for the bit-exact PyTorch twin used by the numerics tests).

Reference parity: the reference has no transformer; semantics follow
google-research/bert ``modeling.py`` (tanh GELU, LayerNorm eps 1e-12, additive -10000 mask,
dropout after the embedding LayerNorm, ``LN(dropout(dense(x)) + x)`` sub-layer outputs).
"""
from __future__ import annotations

import os

import torch

from .native import _K, _BF16, _bf16_weight, _direct_grad, _grad_ready, _p, _st

AD = 64   # attention head dim supported by the MFMA kernels
# fused LayerNorm -> dense dgrad hand-off of the residual gradient (bias_dropout_add_layer_norm)
_RESIDUAL_TO_DENSE = os.environ.get("DTF_RESIDUAL_TO_DENSE", "1") == "1"
if os.environ.get("DTF_ATTN_WIDE"):
    _K.attn_set_wide(int(os.environ["DTF_ATTN_WIDE"]))
if os.environ.get("DTF_ATTN_KEEP"):        # 0: the fused attention backward re-hashes dropout
    _K.attn_set_keep(int(os.environ["DTF_ATTN_KEEP"]))
if os.environ.get("DTF_LN_WIDE"):          # 0: the 8-B-per-lane LayerNorm kernels
    _K.ln_set_wide(int(os.environ["DTF_LN_WIDE"]))
if os.environ.get("DTF_ATTN_FUSED_BWD"):      # 0: the split dQ + dK/dV backward at S == 128
    _K.attn_set_fused(int(os.environ["DTF_ATTN_FUSED_BWD"]))


SEED_DRAWS = [0]   # host-side seed draws so far (train/graphed.py refuses to freeze them)


def next_seed() -> int:
    """Dropout seed from torch's CPU generator (so torch.manual_seed makes runs reproducible)."""
    SEED_DRAWS[0] += 1
    return int(torch.randint(0, 2 ** 31 - 1, (1,), device="cpu").item())


def _f32(t):
    return None if t is None else t.detach().float().contiguous()


# ----------------------------------------------------------------------------- LayerNorm
class _FusedLayerNorm(torch.autograd.Function):
    """y = LN(dropout(a + bias) + res) * gamma + beta   (bias / res / dropout optional)."""

    @staticmethod
    def forward(ctx, a, bias, res, gamma, beta, p, eps, res_to_dense=False):
        H = a.shape[-1]
        a2 = a.reshape(-1, H).contiguous()
        M = a2.shape[0]
        r2 = None if res is None else res.reshape(-1, H).contiguous()
        y = torch.empty_like(a2)
        fused = bias is not None or r2 is not None or p > 0
        s = torch.empty_like(a2) if fused else None
        mean = torch.empty(M, device=a.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        seed = next_seed() if p > 0 else 0
        g32, b32, bias32 = _f32(gamma), _f32(beta), _f32(bias)
        _K.ln_fwd(a2.data_ptr(), _p(bias32), _p(r2), g32.data_ptr(), b32.data_ptr(),
                  y.data_ptr(), _p(s), mean.data_ptr(), rstd.data_ptr(), M, H, float(eps),
                  float(p), seed, 0.0, 0, 0, 0, 0, 0, 0, 1, _st())
        ctx.save_for_backward(s if fused else a2, mean, rstd, g32)
        ctx.cfg = (M, H, float(p), seed, bias is not None, res is not None, a.shape)
        ctx.params = (gamma, beta, bias)
        # d(res) handed to the dense layer that also reads res (see _Dense.backward)
        ctx.res_ref = res if res_to_dense else None
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, g32 = ctx.saved_tensors
        M, H, p, seed, has_bias, has_res, shape = ctx.cfg
        dy2 = dy.reshape(-1, H).to(_BF16).contiguous()
        ds = torch.empty_like(dy2)
        da = torch.empty_like(dy2) if p > 0 else None
        nblk = _K.ln_bwd_blocks(M)
        part = torch.empty(3 * nblk * H, device=dy.device, dtype=torch.float32)
        # gamma / beta / bias gradients summed straight into the optimizer's flat fp32 buffer
        # when it exposes one (saves autograd's separate `grad += g` launch per parameter)
        gamma_p, beta_p, bias_p = ctx.params
        ctx.params = None
        tgt = [_direct_grad(gamma_p), _direct_grad(beta_p),
               _direct_grad(bias_p) if has_bias else None]
        direct = tgt[0] is not None and tgt[1] is not None and (not has_bias or tgt[2] is not None)
        if direct:
            dgamma, dbeta, dbias = tgt
        else:
            dgamma = torch.empty(H, device=dy.device, dtype=torch.float32)
            dbeta = torch.empty_like(dgamma)
            dbias = torch.empty_like(dgamma) if has_bias else None
        _K.ln_bwd(dy2.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g32.data_ptr(),
                  ds.data_ptr(), _p(da), part.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(),
                  _p(dbias), M, H, p, seed, 0.0, 0, _st(), int(direct))
        if direct:
            for q in (gamma_p, beta_p, bias_p if has_bias else None):
                if q is not None:
                    _grad_ready(q)
            dgamma = dbeta = dbias = None
        d_a = (da if da is not None else ds).view(shape)
        d_res = ds.view(shape) if has_res else None
        if d_res is not None and ctx.res_ref is not None:
            ctx.res_ref._dtf_pending_grad = d_res
            d_res = None
        ctx.res_ref = None
        return (d_a, dbias, d_res, dgamma, dbeta, None, None, None)


def layer_norm(x, gamma, beta, eps=1e-12):
    return _FusedLayerNorm.apply(x, None, None, gamma, beta, 0.0, eps)


def bias_dropout_add_layer_norm(a, bias, residual, gamma, beta, p=0.0, training=True, eps=1e-12,
                                residual_to_dense=False):
    return _FusedLayerNorm.apply(a, bias, residual, gamma, beta, p if training else 0.0, eps,
                                 bool(residual_to_dense and _RESIDUAL_TO_DENSE
                                      and residual is not None and residual.requires_grad))


# ----------------------------------------------------------------------------- embeddings
class _EmbeddingLayerNorm(torch.autograd.Function):
    """y = dropout(LN(word[ids] + pos[s] + type[tt]))   -> [B*S, H] bf16."""

    @staticmethod
    def forward(ctx, ids, tt, word, pos, typ, gamma, beta, p, eps):
        B, S = ids.shape
        H = word.shape[1]
        M = B * S
        ids_c = ids.reshape(-1).long().contiguous()
        tt_c = None if tt is None else tt.reshape(-1).long().contiguous()
        wb, pb, tb = _bf16_weight(word), _bf16_weight(pos), _bf16_weight(typ)
        y = torch.empty(M, H, device=ids.device, dtype=_BF16)
        s = torch.empty_like(y)
        mean = torch.empty(M, device=ids.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        seed = next_seed() if p > 0 else 0
        g32, b32 = _f32(gamma), _f32(beta)
        _K.ln_fwd(0, 0, 0, g32.data_ptr(), b32.data_ptr(), y.data_ptr(), s.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), M, H, float(eps), 0.0, 0, float(p), seed,
                  ids_c.data_ptr(), _p(tt_c), wb.data_ptr(), pb.data_ptr(), tb.data_ptr(), S,
                  _st())
        ctx.save_for_backward(ids_c, tt_c if tt_c is not None else ids_c, s, mean, rstd, g32)
        ctx.cfg = (B, S, H, M, float(p), seed, tt is not None, word.shape[0], pos.shape[0],
                   typ.shape[0])
        return y

    @staticmethod
    def backward(ctx, dy):
        ids_c, tt_c, s, mean, rstd, g32 = ctx.saved_tensors
        B, S, H, M, p, seed, has_tt, V, P, NT = ctx.cfg
        dy2 = dy.to(_BF16).contiguous()
        ds = torch.empty_like(dy2)
        nblk = _K.ln_bwd_blocks(M)
        part = torch.empty(2 * nblk * H, device=dy.device, dtype=torch.float32)
        dgamma = torch.empty(H, device=dy.device, dtype=torch.float32)
        dbeta = torch.empty_like(dgamma)
        _K.ln_bwd(dy2.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g32.data_ptr(),
                  ds.data_ptr(), 0, part.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), 0, M, H,
                  0.0, 0, p, seed, _st())
        dword = torch.zeros(V, H, device=dy.device, dtype=torch.float32)
        sorted_ids, perm = torch.sort(ids_c, stable=True)
        _K.segment_sum(sorted_ids.data_ptr(), perm.data_ptr(), ds.data_ptr(), dword.data_ptr(),
                       M, H, _st())
        dpos = torch.zeros(P, H, device=dy.device, dtype=torch.float32)
        if NT <= 4 and H % 8 == 0:
            # position sums over the batch and per-type sums in one pass over ds
            dtype_ = torch.empty(NT, H, device=dy.device, dtype=torch.float32)
            ws = torch.empty(_K.pos_type_grad_ws_floats(S, H, NT), device=dy.device,
                             dtype=torch.float32)
            _K.pos_type_grad(ds.data_ptr(), tt_c.data_ptr() if has_tt else 0, B, S, H, NT,
                             dpos.data_ptr(), dtype_.data_ptr(), ws.data_ptr(), _st())
        else:
            dpos[:S] = ds.view(B, S, H).float().sum(0)
            if has_tt:
                onehot = torch.nn.functional.one_hot(tt_c, NT).to(_BF16)
                dtype_ = (onehot.t() @ ds).float()
            else:
                dtype_ = torch.zeros(NT, H, device=dy.device, dtype=torch.float32)
                dtype_[0] = ds.float().sum(0)
        return None, None, dword, dpos, dtype_, dgamma, dbeta, None, None


def embedding_layer_norm(ids, token_type_ids, word, pos, typ, gamma, beta, p=0.0, training=True,
                         eps=1e-12):
    return _EmbeddingLayerNorm.apply(ids, token_type_ids, word, pos, typ, gamma, beta,
                                     p if training else 0.0, eps)


# ----------------------------------------------------------------------------- bias + GELU
class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, bias):
        N = a.shape[-1]
        a2 = a.reshape(-1, N).contiguous()
        y = torch.empty_like(a2)
        b32 = _f32(bias)
        _K.bias_gelu_fwd(a2.data_ptr(), _p(b32), y.data_ptr(), a2.shape[0], N, _st())
        ctx.save_for_backward(a2, b32)
        ctx.cfg = (bias is not None, a.shape)
        ctx.bias_p = bias
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, dy):
        a2, b32 = ctx.saved_tensors
        has_bias, shape = ctx.cfg
        M, N = a2.shape
        dy2 = dy.reshape(M, N).to(_BF16).contiguous()
        da = torch.empty_like(a2)
        bias_p, ctx.bias_p = ctx.bias_p, None
        target = _direct_grad(bias_p) if has_bias else None
        dbias = target if target is not None else (
            torch.empty(N, device=dy.device, dtype=torch.float32) if has_bias else None)
        part = torch.empty(_K.bias_gelu_bwd_blocks(M) * N, device=dy.device,
                           dtype=torch.float32) if has_bias else None
        _K.bias_gelu_bwd(dy2.data_ptr(), a2.data_ptr(), _p(b32), da.data_ptr(), _p(part),
                         _p(dbias), M, N, _st(), int(target is not None))
        if target is not None:
            _grad_ready(bias_p)
            dbias = None
        return da.view(shape), dbias


def bias_gelu(a, bias=None):
    return _BiasGelu.apply(a, bias)


def gelu(x):
    return _BiasGelu.apply(x, None)


# ----------------------------------------------------------------------------- attention
class _AttentionQKV(torch.autograd.Function):
    """Multi-head self-attention over the fused QKV projection.

    qkv: [B*S, 3*H*64] bf16 (columns: all query heads, all key heads, all value heads);
    mask: additive fp32 [B, S] key mask (0 keep / -10000 pad) or None.  Returns [B*S, H*64]."""

    @staticmethod
    def forward(ctx, qkv, mask, B, S, heads, p, scale):
        if qkv.shape[-1] != 3 * heads * AD:
            raise ValueError(f"qkv last dim {qkv.shape[-1]} != 3*heads*{AD}")
        if S % 64:
            raise ValueError("native attention needs seq_len % 64 == 0")
        q = qkv.contiguous()
        m = None if mask is None else mask.float().contiguous()
        out = torch.empty(B * S, heads * AD, device=qkv.device, dtype=_BF16)
        lse = torch.empty(B * heads * S, device=qkv.device, dtype=torch.float32)
        seed = next_seed() if p > 0 else 0
        # with dropout at S == 128 the forward keeps its keep decisions (1 bit per score) for
        # the fused backward, which then skips re-hashing them
        nk = _K.attn_keep_words(B, S, heads, float(p))
        keep = torch.empty(nk, device=qkv.device, dtype=torch.int32) if nk else None
        _K.attn_fwd(q.data_ptr(), _p(m), out.data_ptr(), lse.data_ptr(), B, S, heads,
                    float(scale), float(p), seed, _st(), _p(keep))
        ctx.keep = keep
        ctx.save_for_backward(q, m if m is not None else lse, out, lse)
        ctx.cfg = (B, S, heads, float(p), seed, float(scale), m is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, m, out, lse = ctx.saved_tensors
        B, S, heads, p, seed, scale, has_mask = ctx.cfg
        do = dout.to(_BF16).contiguous()
        dqkv = torch.empty_like(q)
        delta = torch.empty_like(lse)
        # the fused S == 128 backward also leaves per-sequence column sums of dqkv: the QKV
        # projection's bias gradient is then a B-row sum instead of a pass over dqkv
        part = None
        if _K.attn_bwd_fused(S):
            part = torch.empty(B, 3 * heads * AD, device=q.device, dtype=torch.float32)
        keep, ctx.keep = ctx.keep, None
        if keep is not None and not _K.attn_keep_words(B, S, heads, float(p)):
            keep = None          # knobs changed between forward and backward: re-hash
        _K.attn_bwd(q.data_ptr(), m.data_ptr() if has_mask else 0, out.data_ptr(), do.data_ptr(),
                    lse.data_ptr(), delta.data_ptr(), dqkv.data_ptr(), B, S, heads, scale, p, seed,
                    _st(), _p(part), _p(keep))
        if part is not None:
            # valid only for this exact tensor and version (an in-place add would change it)
            dqkv._dtf_colsum_part = (part, B, dqkv._version)
        return dqkv, None, None, None, None, None, None


def attention_qkv(qkv, mask, batch, seq_len, heads, p=0.0, training=True, scale=None):
    scale = AD ** -0.5 if scale is None else scale
    return _AttentionQKV.apply(qkv, mask, batch, seq_len, heads, p if training else 0.0, scale)


def attention(q, k, v, mask=None, scale=None):
    """[B, H, S, 64] q/k/v API (packs into the fused layout; used by generic callers)."""
    B, H, S, D = q.shape
    if D != AD:
        raise ValueError("native attention supports head_dim 64")
    qkv = torch.cat([t.permute(0, 2, 1, 3).reshape(B * S, H * D) for t in (q, k, v)], dim=1)
    m = None if mask is None else mask.reshape(B, S)
    out = attention_qkv(qkv.to(_BF16), m, B, S, H, 0.0, False, scale)
    return out.view(B, S, H, D).permute(0, 2, 1, 3)


# ----------------------------------------------------------------------------- MLM loss
class _MlmLoss(torch.autograd.Function):
    """``vocab``: the class count when the logits rows are padded past it (the tied decoder's
    vocabulary padded to a multiple of 64): padding columns are not classes and get an exact zero
    gradient."""

    @staticmethod
    def forward(ctx, logits, labels, weights, vocab=None):
        N, ld = logits.shape
        V = ld if vocab is None else int(vocab)
        if not 0 < V <= ld:
            raise ValueError(f"mlm_loss: vocab {vocab} outside the logits width {ld}")
        lg = logits.to(_BF16).contiguous()
        lab = labels.reshape(-1).long().contiguous()
        w = None if weights is None else weights.reshape(-1).float().contiguous()
        denom = (w.sum() if w is not None else torch.tensor(float(N), device=lg.device)).reshape(1)
        denom = denom.float().contiguous()
        rows = torch.empty(N, device=lg.device, dtype=torch.float32)
        grad = torch.empty_like(lg)
        _K.mlm_xent(lg.data_ptr(), lab.data_ptr(), _p(w), denom.data_ptr(), N, V, ld,
                    rows.data_ptr(), grad.data_ptr(), _st())
        ctx.save_for_backward(grad)
        ctx.ldt = logits.dtype
        # Optimizer.compute_gradients runs loss.backward() with the implicit unit gradient and
        # says so through this flag (ctx is the output's grad_fn): the [N, vocab] gradient is
        # then handed on as computed, without a full read + write pass multiplying it by 1
        ctx.dtf_unit_grad_ok = True
        ctx.dtf_unit_grad = False
        return rows.sum()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        if ctx.dtf_unit_grad and grad.dtype == ctx.ldt:
            return grad, None, None, None
        return (grad * g.to(grad.dtype)).to(ctx.ldt), None, None, None


def mlm_loss(logits, labels, weights=None, vocab=None):
    return _MlmLoss.apply(logits, labels, weights, vocab)
