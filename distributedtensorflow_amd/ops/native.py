"""Autograd wrappers around the HIP/CDNA4 kernels in ``csrc/kernels`` (module ``_dtf_hip``).

Every function here launches OUR kernels on the caller's current torch stream; there is no
PyTorch fallback: if the extension is missing this module raises at import (a GPU box without
the built ``.so`` must fail loudly, not silently run eager PyTorch).

Precision contract (mixed precision, TF-style "float32 variables, bf16 compute"):
  * activations bf16 NHWC;
  * weights: fp32 master parameters; kernels consume the bf16 shadow the optimizer maintains
    (``param._dtf_shadow``) or a cast made on the fly;
  * weight gradients are produced directly in fp32 (MFMA fp32 accumulate, no bf16 round trip).
"""
from __future__ import annotations

import os

import torch

from .records import BnDeferred as _BnDeferred  # noqa: F401  (deferred-work records)
from .records import GradSlot as _GradSlot
from .records import LazyBnDx as _LazyBnDx
from .records import LazyStemDz as _LazyStemDz
from .records import MaskedGrad as _MaskedGrad
from .records import Recompute as _Recompute
from .records import end_step as end_step  # noqa: F401
from .reference import resolve_padding, space_to_depth_operands  # noqa: F401

try:
    from .._lib import _dtf_hip as _K  # noqa: N812
except ImportError as e:  # pragma: no cover - exercised on boxes without a build
    raise ImportError(
        "distributedtensorflow_amd HIP extension (_lib/_dtf_hip*.so) is not built; run "
        "`python -m distributedtensorflow_amd._build` (hipcc --offload-arch=gfx950). "
        f"Original error: {e}") from e

_BF16 = torch.bfloat16
_DENSE_IMPL = os.environ.get("DTF_DENSE", "native")     # native | library (hipBLASLt)

# kernel-variant switches for A/B runs on one box (defaults = the measured best)
if os.environ.get("DTF_WGRAD_MODE"):
    _K.wgrad_set_dma_mode(int(os.environ["DTF_WGRAD_MODE"]))
if os.environ.get("DTF_WGRAD_PP"):       # ping-pong wgrad: 0 off, n: split-K target of n rounds
    _K.wgrad_set_pp(int(os.environ["DTF_WGRAD_PP"]))
if os.environ.get("DTF_WGRAD_DENSE"):    # ping-pong wgrad's decode-free one-tap form: 0 off
    _K.wgrad_set_dense(int(os.environ["DTF_WGRAD_DENSE"]))
if os.environ.get("DTF_WGRAD_PIPE"):
    _K.wgrad_set_pipe(int(os.environ["DTF_WGRAD_PIPE"]))
if os.environ.get("DTF_CONV_DMA"):
    _K.conv_set_dma_mode(int(os.environ["DTF_CONV_DMA"]))
if os.environ.get("DTF_CONV_HALO"):
    _K.conv_set_halo(int(os.environ["DTF_CONV_HALO"]))
if os.environ.get("DTF_WGRAD_HALO"):
    _K.wgrad_set_halo(int(os.environ["DTF_WGRAD_HALO"]))
if os.environ.get("DTF_CONV_STEM_HALO"):
    _K.conv_set_stem_halo(int(os.environ["DTF_CONV_STEM_HALO"]))
if os.environ.get("DTF_CONV_HALO_STRIPS"):     # bit f: two strips per block for halo family f
    _K.conv_set_halo_strips(int(os.environ["DTF_CONV_HALO_STRIPS"]))
if os.environ.get("DTF_CONV_HALO_FREG"):       # bit f: halo family f streams its filter via VGPRs
    _K.conv_set_halo_freg(int(os.environ["DTF_CONV_HALO_FREG"]))
if os.environ.get("DTF_CONV_SMALL_K"):
    _K.conv_set_small_k(int(os.environ["DTF_CONV_SMALL_K"]))
if os.environ.get("DTF_GEMM_STREAM"):   # row-streaming GEMM for output-heavy shapes (default on)
    _K.gemm_set_stream(int(os.environ["DTF_GEMM_STREAM"]))
if os.environ.get("DTF_C1_W16"):        # stage-0 fused c3 backward as 16-wave blocks (default 0)
    _K.conv1x1_bwd_set_w16(int(os.environ["DTF_C1_W16"]))
if os.environ.get("DTF_GEMM_GROUP_M"):  # grouped tile order of the dense GEMMs (0: N fastest)
    _K.gemm_set_group(int(os.environ["DTF_GEMM_GROUP_M"]))
if os.environ.get("DTF_BN_GRID_CAP"):     # BN row-sweep grid cap override (2048 = round-2 grids)
    _K.bn_set_grid_cap(int(os.environ["DTF_BN_GRID_CAP"]))
if os.environ.get("DTF_BN_STATS_BLOCKS"):  # BN reduce-pass block target (1024 = round-2)
    _K.bn_set_stats_blocks(int(os.environ["DTF_BN_STATS_BLOCKS"]))
if os.environ.get("DTF_GEMM_PP2"):      # round-5 persistent GEMM: bit 0 gemm_nt (default), 1 convs
    _K.gemm_set_pp2(int(os.environ["DTF_GEMM_PP2"]))
if os.environ.get("DTF_STORE_NT"):      # non-temporal output stores: bit 0 conv, 1 GEMM, 2 BN
    _nt = int(os.environ["DTF_STORE_NT"])
    _K.conv_set_nt(_nt & 1)
    _K.gemm_set_nt((_nt >> 1) & 1)
    _K.bn_set_nt(7 if _nt & 4 else 0)


def _st():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return 0 if t is None else t.data_ptr()


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _bf16_weight(w: torch.Tensor) -> torch.Tensor:
    s = getattr(w, "_dtf_shadow", None)
    if s is not None and s.dtype == _BF16:
        return s
    return w.detach().to(_BF16)


_DIRECT_GRAD = os.environ.get("DTF_DIRECT_GRAD", "1") == "1"


def _direct_grad(p):
    """The fp32 flat-buffer gradient view of parameter ``p`` when our kernels may accumulate into
    it directly (saving autograd's separate ``grad += g`` launch per parameter), else None.

    After writing, the op calls :func:`_grad_ready` so gradient-bucketing strategies see the
    same "this parameter's gradient is complete" event AccumulateGrad would have raised.  Valid
    for parameters consumed once per step (convs / BN in ResNet); set DTF_DIRECT_GRAD=0 to route
    everything through autograd (e.g. for weights shared across several calls)."""
    if not _DIRECT_GRAD or p is None or not getattr(p, "_dtf_flat", False):
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous():
        return None
    return g


# Kernel variants measured neutral or slower (the wgrad DEEP / EARLY schedules, the per-row and
# readlane pixel decodes, deeper halo filter rings) are no longer reachable from the environment:
# their C++ setters stay for the bit-identity tests; the conv weight gradient on a side stream
# (neutral at b1984, profiles/measurements/r5_wgrad_side_stream_ab.jsonl) was removed.


def enable_timing_probe(name, value=1):
    """Tools only: switch on a timing probe that produces WRONG results (``"bnl"`` the BN-on-load
    forward without its y stores, ``"stream_bnb"`` the BN-backward stream GEMM epilogue probes).
    They exist only in a probe build (``DTF_HIP_EXTRA_FLAGS=-DDTF_PROBES``); the default build
    raises.  Never reachable from the environment or from training code."""
    setter = {"bnl": _K.conv_set_bnl_probe, "stream_bnb": _K.gemm_stream_set_bnb_probe}[name]
    setter(int(value))


def _grad_ready(p):
    cb = getattr(p, "_dtf_grad_ready", None)
    if cb is not None:
        cb()


def _check_cuda_bf16(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != _BF16):
            raise TypeError(f"native op expects CUDA bf16 tensors, got {t.dtype} on {t.device}")


# ----------------------------------------------------------------------------- convolution

def _conv_geom_fwd(x, K, R, S, stride, padding):
    n, h, w, c = x.shape
    sh, sw = _pair(stride)
    pt, pb, pl, pr = resolve_padding(padding, h, w, R, S, stride)
    P = (h + pt + pb - R) // sh + 1
    Q = (w + pl + pr - S) // sw + 1
    return n, h, w, c, P, Q, sh, sw, pt, pl


def _fwd_geom(xshape, K, taps, P, Q, sh, sw, Ho, Wo, osh=1, osw=1, oh0=0, ow0=0, accumulate=False):
    n, h, w, c = xshape
    kpad = -(-(len(taps) * c) // 32) * 32
    return [n, h, w, c, P, Q, sh, sw, K, kpad, Ho, Wo, osh, osw, oh0, ow0, int(accumulate)]


def _launch_fwd(x, wmat, K, taps, P, Q, sh, sw, out, Ho, Wo, osh=1, osw=1, oh0=0, ow0=0,
                stats=None, accumulate=False, bnb=(), acc_from=None, bias=None, relu=False,
                bnl=None):
    """wmat: [K, T*C] bf16 (rows zero-padded here to a multiple of 32 for the gather path).
    ``acc_from``: a :class:`_MaskedGrad` the epilogue adds (as dy * mask) instead of reading
    ``out`` back (geom acc mode 2)."""
    n, h, w, c = x.shape
    dh = [t[0] for t in taps]
    dw = [t[1] for t in taps]
    kdim = len(taps) * c
    kpad = -(-kdim // 32) * 32
    if kpad != kdim:
        padded = torch.zeros(K, kpad, device=x.device, dtype=_BF16)
        padded[:, :kdim] = wmat
        wmat = padded
    geom = [n, h, w, c, P, Q, sh, sw, K, kpad, Ho, Wo, osh, osw, oh0, ow0,
            2 if acc_from is not None else int(accumulate)]
    if acc_from is not None:
        if tuple(acc_from.dy.shape) != tuple(out.shape) or acc_from.dy.dtype != _BF16:
            raise ValueError("masked residual gradient does not match the dgrad output")
        _K.conv_igemm(x.data_ptr(), wmat.data_ptr(), out.data_ptr(), geom, dh, dw, 64, _st(),
                      _p(stats), list(bnb), acc_from.dy.data_ptr(), acc_from.mask.data_ptr())
        return
    if bnl is not None:
        # BN + ReLU on load: x is the BatchNorm INPUT, the kernel writes the normalised tensor
        # (bnl.y) itself -- the deferred apply pass never runs
        _K.conv_igemm(bnl.x.data_ptr(), wmat.data_ptr(), out.data_ptr(), geom, dh, dw, 64, _st(),
                      _p(stats), list(bnb), 0, 0, 0, 0, bnl.scale.data_ptr(),
                      bnl.shift.data_ptr(), bnl.y().data_ptr())
        bnl.done = True
        return
    _K.conv_igemm(x.data_ptr(), wmat.data_ptr(), out.data_ptr(), geom, dh, dw, 64, _st(),
                  _p(stats), list(bnb), 0, 0, _p(bias), int(relu))


def _bnl_pending(x):
    rec = getattr(x, "_dtf_bnl", None)
    return rec if rec is not None and not rec.done else None


def conv2d_forward(x, w_bf16, stride, padding, stats=None, bias=None, relu=False):
    """x [N,H,W,C] bf16, w [K,R,S,C] bf16 -> y [N,P,Q,K].  ``stats``: fp32 workspace that also
    receives the per-M-tile BatchNorm partial sums of y (see conv2d(bn_stats=True))."""
    K, R, S, C = w_bf16.shape
    n, h, wd, c, P, Q, sh, sw, pt, pl = _conv_geom_fwd(x, K, R, S, stride, padding)
    assert c == C, (x.shape, w_bf16.shape)
    if bias is None and not relu and _gemm_1x1(C, K, R, S, stride, (pt, pl)) and \
            x.is_contiguous() and w_bf16.is_contiguous():
        if _bnl_pending(x) is not None:
            _bnl_pending(x).materialize()
        y = gemm_nt(x.view(-1, C), w_bf16.view(K, C), stats=stats)
        return y.view(n, P, Q, K)
    taps = [(r - pt, s - pl) for r in range(R) for s in range(S)]
    y = torch.empty(n, P, Q, K, device=x.device, dtype=_BF16)
    bnl = _bnl_pending(x)
    if bnl is not None and (bias is not None or relu or not _K.conv_bnl_ok(
            _fwd_geom(x.shape, K, taps, P, Q, sh, sw, P, Q), [t[0] for t in taps],
            [t[1] for t in taps])):
        bnl.materialize()
        bnl = None
    _launch_fwd(x, w_bf16.reshape(K, R * S * C), K, taps, P, Q, sh, sw, y, P, Q, stats=stats,
                bias=bias, relu=relu, bnl=bnl)
    return y


# ---- batched dgrad filters: every conv forward registers its bf16 filter; the first data-gradient
# of the step transposes ALL registered filters [K,T,C] -> [C,T,K] in one launch
# (csrc/kernels/conv.hip filter_transpose_kernel) instead of one copy kernel per conv.  Keyed by
# the shadow's data_ptr (the optimizer rewrites the shadow in place once per step, after backward);
# a forward re-registration invalidates the previous step's copy.
_WT_PENDING = {}
_WT_CACHE = {}
_BATCH_WT = os.environ.get("DTF_BATCH_FILTER_T", "1") == "1"


def _register_dgrad_filter(wb):
    if _BATCH_WT:
        key = wb.data_ptr()
        _WT_CACHE.pop(key, None)
        _WT_PENDING[key] = wb


def _dgrad_filter(wflat):
    """[K, T, C] bf16 filter -> contiguous [C, T, K]."""
    key = wflat.data_ptr()
    t = _WT_CACHE.get(key)
    if t is not None and t.shape == (wflat.shape[2], wflat.shape[1], wflat.shape[0]):
        return t
    if key in _WT_PENDING:
        items = list(_WT_PENDING.values())
        _WT_PENDING.clear()
        _WT_CACHE.clear()            # bounded: only the current step's filters are kept
        outs = [torch.empty(w.shape[3], w.shape[1] * w.shape[2], w.shape[0], device=w.device,
                            dtype=_BF16) for w in items]
        _K.filter_transpose([w.data_ptr() for w in items], [o.data_ptr() for o in outs],
                            [w.shape[0] for w in items], [w.shape[1] * w.shape[2] for w in items],
                            [w.shape[3] for w in items], _st())
        for w, o in zip(items, outs):
            _WT_CACHE[w.data_ptr()] = o
        t = _WT_CACHE.get(key)
        if t is not None and t.shape == (wflat.shape[2], wflat.shape[1], wflat.shape[0]):
            return t
    return wflat.permute(2, 1, 0).contiguous()


def conv2d_dgrad(dy, w_bf16, x_shape, stride, padding, out=None, bnb=None, acc_from=None):
    """dX of conv2d via per-phase-class tap tables (see csrc/kernels/conv.hip header).
    ``out``: an existing bf16 gradient of x to ADD into.  ``bnb``: the BatchNorm whose output x
    is (its ``_dtf_bnb`` record): the epilogue then also emits that BN's backward partial sums,
    attached to the result as ``_dtf_bnb_part`` (see :class:`_BatchNorm`).  ``acc_from``: a
    :class:`_MaskedGrad` to add (single-phase launches only: stride 1)."""
    K, R, S, C = w_bf16.shape
    n, h, wd, c = x_shape
    sh, sw = _pair(stride)
    pt, pb, pl, pr = resolve_padding(padding, h, wd, R, S, stride)
    dx = None
    wflat = w_bf16.reshape(K, R * S, C)
    if isinstance(bnb, _DualBnb) and not (_gemm_1x1(K, C, R, S, stride, (pt, pl)) and
                                          _stream_bnb_ok(K, C)):
        bnb = None       # the dual sums ride only on the streamed 1x1 data gradient
    if _gemm_1x1(K, C, R, S, stride, (pt, pl)) and (bnb is None or _stream_bnb_ok(K, C)):
        # 1x1 stride 1: dX[M, C] = dY[M, K] . Wt[C, K]^T on the GEMM kernel, residual
        # gradients (materialised or masked) folded into its epilogue
        M = n * h * wd
        wt = _dgrad_filter(wflat).view(C, K)
        dyc = dy.contiguous().view(M, K)
        if bnb is not None:
            return _dgrad_1x1_bnb(dyc, wt, M, C, K, (n, h, wd, C), out, acc_from, bnb)
        if out is not None:
            o2 = out.view(M, C)
            gemm_nt(dyc, wt, out=o2, cin=o2)
            if acc_from is not None:
                out.add_(acc_from.materialize())
            return out
        dx = gemm_nt(dyc, wt, acc_from=acc_from)
        return dx.view(n, h, wd, C)
    need_zero = False
    launches = []
    for a in range(sh):
        for b in range(sw):
            Pc = (h - a + sh - 1) // sh
            Qc = (wd - b + sw - 1) // sw
            if Pc <= 0 or Qc <= 0:
                continue
            taps, idx = [], []
            for r in range(R):
                if (a + pt - r) % sh:
                    continue
                for s in range(S):
                    if (b + pl - s) % sw:
                        continue
                    taps.append(((a + pt - r) // sh, (b + pl - s) // sw))
                    idx.append(r * S + s)
            if not taps:
                need_zero = True
                continue
            launches.append((a, b, Pc, Qc, taps, idx))
    if acc_from is not None and (out is not None or len(launches) != 1 or need_zero):
        out = acc_from.materialize() if out is None else out.add_(acc_from.materialize())
        acc_from = None
    acc = out is not None
    # accumulating: phases without taps contribute zero (nothing to add); the phase launches
    # partition the output, so every element is read-modified-written at most once
    dx = out if acc else (torch.zeros if need_zero else torch.empty)(
        n, h, wd, C, device=dy.device, dtype=_BF16)
    acc = acc or acc_from is not None
    dyc = dy.contiguous()
    part, row0 = None, 0
    if bnb is not None:
        xb, stats, mask, relu, has_res, tok = bnb
        _materialized(xb)              # a lazy c3 output: the tap kernels read it
        # slab rows of exactly the kernel each launch takes (the halo kernels: one per block)
        rows = [_K.conv_tile_rows(_fwd_geom(dyc.shape, C, taps, Pc, Qc, 1, 1, h, wd, sh, sw, a, b,
                                            acc),
                                  [t[0] for t in taps], [t[1] for t in taps], 1)
                for (a, b, Pc, Qc, taps, _) in launches]
        G = sum(rows)
        part = torch.empty(_K.bn_workspace_floats_g(G, C), device=dy.device, dtype=torch.float32)
        mkind = (1 if has_res else 2) if relu else 0
        fsc, fsh = (stats[2].data_ptr(), stats[3].data_ptr()) if mkind == 2 else (0, 0)
        base = [xb.data_ptr(), stats[0].data_ptr(), stats[1].data_ptr(), fsc, fsh,
                _p(mask) if mkind == 1 else 0, part.data_ptr(), mkind]
    def class_filter(idx):
        if len(idx) == R * S:
            return _dgrad_filter(wflat)                        # [C, T, K]
        sel = wflat[:, _tap_index(idx, dy.device), :]
        return sel.permute(2, 1, 0).contiguous()

    if (_DGRAD_GROUPED and len(launches) > 1 and acc_from is None and part is None and
            len({(l[2], l[3]) for l in launches}) == 1 and K % 32 == 0):
        # every phase class in ONE launch (csrc/kernels/conv.hip conv_igemm_grouped_kernel),
        # classes interleaved per M-tile: 1.00 vs 1.15 ms for the 56x56x128 stride-2 layer at
        # b1984.  Not with the fused BN-backward sums: that form ran 1.97 vs 1.78 ms
        # (tools/conv_gap.py, profiles/r6).  False: the register kernel is not the one these
        # classes would take -- launched one by one below
        mats = [class_filter(l[5]).reshape(C, -1) for l in launches]
        Pc, Qc = launches[0][2], launches[0][3]
        geom = _fwd_geom(dyc.shape, C, launches[0][4], Pc, Qc, 1, 1, h, wd, sh, sw, 0, 0, acc)
        if _K.conv_igemm_grouped(dyc.data_ptr(), dx.data_ptr(), geom,
                                 [m.data_ptr() for m in mats], [l[0] for l in launches],
                                 [l[1] for l in launches], [len(l[4]) * K for l in launches],
                                 [[t[0] for t in l[4]] for l in launches],
                                 [[t[1] for t in l[4]] for l in launches], _st(), [], []):
            return dx
    for li, (a, b, Pc, Qc, taps, idx) in enumerate(launches):
        wd_mat = class_filter(idx)
        extra = ()
        if part is not None:
            extra = base + [row0]
            row0 += rows[li]
        _launch_fwd(dyc, wd_mat.reshape(C, -1), C, taps, Pc, Qc, 1, 1, dx, h, wd, sh, sw, a, b,
                    accumulate=acc, bnb=extra, acc_from=acc_from)
    if part is not None:
        dx._dtf_bnb_part = (part, G, n * h * wd, C, tok, dx._version)
    return dx


def _stream_bnb_ok(K, C):
    """The 1x1 data gradient [M, K] x [C, K]^T runs on the row-streaming GEMM (reduction K in
    {64, 128, 256}, output C >= K), which can also emit the consuming BatchNorm's backward sums."""
    return _GEMM_STREAM and K in (64, 128, 256) and C >= K and C % 64 == 0 and C <= 2048


class _DualBnb:
    """The consuming conv's record of relu(BN(x) + BN_p(xp)) (:class:`_BatchNormAddBatchNorm`):
    its streamed data gradient also emits both BatchNorms' backward sums."""
    __slots__ = ("x", "stats", "mask", "xp", "stats_p", "tok")

    def __init__(self, x, stats, mask, xp, stats_p, tok):
        self.x, self.stats, self.mask, self.xp, self.stats_p, self.tok = \
            x, stats, mask, xp, stats_p, tok


def _dgrad_1x1_bnb(dyc, wt, M, C, K, xshape, out, acc_from, bnb):
    """1x1 data gradient on the row-streaming GEMM whose epilogue also reduces the BN backward
    sums (sum dz, sum dz x-hat) of the BatchNorm that produced x: its separate reduce pass over
    (dy, x) is skipped (the sums ride on the data gradient still in registers; only x is read).
    A :class:`_DualBnb` adds the shortcut BatchNorm's sums (its dual reduce pass is skipped)."""
    if isinstance(bnb, _DualBnb):
        return _dgrad_1x1_bnb_dual(dyc, wt, M, C, K, xshape, out, acc_from, bnb)
    xb, stats, mask, relu, has_res, tok = bnb
    if out is not None and acc_from is not None:
        out.add_(acc_from.materialize())
        acc_from = None
    o2 = out.view(M, C) if out is not None else torch.empty(M, C, device=dyc.device, dtype=_BF16)
    G = _K.gemm_tile_rows(M)
    part = torch.empty(_K.bn_workspace_floats_g(G, C), device=dyc.device, dtype=torch.float32)
    kind = (1 if has_res else 2) if relu else 0
    # lazy x3 (RC): the epilogue recomputes the BN input from the producing conv's operands
    rc = getattr(xb, "_dtf_recompute", None)
    if rc is not None and (rc.done or kind != 1 or K > 128 or rc.k3 not in (64, 128)):
        _materialized(xb)
        rc = None
    y2, w3, k3 = (rc.y.data_ptr(), rc.wb.data_ptr(), rc.k3) if rc is not None else (0, 0, 0)
    _K.gemm_stream_bnb(dyc.data_ptr(), wt.data_ptr(), o2.data_ptr(), M, C, K, K, K, C,
                       o2.data_ptr() if out is not None else 0,
                       acc_from.dy.data_ptr() if acc_from is not None else 0,
                       acc_from.mask.data_ptr() if acc_from is not None else 0,
                       xb.data_ptr(), stats[0].data_ptr(), stats[1].data_ptr(),
                       stats[2].data_ptr() if kind == 2 else 0,
                       stats[3].data_ptr() if kind == 2 else 0,
                       _p(mask) if kind == 1 else 0, kind, part.data_ptr(), _st(), y2, w3, k3)
    dx = o2.view(xshape)
    # valid only for this exact gradient: autograd may add another contribution IN PLACE
    # (a residual gradient summed outside the epilogue), which bumps the version counter
    dx._dtf_bnb_part = (part, G, M, C, tok, dx._version)
    return dx


def _dgrad_1x1_bnb_dual(dyc, wt, M, C, K, xshape, out, acc_from, d):
    _materialized(d.x)
    _materialized(d.xp)
    if out is not None and acc_from is not None:
        out.add_(acc_from.materialize())
        acc_from = None
    o2 = out.view(M, C) if out is not None else torch.empty(M, C, device=dyc.device, dtype=_BF16)
    G = _K.gemm_tile_rows(M)
    ws = _K.bn_workspace_floats_g(G, C)
    part = torch.empty(ws, device=dyc.device, dtype=torch.float32)
    part_p = torch.empty(ws, device=dyc.device, dtype=torch.float32)
    _K.gemm_stream_bnb_dual(dyc.data_ptr(), wt.data_ptr(), o2.data_ptr(), M, C, K, K, K, C,
                            o2.data_ptr() if out is not None else 0,
                            acc_from.dy.data_ptr() if acc_from is not None else 0,
                            acc_from.mask.data_ptr() if acc_from is not None else 0,
                            d.x.data_ptr(), d.stats[0].data_ptr(), d.stats[1].data_ptr(),
                            d.mask.data_ptr(), part.data_ptr(), d.xp.data_ptr(),
                            d.stats_p[0].data_ptr(), d.stats_p[1].data_ptr(), part_p.data_ptr(),
                            _st())
    dx = o2.view(xshape)
    dx._dtf_bnb_part = (part, G, M, C, d.tok, dx._version)
    dx._dtf_bnb_part_p = part_p
    return dx


_TAP_IDX = {}


def _tap_index(idx, device):
    """Device index tensor of a dgrad phase class's taps, built once (no host-to-device copy in
    the step: a HIP-graph capture of the step must not contain one)."""
    key = (tuple(idx), device)
    t = _TAP_IDX.get(key)
    if t is None:
        t = _TAP_IDX[key] = torch.tensor(idx, device=device)
    return t


_WGRAD_WS_CAP = 32 << 20   # floats of split-K slab workspace per call (128 MB)


def conv2d_wgrad(x, dy, w_shape, stride, padding, out=None):
    """dW [K,R,S,C] fp32 via the MFMA wgrad kernel; deterministic split-K slab reduction.
    With ``out`` (a contiguous fp32 [K,R,S,C] buffer) the result is ADDED into it."""
    K, R, S, C = w_shape
    n, h, wd, c = x.shape
    sh, sw = _pair(stride)
    pt, pb, pl, pr = resolve_padding(padding, h, wd, R, S, stride)
    _, P, Q, _ = dy.shape
    taps = [(r - pt, s - pl) for r in range(R) for s in range(S)]
    tc = R * S * C
    geom = [n, h, wd, c, P, Q, sh, sw, K, tc]
    dhs, dws = [t[0] for t in taps], [t[1] for t in taps]
    # stage-1 3x3 layers: the halo kernel (one fp32 slab per block) when it applies
    splits = _K.conv_wgrad_halo_splits(geom, dhs, dws) or \
        _K.conv_wgrad_splits(n * P * Q, K, tc, _WGRAD_WS_CAP, R * S)
    acc = out is not None
    dW = out if acc else torch.empty(K, tc, device=x.device, dtype=torch.float32)
    ws = (torch.empty(splits * K * tc, device=x.device, dtype=torch.float32)
          if splits > 1 or acc else None)
    _K.conv_wgrad(x.data_ptr(), dy.contiguous().data_ptr(), dW.data_ptr(), _p(ws), geom,
                  dhs, dws, splits, _st(), 1, int(acc))
    return dW.reshape(K, R, S, C)


def space_to_depth_input(x, stride, pad, R, S):
    """The x half of ``reference.space_to_depth_operands`` (same layout, bit-identical) in one
    HIP pass; for an input that needs no gradient (the image)."""
    n, h, wd, c = x.shape
    s = stride
    P = (h + 2 * pad - R) // s + 1
    Q = (wd + 2 * pad - S) // s + 1
    Ho, Wo = P + -(-R // s) - 1, Q + -(-S // s) - 1
    cp = c
    while (s * s * cp) % 8:
        cp += 1
    x = x.contiguous()
    xs = torch.empty(n, Ho, Wo, s * s * cp, device=x.device, dtype=_BF16)
    _K.s2d_input(x.data_ptr(), xs.data_ptr(), n, h, wd, c, Ho, Wo, s, cp, pad, _st())
    return xs


def _pad_c8(t):
    """Zero-pad the channel (last) axis to a multiple of 8 so every 16-B load holds whole taps."""
    c = t.shape[-1]
    pc = -(-c // 8) * 8
    return t if pc == c else torch.nn.functional.pad(t, (0, pc - c))


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_master, stride, padding, stats=None, share=None):
        if _bnl_pending(x) is not None and (not x.is_contiguous() or x.shape[-1] % 8):
            _bnl_pending(x).materialize()        # BN on load needs the tensor itself as input
        xb = x.contiguous()
        ctx.share = share
        wb = _bf16_weight(w_master)
        ctx.c_orig = xb.shape[-1]
        if xb.shape[-1] % 8:
            # stem (C=3) / MNIST conv1 (C=1): pad to 8 channels -> 16-B chunk-gather kernels
            # for fwd and wgrad instead of per-element gathers (~4x faster, see tools/conv_bench)
            xb, wb = _pad_c8(xb), _pad_c8(wb)
        ctx.save_for_backward(xb, wb)
        ctx.stride, ctx.padding = stride, padding
        ctx.w_dtype = w_master.dtype
        ctx.w_param = w_master
        ctx.x_ref = x            # a residual BN may stash its residual gradient on x
        bnb = getattr(x, "_dtf_bnb", None)
        K_, R_, S_, _ = w_master.shape
        pads = resolve_padding(padding, xb.shape[1], xb.shape[2], R_, S_, stride)
        stream_bnb = (_FUSE_BN_BWD_STREAM and _gemm_1x1(K_, xb.shape[-1], R_, S_, stride,
                                                        (pads[0], pads[2]))
                      and _stream_bnb_ok(K_, xb.shape[-1]))
        halo_bnb = (_FUSE_BN_BWD_HALO and (R_, S_) == (3, 3) and tuple(_pair(stride)) == (1, 1)
                    and tuple(pads) == (1, 1, 1, 1)
                    and _halo_dgrad_shape(K_, xb.shape[-1], xb.shape[1], xb.shape[2]))
        # stride-2 3x3 data gradients (the first block of stages 2-4) run at 0.25-0.34 of the MFMA
        # roof: the BN-sum epilogue's extra read of x fits under the 128-output one
        s2_bnb = (_FUSE_BN_BWD_S2 and (R_, S_) == (3, 3) and tuple(_pair(stride)) == (2, 2)
                  and xb.shape[-1] % 32 == 0
                  and (_FUSE_BN_BWD_S2_ALL or xb.shape[-1] < 256))
        ctx.bnb = bnb if ((_FUSE_BN_BWD or stream_bnb or halo_bnb or s2_bnb) and bnb is not None
                          and xb is x) else None
        dual = getattr(x, "_dtf_bnb_dual", None)
        if dual is not None and stream_bnb and ctx.bnb is None and xb is x:
            ctx.bnb = _DualBnb(*dual)
        if x.requires_grad and xb is x and wb.is_contiguous():
            _register_dgrad_filter(wb)
        out = conv2d_forward(xb, wb, stride, padding, stats)
        ctx.stem_slot = None
        if (_FUSE_STEM_WGRAD and not x.requires_grad and _stem_wgrad_shape(xb, wb, stride, padding)
                and _K.wgrad_stem_dz_splits(xb.shape[0]) > 0):
            # the fused BN + ReLU + max-pool consuming `out` may hand d(out) over unformed
            # (_LazyStemDz): the weight gradient then forms it on load and it is never stored
            ctx.stem_slot = _GradSlot()
            out._dtf_stem_slot = ctx.stem_slot
            ctx.set_materialize_grads(False)
        return out

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        dx = dw = None
        C = ctx.c_orig
        padded = xb.shape[-1] != C
        slot, ctx.stem_slot = ctx.stem_slot, None
        rec = None
        if slot is not None:
            rec, slot.grad = slot.grad, None
        if dy is None and rec is None:
            ctx.x_ref = ctx.bnb = ctx.share = None
            return None, None, None, None, None, None
        if rec is not None and (dy is not None or not ctx.needs_input_grad[1]):
            m = rec.materialize()                # another consumer of the conv output
            dy = m if dy is None else dy + m
            rec = None
        if rec is not None:
            # the stem: dW with d(out) formed on load from the BN + ReLU + pool backward's operands
            target = _direct_grad(ctx.w_param)
            K, R, S, _ = wb.shape
            n = xb.shape[0]
            splits = _K.wgrad_stem_dz_splits(n)
            dW = target if target is not None else torch.empty(K, R * S * C, device=xb.device,
                                                                dtype=torch.float32)
            ws = torch.empty(splits * K * R * S * C, device=xb.device, dtype=torch.float32)
            _K.conv_wgrad_stem_dz(xb.data_ptr(), rec.dp.data_ptr(), rec.arg.data_ptr(),
                                  rec.x.data_ptr(), rec.gb[2].data_ptr(), rec.gb[3].data_ptr(),
                                  rec.gb[4].data_ptr(), rec.fsc.data_ptr(), rec.fsh.data_ptr(),
                                  dW.data_ptr(), ws.data_ptr(), n, int(target is not None), _st())
            rec.release()
            if target is not None:
                _grad_ready(ctx.w_param)
            else:
                dw = dW.reshape(K, R, S, C).to(ctx.w_dtype)
            ctx.x_ref = ctx.bnb = ctx.share = None
            return None, dw, None, None, None, None
        if ctx.needs_input_grad[1]:
            # weight gradient first: it only depends on dy, so the bucketed all-reduce of this
            # layer can start while dgrad still runs
            target = _direct_grad(ctx.w_param)
            if target is not None and not padded:
                conv2d_wgrad(xb, dy, wb.shape, ctx.stride, ctx.padding, out=target)
                _grad_ready(ctx.w_param)
            else:
                dw = conv2d_wgrad(xb, dy, wb.shape, ctx.stride, ctx.padding)
                if padded:
                    dw = dw[..., :C]
                if target is not None:
                    target.add_(dw)
                    _grad_ready(ctx.w_param)
                    dw = None
                else:
                    dw = dw.to(ctx.w_dtype)
        share, ctx.share = ctx.share, None
        if ctx.needs_input_grad[0] and share is not None and not padded:
            # several convs read x: the first to run backward creates dx, the others add their
            # dgrad onto it in the epilogue; only the last hands the sum to autograd
            last = share.left == 1
            dx = conv2d_dgrad(dy, wb, xb.shape, ctx.stride, ctx.padding, out=share.buf,
                              bnb=ctx.bnb if last else None)
            share.left -= 1
            share.buf = dx if share.left > 0 else None
            if share.left > 0:
                dx = None
        elif ctx.needs_input_grad[0]:
            pending = getattr(ctx.x_ref, "_dtf_pending_grad", None)
            if pending is not None and not padded and _pair(ctx.stride) == (1, 1):
                # identity shortcut: the block's final BN left d(residual) here; accumulate this
                # conv's dgrad onto it in the epilogue instead of a separate bf16 add kernel
                del ctx.x_ref._dtf_pending_grad
                if isinstance(pending, _MaskedGrad):
                    dx = conv2d_dgrad(dy, wb, xb.shape, ctx.stride, ctx.padding, bnb=ctx.bnb,
                                      acc_from=pending)
                else:
                    dx = conv2d_dgrad(dy, wb, xb.shape, ctx.stride, ctx.padding, out=pending,
                                      bnb=ctx.bnb)
            else:
                dx = conv2d_dgrad(dy, wb, xb.shape, ctx.stride, ctx.padding,
                                  bnb=ctx.bnb if pending is None and not padded else None)
                if padded:
                    dx = dx[..., :C].contiguous()
                if pending is not None:
                    del ctx.x_ref._dtf_pending_grad
                    if isinstance(pending, _MaskedGrad):
                        pending = pending.materialize()
                    dx = dx + pending
        ctx.x_ref = None
        ctx.bnb = None
        return dx, dw, None, None, None, None


class _Conv2dBiasRelu(torch.autograd.Function):
    """tf.layers.conv2d(..., activation=tf.nn.relu) with the bias add and ReLU in the conv
    kernel's epilogue (reference ``run_mnist_distributed.py:52-64``).  Backward:
    ReluGrad + BiasAddGrad in one fused pass over dy (csrc/kernels/dense.hip), then the
    MFMA weight-gradient (fp32 straight into the flat buffer) and data-gradient kernels."""

    @staticmethod
    def forward(ctx, x, w_master, b_master, stride, padding, relu):
        xb = x.contiguous()
        wb = _bf16_weight(w_master)
        C = xb.shape[-1]
        if C % 8:
            xb, wb = _pad_c8(xb), _pad_c8(wb)
        bias = b_master.detach().float().contiguous() if b_master is not None else None
        y = conv2d_forward(xb, wb, stride, padding, bias=bias, relu=relu)
        ctx.save_for_backward(xb, wb, y if relu else None)
        ctx.meta = (stride, padding, relu, C)
        ctx.params = (w_master, b_master)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wb, y = ctx.saved_tensors
        stride, padding, relu, C = ctx.meta
        w_master, b_master = ctx.params
        ctx.params = None
        dy = dy.contiguous()
        K = dy.shape[-1]
        M = dy.numel() // K
        dx = dw = db = None
        need_b = b_master is not None and ctx.needs_input_grad[2]
        dz = dy
        if relu or need_b:
            dz = torch.empty_like(dy) if relu else dy
            ws = torch.empty(_K.bias_relu_bwd_ws_floats(K), device=dy.device, dtype=torch.float32)
            tb = _direct_grad(b_master) if need_b else None
            dbuf = (tb if tb is not None else torch.empty(K, device=dy.device,
                                                          dtype=torch.float32)) if need_b else None
            _K.bias_relu_bwd(dy.data_ptr(), _p(y) if relu else dy.data_ptr(), dz.data_ptr(), M, K,
                             ws.data_ptr(), _p(dbuf), int(tb is not None), int(relu), _st())
            if need_b:
                if tb is not None:
                    _grad_ready(b_master)
                else:
                    db = dbuf.to(b_master.dtype)
        padded = xb.shape[-1] != C
        if ctx.needs_input_grad[1]:
            target = _direct_grad(w_master)
            if target is not None and not padded:
                conv2d_wgrad(xb, dz, wb.shape, stride, padding, out=target)
                _grad_ready(w_master)
            else:
                g = conv2d_wgrad(xb, dz, wb.shape, stride, padding)[..., :C]
                if target is not None:
                    target.add_(g)
                    _grad_ready(w_master)
                else:
                    dw = g.to(w_master.dtype)
        if ctx.needs_input_grad[0]:
            dx = conv2d_dgrad(dz, wb, xb.shape, stride, padding)
            if padded:
                dx = dx[..., :C].contiguous()
        return dx, dw, db, None, None, None


def conv2d_bias_relu(x, w, bias=None, stride=1, padding=0, relu=True):
    _check_cuda_bf16(x)
    K, R, S, C = w.shape
    if K % 8 or R * S > 64:
        raise ValueError(f"native conv2d: unsupported filter {tuple(w.shape)}")
    return _Conv2dBiasRelu.apply(x, w, bias, stride, padding, bool(relu))


_SHARE_INPUT_GRAD = os.environ.get("DTF_SHARE_INPUT_GRAD", "1") == "1"
# BatchNorm backward sums fused into the consuming conv's dgrad epilogue.  Off by default:
# measured on MI355X (ResNet-50 b512) the epilogue's extra read of the BN input costs the dgrad
# kernels as much time (+3.8 ms/step) as the separate reduce pass it removes (-3.9 ms/step) --
# the 1x1 dgrads are bandwidth-bound, and the streaming reduce runs at ~5.3 TB/s.
_FUSE_BN_BWD = os.environ.get("DTF_FUSE_BN_BWD", "0") == "1"
# ... except where that data gradient runs on the row-streaming GEMM (identity-block c1 convs):
# there the gradient is still in registers, the epilogue reads only x (prefetched one chunk
# ahead, streaming), and the reduce pass's re-read of dy and the mask disappears
_FUSE_BN_BWD_STREAM = os.environ.get("DTF_FUSE_BN_BWD_STREAM", "1") == "1"


# ... and where it runs on the 3x3 halo kernels (stage-1/2 c2 data gradients -> BN1): the x
# rows load under the main loop, and the BN1 reduce pass (a re-read of dy and x) goes (+0.2 %)
_FUSE_BN_BWD_HALO = os.environ.get("DTF_FUSE_BN_BWD_HALO", "1") == "1"
# ... and in the stride-2 3x3 data gradient of s1b0c2 (stage 1's first block; 128 outputs: the register
# implicit-GEMM kernel either way): the 3.2 GB BN1 reduce pass goes, throughput-neutral
# (profiles/measurements/r4_stride2_dgrad_bn_sums_ab.jsonl)
_FUSE_BN_BWD_S2 = os.environ.get("DTF_FUSE_BN_BWD_S2", "1") == "1"
# the phase classes of a strided data gradient in one grouped launch (conv2d_dgrad)
_DGRAD_GROUPED = os.environ.get("DTF_DGRAD_GROUPED", "1") == "1"
# ... also where the data gradient (C >= 256 outputs) would otherwise run on the ping-pong GEMM
# route, which takes no BN-sum epilogue (measured -0.3 % with it)
_FUSE_BN_BWD_S2_ALL = os.environ.get("DTF_FUSE_BN_BWD_S2_ALL", "0") == "1"


def _halo_dgrad_shape(K, C, H, W):
    """The data gradient of a 3x3 stride-1 'same' conv C -> K runs on a halo kernel family
    (csrc/kernels/conv.hip halo_family: 56 x 56 x 64 or 28 x 28 x 128 input to the dgrad)."""
    return H % 4 == 0 and ((K == 64 and W == 56 and C % 64 == 0) or
                           (K == 128 and W == 28 and C % 128 == 0))


def conv2d(x, w, stride=1, padding=0, bn_stats=False, grad_share=None):
    """NHWC conv.  ``bn_stats=True`` (a training-mode BatchNorm consumes the output): the conv
    epilogue also emits the BN partial sums, attached to the output as ``_dtf_bn_part`` and picked
    up by :func:`batch_norm`, which then skips its own statistics pass over the tensor."""
    _check_cuda_bf16(x)
    K, R, S, C = w.shape
    if K % 8 or R * S > 64:
        raise ValueError(f"native conv2d: unsupported filter {tuple(w.shape)}")
    if grad_share is not None and (x.shape[-1] % 8 or not _SHARE_INPUT_GRAD):
        grad_share = None        # channel-padded convs produce their own (sliced) dx
    if not bn_stats:
        return _Conv2d.apply(x, w, stride, padding, None, grad_share)
    n, h, wd, c, P, Q, sh, sw, pt, pl = _conv_geom_fwd(x, K, R, S, stride, padding)
    M = n * P * Q
    taps = [(r - pt, s - pl) for r in range(R) for s in range(S)]
    cp = -(-c // 8) * 8                      # the op zero-pads C to 8 before launching
    if _gemm_1x1(cp, K, R, S, stride, (pt, pl)):
        G = _K.gemm_tile_rows(M)
    else:
        G = _K.conv_tile_rows(_fwd_geom((n, h, wd, cp), K, taps, P, Q, sh, sw, P, Q),
                              [t[0] for t in taps], [t[1] for t in taps])
    part = torch.empty(_K.bn_workspace_floats_g(G, K), device=x.device, dtype=torch.float32)
    y = _Conv2d.apply(x, w, stride, padding, part, grad_share)
    y._dtf_bn_part = (part, G, M, K)
    return y


# ----------------------------------------------------------------------------- batch norm

_FUSE_RESIDUAL_GRAD = os.environ.get("DTF_FUSE_RESIDUAL_GRAD", "1") == "1"
# BN1 + ReLU applied on the c2 halo conv's input load (batch_norm(defer=True)); A/B knob
_BN_ON_LOAD = os.environ.get("DTF_BN_ON_LOAD", "1") == "1"
_LAZY_RESIDUAL_GRAD = os.environ.get("DTF_LAZY_RESIDUAL_GRAD", "1") == "1"
# stem backward: pool gather fused into both BatchNorm backward passes (_BatchNormReluMaxPool)
_FUSE_STEM_POOL_BWD = os.environ.get("DTF_FUSE_STEM_POOL_BWD", "1") == "1"
# ... and its apply pass folded into the stem weight gradient (d(stem conv output) never stored:
# conv_wgrad_stem_dz); a module switch for the A/B tests, no environment knob
_FUSE_STEM_WGRAD = True


def _stem_wgrad_shape(xb, wb, stride, padding):
    """The ResNet stem on its space-to-depth image: a 4 x 4 stride-1 VALID conv, 115 x 115 x 16
    -> 112 x 112 x 64 (the conv_wgrad_stem_kernel geometry)."""
    return (tuple(xb.shape[1:]) == (115, 115, 16) and tuple(wb.shape) == (64, 4, 4, 16)
            and tuple(_pair(stride)) == (1, 1) and padding in (0, "VALID", "valid", (0, 0))
            and xb.is_contiguous())


class _BatchNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, momentum, eps, relu,
                residual, residual_to_conv=False, defer=False):
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dev = x.device
        st = _st()
        stats, g32 = _bn_forward_stats(x, gamma, beta, running_mean, running_var, training,
                                       momentum, eps)
        scale, shift = stats[2], stats[3]
        res = residual.contiguous() if residual is not None else None
        y = torch.empty_like(x)
        # residual + ReLU: the backward's ReLU mask cannot be recomputed from x alone, so the
        # apply also writes it as 1 bit per element (1/16 of the bytes of y, read twice)
        mask = (torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
                if relu and residual is not None else None)
        rc = getattr(x, "_dtf_recompute", None)
        if rc is not None and not (relu and res is not None):
            rc.materialize()
            rc = None
        deferred = None
        if defer and relu and res is None and training and rc is None:
            # the consuming 3x3 conv applies this BN + ReLU on load and writes y (_BnDeferred)
            deferred = _BnDeferred(x, scale, shift, y)
        elif rc is not None:
            # lazy x3: the apply recomputes the conv output in a stream GEMM whose epilogue is
            # this apply (bit-identical to storing x3 and running the pass over it)
            _K.gemm_stream_apply(rc.y.data_ptr(), rc.wb.data_ptr(), y.data_ptr(), M, C, rc.k3,
                                 res.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                 mask.data_ptr(), st)
        else:
            _K.bn_apply(x.data_ptr(), _p(res), y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                        M, C, int(relu), st, _p(mask))
        if deferred is not None:
            y._dtf_bnl = deferred
        ctx.save_for_backward(x, mask, g32, stats)
        ctx.relu = relu
        ctx.has_res = residual is not None
        if training:
            # a conv consuming y computes this BN's backward sums in its dgrad epilogue
            ctx.bnb_token = object()
            y._dtf_bnb = (x, stats, mask, relu, residual is not None, ctx.bnb_token)
        ctx.gdt, ctx.bdt = gamma.dtype, beta.dtype
        ctx.params = (gamma, beta)
        # identity-shortcut blocks: hand d(residual) to the conv that also reads the residual
        # tensor (it accumulates its dgrad onto it) instead of returning it to autograd
        ctx.res_ref = residual if (residual_to_conv and _FUSE_RESIDUAL_GRAD) else None
        # projection shortcuts: this BN (no ReLU, no residual) feeds a residual BN as its
        # residual; that BN leaves d(y) here as (dy, ReLU bit mask) instead of writing it
        ctx.slot = None
        if training and not relu and residual is None and _LAZY_RESIDUAL_GRAD:
            ctx.slot = _GradSlot()
            y._dtf_grad_slot = ctx.slot
            ctx.set_materialize_grads(False)
        ctx.res_slot = (getattr(residual, "_dtf_grad_slot", None)
                        if residual is not None and not residual_to_conv else None)
        # a fused c3 backward that forms d(x) itself from (dy, x, mask, coefficients)
        ctx.in_slot = (getattr(x, "_dtf_lazy_slot", None)
                       if training and relu and residual is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, g32, stats = ctx.saved_tensors
        relu = None
        if dy is None:
            mg = ctx.slot.grad if ctx.slot is not None else None
            if mg is None:
                return (None,) * 12
            ctx.slot.grad = None
            # d(y) = dy_res * mask: the reduce / apply kernels apply the bit mask on load
            dy, mask, relu = mg.dy, mg.mask, True
        ctx.slot = None
        dx, dg, db, dres = _bn_backward_core(ctx, dy, x, mask, g32, stats, relu)
        return dx, dg, db, None, None, None, None, None, None, dres, None, None


def _bn_forward_stats(x, gamma, beta, running_mean, running_var, training, momentum, eps):
    """Per-channel (mean, invstd, scale, shift) as a [4, C] fp32 tensor, from the producing
    conv's fused partial sums when present, else a statistics pass; plus fp32 gamma."""
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    stats = torch.empty(4, C, device=dev, dtype=torch.float32)  # mean, invstd, scale, shift
    mean, invstd, scale, shift = stats[0], stats[1], stats[2], stats[3]
    st = _st()
    g32, b32 = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
    fused = getattr(x, "_dtf_bn_part", None)
    if training and fused is not None and fused[2:] == (M, C):
        # statistics already produced by the producing conv's epilogue
        part, G = fused[0], fused[1]
        _K.bn_fwd_finalize_g(part.data_ptr(), G, M, C, g32.data_ptr(), b32.data_ptr(),
                             _p(running_mean), _p(running_var), float(momentum), float(eps),
                             mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(),
                             shift.data_ptr(), st)
    elif training:
        part = torch.empty(_K.bn_workspace_floats(M, C), device=dev, dtype=torch.float32)
        _K.bn_fwd_stats(x.data_ptr(), M, C, part.data_ptr(), st)
        _K.bn_fwd_finalize(part.data_ptr(), M, C, g32.data_ptr(), b32.data_ptr(),
                           _p(running_mean), _p(running_var), float(momentum), float(eps),
                           mean.data_ptr(), invstd.data_ptr(), scale.data_ptr(),
                           shift.data_ptr(), st)
    else:
        _K.bn_infer_finalize(C, g32.data_ptr(), b32.data_ptr(), running_mean.data_ptr(),
                             running_var.data_ptr(), float(eps), mean.data_ptr(),
                             invstd.data_ptr(), scale.data_ptr(), shift.data_ptr(), st)
    return stats, g32


def _bn_bwd_finalize(ctx, part, G, M, C, g32, stats):
    """Combine the backward partial sums -> dgamma / dbeta (straight into the flat gradient
    buffer when it exposes one) and the dx = A dz + B x + C coefficients; returns (gb, direct)
    with gb = [dgamma, dbeta, A, B, C]."""
    return _bn_bwd_finalize_p(ctx.params, part, G, M, C, g32, stats)


def _bn_bwd_finalize_p(params, part, G, M, C, g32, stats):
    st = _st()
    mean, invstd = stats[0], stats[1]
    gb = torch.empty(5, C, device=g32.device, dtype=torch.float32)
    tg, tb = (_direct_grad(p) for p in params)
    direct = tg is not None and tb is not None
    dg_ptr, db_ptr = ((tg.data_ptr(), tb.data_ptr()) if direct
                      else (gb[0].data_ptr(), gb[1].data_ptr()))
    if G is None:
        _K.bn_bwd_finalize(part.data_ptr(), M, C, g32.data_ptr(), mean.data_ptr(),
                           invstd.data_ptr(), dg_ptr, db_ptr, gb[2].data_ptr(),
                           gb[3].data_ptr(), gb[4].data_ptr(), int(direct), st)
    else:
        _K.bn_bwd_finalize_g(part.data_ptr(), G, M, C, g32.data_ptr(), mean.data_ptr(),
                             invstd.data_ptr(), dg_ptr, db_ptr, gb[2].data_ptr(),
                             gb[3].data_ptr(), gb[4].data_ptr(), int(direct), st)
    if direct:
        for p in params:
            _grad_ready(p)
    return gb, direct


def _bn_backward_core(ctx, dy, x, mask, g32, stats, relu=None):
    """BatchNorm(+ReLU)(+residual) backward shared by :class:`_BatchNorm` and
    :class:`_BatchNormReluMaxPool`; returns (dx, dgamma, dbeta, dresidual) (None where the
    gradient went straight into the flat buffer or to a consuming conv)."""
    dy = dy.contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    st = _st()
    mean, invstd = stats[0], stats[1]
    # ReLU mask: the forward's bit mask when a residual was added before the ReLU, else
    # recomputed from x with the forward's scale/shift (neither pass reads y)
    relu = ctx.relu if relu is None else relu
    mask_x = relu and mask is None
    sc_ptr, sh_ptr = (stats[2].data_ptr(), stats[3].data_ptr()) if mask_x else (0, 0)
    fused = getattr(dy, "_dtf_bnb_part", None)
    tok = getattr(ctx, "bnb_token", None)
    if (fused is not None and tok is not None and fused[4] is tok and fused[2:4] == (M, C)
            and fused[5] == dy._version):
        # sums already produced by the dgrad epilogue of the conv that consumed y
        part, G = fused[0], fused[1]
    else:
        _materialized(x)                   # a lazy c3 output: recomputed for the reduce pass
        part, G = torch.empty(_K.bn_workspace_floats(M, C), device=dev,
                              dtype=torch.float32), None
        _K.bn_bwd_reduce(dy.data_ptr(), 0, x.data_ptr(), mean.data_ptr(),
                         invstd.data_ptr(), M, C, int(relu), part.data_ptr(), st,
                         sc_ptr, sh_ptr, _p(mask))
    gb, direct = _bn_bwd_finalize(ctx, part, G, M, C, g32, stats)
    dx = torch.empty_like(x) if getattr(ctx, "in_slot", None) is None else None
    lazy = (ctx.has_res and ctx.res_ref is not None and _LAZY_RESIDUAL_GRAD
            and mask is not None)
    res_slot = getattr(ctx, "res_slot", None)
    lazy_slot = (ctx.has_res and not lazy and res_slot is not None and _LAZY_RESIDUAL_GRAD
                 and mask is not None)
    dres = torch.empty_like(x) if ctx.has_res and not (lazy or lazy_slot) else None
    in_slot = getattr(ctx, "in_slot", None)
    ctx.in_slot = None
    if in_slot is not None and dres is None and mask is not None and relu:
        # the producing conv's fused backward forms dx per tile from these and never stores it
        in_slot.grad = _LazyBnDx(dy, x, mask, gb)
        dx = None
    else:
        if dx is None:
            dx = torch.empty_like(x)
        _materialized(x)
        _K.bn_bwd_apply(dy.data_ptr(), 0, x.data_ptr(), gb[2].data_ptr(),
                        gb[3].data_ptr(), gb[4].data_ptr(), dx.data_ptr(), _p(dres), M, C,
                        int(relu), st, sc_ptr, sh_ptr, _p(mask))
    if lazy:
        # d(residual) = dy * relu_mask is never written: the consuming dgrad forms it in its
        # epilogue from dy and the bit mask (conv geom acc mode 2)
        ctx.res_ref._dtf_pending_grad = _MaskedGrad(dy, mask)
    elif lazy_slot:
        # projection shortcut: the shortcut BN's backward reads dy and the mask itself
        res_slot.grad = _MaskedGrad(dy, mask)
        ctx.res_slot = None
    elif dres is not None and ctx.res_ref is not None:
        ctx.res_ref._dtf_pending_grad = dres
        dres = None
    ctx.res_ref = None
    if direct:
        return dx, None, None, dres
    return dx, gb[0].to(ctx.gdt), gb[1].to(ctx.bdt), dres


def batch_norm(x, gamma, beta, running_mean=None, running_var=None, training=True,
               momentum=0.997, eps=1e-5, relu=False, residual=None, residual_to_conv=False,
               defer=False):
    """``defer``: BN + ReLU whose only consumer is a 3x3 conv -- the apply pass is left to the
    conv's input load where its kernel supports it (see :class:`_BnDeferred`)."""
    _check_cuda_bf16(x, residual)
    C = x.shape[-1]
    if C % 8 or C > 2048:
        raise ValueError(f"native batch_norm: unsupported channel count {C}")
    if residual is not None and residual.shape != x.shape:
        raise ValueError("residual shape mismatch")
    return _BatchNorm.apply(x, gamma, beta, running_mean, running_var, training, momentum, eps,
                            relu, residual, residual_to_conv, bool(defer and _BN_ON_LOAD))


class _BnReluConv1x1(torch.autograd.Function):
    """conv1x1(relu(BN(x)), w) with the BatchNorm + ReLU applied inside the row-streaming GEMM
    (csrc/kernels/gemm_stream.hip PRE): the GEMM reads x, normalises its A rows in registers with
    the BN apply pass's exact arithmetic and writes them once as y (the weight gradient's
    operand) -- the separate apply pass (read x, write y) and the GEMM's read of y become one read
    of x and one write of y.  Bit-identical to batch_norm(relu) + conv2d.  The output carries its
    own BN statistics (``_dtf_bn_part``) for the BatchNorm that consumes it.  Backward: the conv's
    weight / data gradients from y, then the BN backward (ReLU recomputed from x)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, w_master, momentum, eps,
                lazy_out=False):
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        stats, g32 = _bn_forward_stats(x, gamma, beta, running_mean, running_var, True,
                                       momentum, eps)
        wb = _bf16_weight(w_master)
        K = wb.shape[0]
        y = torch.empty_like(x)
        # lazy x3: the output tensor is allocated but never written -- the residual BN consuming
        # it recomputes bf16(y . w^T) (the same MFMA chain) wherever it needs the values
        lazy = bool(lazy_out) and _lazy_x3_ok(M, C, K)
        out = torch.empty(*x.shape[:-1], K, device=x.device, dtype=_BF16)
        G = _K.gemm_tile_rows(M)
        part = torch.empty(_K.bn_workspace_floats_g(G, K), device=x.device, dtype=torch.float32)
        _K.gemm_stream_pre(x.data_ptr(), wb.data_ptr(), out.data_ptr(), M, K, C,
                           stats[2].data_ptr(), stats[3].data_ptr(), y.data_ptr(),
                           part.data_ptr(), _st(), int(lazy))
        out._dtf_bn_part = (part, G, M, K)
        if lazy:
            out._dtf_recompute = _Recompute(y, wb, out)
        if wb.is_contiguous():
            _register_dgrad_filter(wb)
        ctx.lz_slot = None
        if _FUSE_C1_BWD and _FUSE_C3_LAZY and _K.conv1x1_bwd_lazy_ok(M, C, K):
            # the residual BN consuming `out` may hand its d(out) over unformed (_LazyBnDx)
            ctx.lz_slot = _GradSlot()
            out._dtf_lazy_slot = ctx.lz_slot
            ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, y, wb, g32, stats)
        ctx.w_param, ctx.w_dtype = w_master, w_master.dtype
        # the BatchNorm-backward core's context
        ctx.relu, ctx.has_res, ctx.res_ref, ctx.res_slot = True, False, None, None
        ctx.params = (gamma, beta)
        ctx.gdt, ctx.bdt = gamma.dtype, beta.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y, wb, g32, stats = ctx.saved_tensors
        lz, ctx.lz_slot = ctx.lz_slot, None
        rec = lz.grad if lz is not None else None
        if lz is not None:
            lz.grad = None
        if dout is None and rec is None:
            ctx.w_param = ctx.params = None
            return (None,) * 9
        if dout is not None and rec is not None:
            dout = dout + rec.materialize()      # another consumer of the conv output
            rec = None
        K, _, _, C = wb.shape
        M = y.numel() // C
        dw = None
        target = _direct_grad(ctx.w_param)
        if rec is not None:
            dy, dw = _conv1x1_bwd_fused(ctx, None, x, y, wb, stats, target, M, C, K, lazy=rec)
            dx, dg, db, _ = _bn_backward_core(ctx, dy, x, None, g32, stats)
            ctx.w_param = ctx.params = None
            return dx, dg, db, None, None, dw, None, None, None
        dout = dout.contiguous()
        if _FUSE_C1_BWD and _K.conv1x1_bwd_ok(M, C, K):
            dy, dw = _conv1x1_bwd_fused(ctx, dout, x, y, wb, stats, target, M, C, K)
            dx, dg, db, _ = _bn_backward_core(ctx, dy, x, None, g32, stats)
            ctx.w_param = ctx.params = None
            return dx, dg, db, None, None, dw, None, None, None
        if target is not None:
            conv2d_wgrad(y, dout, wb.shape, 1, 0, out=target)
            _grad_ready(ctx.w_param)
        else:
            dw = conv2d_wgrad(y, dout, wb.shape, 1, 0).to(ctx.w_dtype)
        dy = conv2d_dgrad(dout, wb, y.shape, 1, 0)
        dx, dg, db, _ = _bn_backward_core(ctx, dy, x, None, g32, stats)
        ctx.w_param = ctx.params = None
        return dx, dg, db, None, None, dw, None, None, None


def _conv1x1_bwd_fused(ctx, dout, x, y, wb, stats, target, M, C, K, lazy=None):
    """Stage-0 / stage-1 c3 (64 -> 256, 128 -> 512) backward in ONE pass (csrc/kernels/conv1x1_bwd.hip): the
    data gradient dy, the weight gradient (per-block fp32 slabs, reduced here in fixed order
    into the flat gradient buffer or a fresh tensor) and the consuming BatchNorm's backward
    sums (attached to dy as ``_dtf_bnb_part`` for :func:`_bn_backward_core`).  Replaces the
    wgrad pass, the dgrad GEMM and the BN reduce pass (1536 -> 896 B of HBM traffic per row)."""
    dev = y.device
    st = _st()
    G = _K.conv1x1_bwd_lazy_blocks(M, C) if lazy is not None else _K.conv1x1_bwd_blocks(M, C)
    wpart = torch.empty(G * K * C, device=dev, dtype=torch.float32)
    part = torch.empty(_K.bn_workspace_floats_g(G, C), device=dev, dtype=torch.float32)
    dy = torch.empty_like(y)
    wt = _dgrad_filter(wb.reshape(K, 1, C)).view(C, K)
    common = (wt.data_ptr(), y.data_ptr(), x.data_ptr(), stats[0].data_ptr(),
              stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(), dy.data_ptr(),
              wpart.data_ptr(), part.data_ptr(), M, C, K)
    if lazy is not None:
        # d(conv output) formed per tile from the residual BN's (dy, x, mask, coefficients); at
        # stage 0 x (this conv's output) is recomputed from y and w instead of read
        _K.conv1x1_bwd_lazy(lazy.dy.data_ptr(), lazy.x.data_ptr(), lazy.mask.data_ptr(),
                            lazy.gb[2].data_ptr(), lazy.gb[3].data_ptr(), lazy.gb[4].data_ptr(),
                            *common, wb.data_ptr(), st)
    else:
        _K.conv1x1_bwd(dout.data_ptr(), *common, st)
    dw = None
    if target is not None:
        _K.slab_reduce(wpart.data_ptr(), target.data_ptr(), K * C, G, 1, st)
        _grad_ready(ctx.w_param)
    else:
        out = torch.empty(K, 1, 1, C, device=dev, dtype=torch.float32)
        _K.slab_reduce(wpart.data_ptr(), out.data_ptr(), K * C, G, 0, st)
        dw = out.to(ctx.w_dtype)
    ctx.bnb_token = tok = object()
    dy._dtf_bnb_part = (part, G, M, C, tok, dy._version)
    return dy, dw


# stage-0 / stage-1 c3 backward as one fused pass (A/B knob; summation order of dW and the BN sums
# differs from the separate passes)
_FUSE_C1_BWD = os.environ.get("DTF_FUSE_C1_BWD", "1") == "1"
# ... at stage 0 also without the residual BN's apply pass writing d(conv output) (_LazyBnDx)
_FUSE_C3_LAZY = os.environ.get("DTF_FUSE_C3_LAZY", "1") == "1"


def bn_relu_conv1x1_ok(x, w):
    """The fused BN + ReLU + 1x1 conv applies: the conv is stream-routed (reduction C in
    {64, 128, 256}, output K >= C, K % 64 == 0) on a bf16 CUDA tensor."""
    if not (_FUSE_BN_CONV and _GEMM_STREAM and x.is_cuda and x.dtype == _BF16 and w.dim() == 4):
        return False
    K, R, S, C = w.shape
    return (R == 1 and S == 1 and x.shape[-1] == C and C in (64, 128, 256) and K >= C
            and K % 64 == 0)


def bn_relu_conv1x1(x, gamma, beta, running_mean, running_var, w, momentum=0.997, eps=1e-5,
                    lazy_out=False):
    _check_cuda_bf16(x)
    return _BnReluConv1x1.apply(x, gamma, beta, running_mean, running_var, w, momentum, eps,
                                bool(lazy_out))


def _lazy_x3_ok(M, C, K):
    """Lazy x3 for this c3 (reduction C, output K): every reader can recompute it -- the stream
    apply (C in {64, 128}), the consumers' RC BN-sum epilogue (K3 = C <= 128) and the fused c3
    backward, which recomputes x3 only at stage 0 (C = 64; stage 1 reads it)."""
    return _LAZY_X3 and C == 64 and K % 64 == 0 and K <= 2048 and \
        _K.conv1x1_bwd_lazy_ok(M, C, K) and _FUSE_C1_BWD and _FUSE_C3_LAZY


# never store the stage-0 identity blocks' c3 output (A/B knob)
_LAZY_X3 = os.environ.get("DTF_LAZY_X3", "1") == "1"


def _materialized(x):
    """``x`` with its values: a lazy c3 output is recomputed into its own storage first."""
    rc = getattr(x, "_dtf_recompute", None)
    if rc is not None:
        rc.materialize()
    return x


# BN + ReLU of a bottleneck's c2 output applied inside c3's streaming GEMM (A/B knob)
_FUSE_BN_CONV = os.environ.get("DTF_FUSE_BN_CONV", "1") == "1"


class _BatchNormAddBatchNorm(torch.autograd.Function):
    """relu(BN(x) + BN_p(xp)): a projection block's residual BatchNorm and its shortcut's
    BatchNorm as ONE op.  Forward: one apply pass normalises both conv outputs (the shortcut
    BN's output is never stored or re-read; it is rounded to bf16 in registers exactly as its own
    pass would have stored it, so the result is bit-identical to the two-op form).  Backward:
    both BNs see the same dz = dy * relu_mask, so one reduce pass reads dy and the bit mask once
    for both BNs' sums and one apply pass writes dx and dxp (csrc/kernels/batchnorm.hip DUAL
    variants).  Saves ~8 B of HBM traffic per shortcut element per step."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, xp, gamma_p, beta_p,
                running_mean_p, running_var_p, training, momentum, eps):
        x, xp = x.contiguous(), xp.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        stats, g32 = _bn_forward_stats(x, gamma, beta, running_mean, running_var, training,
                                       momentum, eps)
        stats_p, g32_p = _bn_forward_stats(xp, gamma_p, beta_p, running_mean_p, running_var_p,
                                           training, momentum, eps)
        y = torch.empty_like(x)
        mask = torch.empty(M * C // 8, device=x.device, dtype=torch.uint8)
        _K.bn_apply_dual(x.data_ptr(), xp.data_ptr(), y.data_ptr(), mask.data_ptr(),
                         stats[2].data_ptr(), stats[3].data_ptr(), stats_p[2].data_ptr(),
                         stats_p[3].data_ptr(), M, C, 1, _st())
        ctx.save_for_backward(x, xp, mask, g32, g32_p, stats, stats_p)
        ctx.params = (gamma, beta)
        ctx.params_p = (gamma_p, beta_p)
        ctx.dtypes = (gamma.dtype, beta.dtype, gamma_p.dtype, beta_p.dtype)
        # the projection block's c3 (a fused BN + ReLU + 1x1 conv) may form d(x) itself
        ctx.in_slot = getattr(x, "_dtf_lazy_slot", None) if training else None
        ctx.bnb_token = None
        if training and _FUSE_DUAL_BNB:
            # a streamed 1x1 data gradient of y (the next block's c1) emits both BNs' sums
            ctx.bnb_token = object()
            y._dtf_bnb_dual = (x, stats, mask, xp, stats_p, ctx.bnb_token)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xp, mask, g32, g32_p, stats, stats_p = ctx.saved_tensors
        dy = dy.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        st = _st()
        fused = getattr(dy, "_dtf_bnb_part", None)
        tok = ctx.bnb_token
        if (fused is not None and tok is not None and fused[4] is tok and fused[2:4] == (M, C)
                and fused[5] == dy._version and getattr(dy, "_dtf_bnb_part_p", None) is not None):
            # both BNs' sums came from the streamed data gradient that produced dy
            part, G = fused[0], fused[1]
            part_p = dy._dtf_bnb_part_p
        else:
            ws = _K.bn_workspace_floats(M, C)
            part = torch.empty(ws, device=x.device, dtype=torch.float32)
            part_p = torch.empty(ws, device=x.device, dtype=torch.float32)
            G = None
            _K.bn_bwd_reduce_dual(dy.data_ptr(), mask.data_ptr(), x.data_ptr(),
                                  stats[0].data_ptr(), stats[1].data_ptr(), xp.data_ptr(),
                                  stats_p[0].data_ptr(), stats_p[1].data_ptr(), M, C,
                                  part.data_ptr(), part_p.data_ptr(), st)
        gb, direct = _bn_bwd_finalize_p(ctx.params, part, G, M, C, g32, stats)
        gbp, direct_p = _bn_bwd_finalize_p(ctx.params_p, part_p, G, M, C, g32_p, stats_p)
        in_slot, ctx.in_slot = ctx.in_slot, None
        dx = None if in_slot is not None else torch.empty_like(x)
        dxp = torch.empty_like(xp)
        _K.bn_bwd_apply_dual(dy.data_ptr(), mask.data_ptr(), x.data_ptr(), gb[2].data_ptr(),
                             gb[3].data_ptr(), gb[4].data_ptr(), _p(dx), xp.data_ptr(),
                             gbp[2].data_ptr(), gbp[3].data_ptr(), gbp[4].data_ptr(),
                             dxp.data_ptr(), M, C, st)
        if in_slot is not None:
            in_slot.grad = _LazyBnDx(dy, x, mask, gb)
        gd, bd, gpd, bpd = ctx.dtypes
        ctx.params = ctx.params_p = None
        dg, db = (None, None) if direct else (gb[0].to(gd), gb[1].to(bd))
        dgp, dbp = (None, None) if direct_p else (gbp[0].to(gpd), gbp[1].to(bpd))
        return dx, dg, db, None, None, dxp, dgp, dbp, None, None, None, None, None


# the streamed c1 data gradient of the next block emits a projection block's dual BN sums
_FUSE_DUAL_BNB = os.environ.get("DTF_FUSE_DUAL_BNB", "1") == "1"


def batch_norm_add_batch_norm(x, gamma, beta, running_mean, running_var, xp, gamma_p, beta_p,
                              running_mean_p, running_var_p, training=True, momentum=0.997,
                              eps=1e-5):
    """relu(batch_norm(x) + batch_norm(xp)) (training or inference statistics)."""
    _check_cuda_bf16(x, xp)
    C = x.shape[-1]
    if C % 8 or C > 2048:
        raise ValueError(f"native batch_norm: unsupported channel count {C}")
    if xp.shape != x.shape:
        raise ValueError("batch_norm_add_batch_norm: shortcut shape mismatch")
    return _BatchNormAddBatchNorm.apply(x, gamma, beta, running_mean, running_var, xp, gamma_p,
                                        beta_p, running_mean_p, running_var_p, training,
                                        momentum, eps)


class _BatchNormReluMaxPool(torch.autograd.Function):
    """maxpool(relu(BN(x))) without storing the BN output (the ResNet stem: 112x112x64 per
    image): one kernel computes the window maxima of the rounded BN+ReLU values and the argmax;
    the backward is the pool's gather into d(BN output), then the usual BN backward (its ReLU
    mask recomputed from x)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, momentum, eps, kernel,
                stride, padding):
        x = x.contiguous()
        n, h, w, c = x.shape
        stats, g32 = _bn_forward_stats(x, gamma, beta, running_mean, running_var, training,
                                       momentum, eps)
        kh, kw = _pair(kernel)
        sh, sw = _pair(stride)
        pt, pb, pl, pr = resolve_padding(padding, h, w, kh, kw, stride)
        P = (h + pt + pb - kh) // sh + 1
        Q = (w + pl + pr - kw) // sw + 1
        y = torch.empty(n, P, Q, c, device=x.device, dtype=x.dtype)
        arg = torch.empty(n, P, Q, c, device=x.device, dtype=torch.uint8)
        _K.bn_relu_maxpool_fwd(x.data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                               y.data_ptr(), arg.data_ptr(), n, h, w, c, P, Q, kh, kw, sh, sw,
                               pt, pl, _st())
        ctx.save_for_backward(x, g32, stats, arg)
        ctx.geom = (n, h, w, c, P, Q, kh, kw, sh, sw, pt, pl)
        ctx.stem_slot = getattr(x, "_dtf_stem_slot", None) if training else None
        ctx.relu, ctx.has_res, ctx.res_ref = True, False, None
        ctx.gdt, ctx.bdt = gamma.dtype, beta.dtype
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dp):
        x, g32, stats, arg = ctx.saved_tensors
        n, h, w, c, P, Q, kh, kw, sh, sw, pt, pl = ctx.geom
        if (_FUSE_STEM_POOL_BWD and (kh, kw, sh, sw, pt, pl) == (3, 3, 2, 2, 1, 1)
                and 256 % (c // 8) == 0):
            # the pool gather feeds both BN backward passes; d(BN output) is never stored
            dp = dp.contiguous()
            M, st = n * h * w, _st()
            G = _K.pool_bn_bwd_blocks(n, h, w, c)
            part = torch.empty(_K.bn_workspace_floats_g(G, c), device=x.device,
                               dtype=torch.float32)
            _K.pool_bn_bwd_reduce(dp.data_ptr(), arg.data_ptr(), x.data_ptr(),
                                  stats[0].data_ptr(), stats[1].data_ptr(), stats[2].data_ptr(),
                                  stats[3].data_ptr(), part.data_ptr(), n, h, w, c, P, Q, st)
            gb, direct = _bn_bwd_finalize(ctx, part, G, M, c, g32, stats)
            slot, ctx.stem_slot = ctx.stem_slot, None
            if slot is not None and (h, w, c, P, Q) == (112, 112, 64, 56, 56):
                # the stem conv's weight gradient forms d(x) on load; it is never stored
                slot.grad = _LazyStemDz(dp, arg, x, gb, stats[2], stats[3], (n, h, w, c, P, Q))
                dx = None
            else:
                dx = torch.empty_like(x)
                _K.pool_bn_bwd_apply(dp.data_ptr(), arg.data_ptr(), x.data_ptr(),
                                     gb[2].data_ptr(), gb[3].data_ptr(), gb[4].data_ptr(),
                                     stats[2].data_ptr(), stats[3].data_ptr(), dx.data_ptr(), n,
                                     h, w, c, P, Q, st)
            dg, db = (None, None) if direct else (gb[0].to(ctx.gdt), gb[1].to(ctx.bdt))
            return dx, dg, db, None, None, None, None, None, None, None, None
        dy = torch.empty(n, h, w, c, device=dp.device, dtype=dp.dtype)
        _K.maxpool_bwd(dp.contiguous().data_ptr(), arg.data_ptr(), dy.data_ptr(), n, h, w, c, P,
                       Q, kh, kw, sh, sw, pt, pl, _st())
        dx, dg, db, _ = _bn_backward_core(ctx, dy, x, None, g32, stats)
        return dx, dg, db, None, None, None, None, None, None, None, None


def batch_norm_relu_max_pool(x, gamma, beta, running_mean=None, running_var=None, training=True,
                             momentum=0.997, eps=1e-5, kernel=3, stride=2, padding=1):
    _check_cuda_bf16(x)
    C = x.shape[-1]
    if C % 8 or C > 2048:
        raise ValueError(f"native batch_norm: unsupported channel count {C}")
    return _BatchNormReluMaxPool.apply(x, gamma, beta, running_mean, running_var, training,
                                       momentum, eps, kernel, stride, padding)


# ----------------------------------------------------------------------------- ReLU (standalone)

def relu(x):
    return torch.relu(x)   # folded into conv/BN epilogues on the hot path


# ----------------------------------------------------------------------------- pooling

class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, stride, padding):
        x = x.contiguous()
        n, h, w, c = x.shape
        kh, kw = _pair(kernel)
        sh, sw = _pair(stride)
        pt, pb, pl, pr = resolve_padding(padding, h, w, kh, kw, stride)
        P = (h + pt + pb - kh) // sh + 1
        Q = (w + pl + pr - kw) // sw + 1
        y = torch.empty(n, P, Q, c, device=x.device, dtype=x.dtype)
        arg = torch.empty(n, P, Q, c, device=x.device, dtype=torch.uint8)
        _K.maxpool_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), n, h, w, c, P, Q, kh, kw, sh,
                       sw, pt, pl, _st())
        ctx.save_for_backward(arg)
        ctx.geom = (n, h, w, c, P, Q, kh, kw, sh, sw, pt, pl)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        n, h, w, c, P, Q, kh, kw, sh, sw, pt, pl = ctx.geom
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=dy.dtype)
        _K.maxpool_bwd(dy.contiguous().data_ptr(), arg.data_ptr(), dx.data_ptr(), n, h, w, c, P,
                       Q, kh, kw, sh, sw, pt, pl, _st())
        return dx, None, None, None


def max_pool2d(x, kernel=2, stride=2, padding=0):
    _check_cuda_bf16(x)
    if x.shape[-1] % 8:
        raise ValueError("native max_pool2d needs C % 8 == 0")
    kh, kw = _pair(kernel)
    if kh * kw > 255:
        raise ValueError("pool window too large")
    return _MaxPool.apply(x, kernel, stride, padding)


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        n, h, w, c = x.shape
        y = torch.empty(n, c, device=x.device, dtype=x.dtype)
        _K.gap_fwd(x.data_ptr(), y.data_ptr(), n, h * w, c, _st())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shape
        dx = torch.empty(ctx.shape, device=dy.device, dtype=dy.dtype)
        _K.gap_bwd(dy.contiguous().data_ptr(), dx.data_ptr(), n, h * w, c, _st())
        return dx


def global_avg_pool(x):
    _check_cuda_bf16(x)
    if x.shape[-1] % 8:
        raise ValueError("native global_avg_pool needs C % 8 == 0")
    return _GAP.apply(x)


# ----------------------------------------------------------------------------- dense (library GEMM)

def _wgrad_splits(T, o, i):
    """Token-axis split count for the dW = dY^T X GEMM: hipBLASLt tiles only the small o x i
    output (36-144 tiles of 128 x 128 at BERT-base shapes) and leaves most CUs idle, so the
    reduction is split into S batched slices and their fp32 partials summed.  Measured on MI355X
    (a round-1 probe, since removed; T = 16384): 1.6-2.1x over the single GEMM."""
    tiles = -(-o // 128) * -(-i // 128)
    best = 1
    for s in (2, 4, 8):
        if T % s == 0 and T // s >= 1024 and tiles * s <= 1024:
            best = s
    return best


def gemm_nt(a, b, out=None, bias=None, cin=None, relu=False, stats=None, acc_from=None):
    """C[M, N] = A[M, K] . B[N, K]^T (+ bias) (ReLU) (+ cin) on the hand-written MFMA GEMM
    (csrc/kernels/gemm.hip).  A, B bf16 with unit-stride rows; K and N multiples of 8.
    ``stats``: fp32 [tiles_m, 2, N] BatchNorm partial sums of the bf16 output (tiles_m =
    ``gemm_tile_rows(M)``).  ``acc_from``: a :class:`_MaskedGrad` added as dy * mask."""
    _check_cuda_bf16(a, b)
    a2 = a.reshape(-1, a.shape[-1])
    if a2.stride(-1) != 1 or b.stride(-1) != 1:
        raise ValueError("gemm_nt: operands need unit-stride rows")
    M, K = a2.shape
    N = b.shape[0]
    if b.shape[1] != K:
        raise ValueError(f"gemm_nt: K mismatch {tuple(a.shape)} x {tuple(b.shape)}")
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=_BF16)
    if cin is not None and (cin.shape != out.shape or cin.dtype != _BF16 or not cin.is_contiguous()):
        raise ValueError("gemm_nt: cin must be a contiguous bf16 [M, N] tensor")
    if bias is not None:
        bias = bias.detach().float().contiguous()
    src = mask = 0
    if acc_from is not None:
        if acc_from.dy.numel() != out.numel() or acc_from.dy.dtype != _BF16:
            raise ValueError("gemm_nt: masked residual gradient does not match the output")
        src, mask = acc_from.dy.data_ptr(), acc_from.mask.data_ptr()
    _K.gemm_nt(a2.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a2.stride(0), b.stride(0),
               out.stride(0), _p(bias), _p(cin), int(relu), _st(), _p(stats), src, mask)
    return out


_CONV_GEMM = os.environ.get("DTF_CONV_GEMM", "1") == "1"


def _gemm_1x1(C, K, R, S, stride, pads):
    """1x1 stride-1 unpadded convs with a deep reduction or a wide output run on the GEMM
    kernel (NHWC makes them exactly [N*H*W, C] x [K, C]^T).  With the fused BN statistics the
    GEMM is 1.13-1.40x the implicit-GEMM conv kernel where the reduction C >= 512 and the
    output K >= 256, and within noise or slower below: shallow reductions leave the one-block-
    per-CU GEMM's prologue / epilogue exposed, where the conv kernel runs 3-4 blocks per CU
    (profiles/measurements/r2_gemm_vs_conv_resnet1x1_b1280.jsonl, same-box bench A/B)."""
    if not (_CONV_GEMM and R == 1 and S == 1 and tuple(_pair(stride)) == (1, 1)
            and not any(pads) and C % 64 == 0 and K % 8 == 0):
        return False
    # short reduction, output at least as wide (C in {64, 128, 256}, K >= C): the GEMM dispatch
    # takes the row-streaming kernel (csrc/kernels/gemm_stream.hip), whose stores drain under
    # the next chunk's MFMAs: 1.19-1.34x the conv kernel with the BN statistics epilogue at
    # b1984 (profiles/measurements/r3_gemm_stream_resnet1x1_b1984.jsonl)
    if _GEMM_STREAM and C in (64, 128, 256) and K >= C and K % 64 == 0:
        return True
    return C >= _GEMM_1X1_MIN_C and K >= 256


# reduction depth from which a 1x1 conv runs on the GEMM kernel (A/B knob)
_GEMM_1X1_MIN_C = int(os.environ.get("DTF_GEMM_1X1_MIN_C", "512"))
# output-heavy 1x1 convs on the row-streaming GEMM (A/B knob; the C++ dispatch has its own
# switch, gemm_set_stream, for direct gemm_nt calls)
_GEMM_STREAM = os.environ.get("DTF_GEMM_STREAM", "1") == "1"


def _dense_weight_grad(w_param, x2, dy2):
    """dW = dY^T X (fp32) of a library-GEMM dense layer: added straight into the flat gradient
    buffer when the variable exposes one (returns None then), else returned."""
    T, i = x2.shape
    o = dy2.shape[1]
    dw = None
    target = _direct_grad(w_param)
    S = _wgrad_splits(T, o, i) if (o * i) % 4 == 0 and dy2.dtype == x2.dtype else 1
    if dy2.dtype == _BF16 and x2.dtype == _BF16 and o % 8 == 0 and i % 8 == 0:
        # the TN conv weight-gradient kernel, fp32 (straight into the flat buffer when there is
        # one): 1.05-1.40x the split-K library path up to 2304 x 768 (BERT qkv / attention output
        # / MLM transform), 0.97-1.00x on the FFN shapes
        # (profiles/measurements/r3_bert_dense_wgrad_native_vs_library.jsonl); since the decode-
        # free dense form (round 5) every BERT-base layer, the padded tied decoder included
        xw, dw4 = x2.contiguous().view(T, 1, 1, i), dy2.contiguous().view(T, 1, 1, o)
        if target is not None:
            conv2d_wgrad(xw, dw4, (o, 1, 1, i), 1, 0, out=target.view(o, 1, 1, i))
        else:
            dw = conv2d_wgrad(xw, dw4, (o, 1, 1, i), 1, 0).view(o, i)
    elif S == 1:
        if target is not None:
            torch.addmm(target, dy2.t(), x2, out_dtype=torch.float32, out=target)
        else:
            dw = torch.mm(dy2.t(), x2, out_dtype=torch.float32)
    else:
        part = torch.bmm(dy2.view(S, T // S, o).transpose(1, 2), x2.view(S, T // S, i),
                         out_dtype=torch.float32)
        out = target if target is not None else torch.empty(o, i, device=x2.device,
                                                            dtype=torch.float32)
        # deterministic in-order slab sum, fused with the += into the flat grad buffer
        _K.slab_reduce(part.data_ptr(), out.data_ptr(), o * i, S, int(target is not None), _st())
        if target is None:
            dw = out
    if target is not None:
        _grad_ready(w_param)
    elif w_param.dtype != torch.float32:
        dw = dw.to(w_param.dtype)
    return dw


# BERT's plain dense GEMMs (forward y = x W^T + b and the data gradient dx = dy W, beta = 1 onto a
# pending residual gradient) on our persistent MFMA GEMM (gemm.hip gemm_pp2, variant 15) instead of
# hipBLASLt: "native" (default since its interleaved full-line epilogue: 0.92-1.05x the library
# per GEMM, the BERT step within 0.3 %, profiles/measurements/r5_bert_dense_native_vs_library.jsonl)
# / "library" (A/B knob; see _dense_gemm_native)
_DENSE_GEMM = os.environ.get("DTF_DENSE_GEMM", "native")


def _dense_gemm_native(M, N, K):
    """Our GEMM takes this dense layer's forward / data gradient: DTF_DENSE_GEMM=native and the
    shape is the persistent kernel's (N % 8, K % 64, K >= 128, 32-bit operand offsets)."""
    return (_DENSE_GEMM == "native" and N % 8 == 0 and N > 128 and K % 64 == 0 and K >= 128
            and _K.gemm_pp2_ok(M, N, K, K, K))


class _Dense(torch.autograd.Function):
    """y = x @ W^T (+ b) with the bf16 weight shadow -- by default (DTF_DENSE_GEMM=native) on our
    persistent MFMA GEMM (hipBLASLt under DTF_DENSE_GEMM=library and for shapes it does not
    take) with the bias in its epilogue (forward) and the pending residual
    gradient accumulated with beta = 1 (data gradient); backward produces dW and db in fp32
    straight into the optimizer's flat gradient buffer (no bf16 dW, no cast/add kernels)."""

    @staticmethod
    def forward(ctx, x, w_master, wb, b, gelu_b=None):
        ctx.save_for_backward(x, wb)
        ctx.w_param, ctx.b_param = w_master, b
        ctx.x_ref = x     # a fused LayerNorm may leave d(x) here (residual_to_dense)
        ctx.has_b = b is not None
        if gelu_b is not None:
            # (z, h) = (x W^T + gelu_b, gelu(z)) from ONE pass of our MFMA GEMM with the bias +
            # GELU epilogue (gemm.hip gelu_out).  gelu_b is not a differentiable input here: its
            # gradient is the column sum of dz, which the consumer (_BiasGeluDense) forms.
            o, i = wb.shape
            x2 = x.reshape(-1, i)
            M = x2.shape[0]
            if x.requires_grad and wb.is_contiguous():
                # W^T for the data gradient from the step's batched filter transpose (it was a
                # separate 17 us permute copy per layer)
                _register_dgrad_filter(wb.view(o, 1, 1, i))
            z = torch.empty(M, o, device=x.device, dtype=_BF16)
            h = torch.empty_like(z)
            _K.gemm_nt_bias_gelu(x2.data_ptr(), wb.data_ptr(), z.data_ptr(), h.data_ptr(), M, o,
                                 i, x2.stride(0), wb.stride(0), gelu_b.data_ptr(), _st())
            ctx.mark_non_differentiable(h)
            # no zero-filled [T, 3072] gradient for h (0.7 ms/step of fills at BERT-base b512)
            ctx.set_materialize_grads(False)
            shape = (*x.shape[:-1], o)
            return z.view(shape), h.view(shape)
        o, i = wb.shape
        if x.is_contiguous() and wb.is_contiguous() and _dense_gemm_native(x.numel() // i, o, i):
            if x.requires_grad:
                _register_dgrad_filter(wb.view(o, 1, 1, i))    # batched W^T for the backward
            y = gemm_nt(x.view(-1, i), wb, bias=None if b is None else b.detach())
            return y.view(*x.shape[:-1], o)
        return torch.nn.functional.linear(x, wb, None if b is None else b.to(x.dtype))

    @staticmethod
    def backward(ctx, dy, *_unused):
        if dy is None:      # the GELU form's pre-activation received no gradient
            ctx.w_param = ctx.b_param = ctx.x_ref = None
            return None, None, None, None, None
        x, wb = ctx.saved_tensors
        o, i = wb.shape
        x2, dy2 = x.reshape(-1, i), dy.reshape(-1, o)
        T = x2.shape[0]
        dx = dw = db = None
        pending = getattr(ctx.x_ref, "_dtf_pending_grad", None)
        if pending is not None:
            del ctx.x_ref._dtf_pending_grad
        ctx.x_ref = None
        if ctx.needs_input_grad[0]:
            native = (dy2.dtype == _BF16 and _dense_gemm_native(T, i, o))
            if native:
                dyc = dy2 if dy2.is_contiguous() else dy2.contiguous()
                wt = _transposed_bf16(wb)                              # [i, o]
            if pending is not None and pending.dtype == dy2.dtype and pending.is_contiguous():
                # d(x) = d(residual) + dy @ W as one GEMM with beta = 1 on the residual gradient
                if native:
                    pv = pending.view(-1, i)
                    dx = gemm_nt(dyc, wt, out=pv, cin=pv).view(x.shape)
                else:
                    dx = pending.view(-1, i).addmm_(dy2, wb).view(x.shape)
            else:
                dx = (gemm_nt(dyc, wt) if native else dy2 @ wb).reshape(x.shape)
                if pending is not None:
                    dx = dx + pending.view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = _dense_weight_grad(ctx.w_param, x2, dy2)
        if ctx.has_b and ctx.needs_input_grad[3]:
            tb = _direct_grad(ctx.b_param)
            out = tb if tb is not None else torch.empty(o, device=x.device, dtype=torch.float32)
            cp = getattr(dy, "_dtf_colsum_part", None)
            if cp is not None and cp[2] == dy._version and cp[0].shape[1] == o and o % 4 == 0:
                # column partials left by the producer of dy (the fused attention backward):
                # B rows summed in fixed order instead of another pass over dy
                _K.slab_reduce(cp[0].data_ptr(), out.data_ptr(), o, cp[1],
                               int(tb is not None), _st())
            elif dy2.dtype == _BF16 and o % 2 == 0:
                # the fixed-order two-level column sum (16-B loads; 4-B loads for the 30522-wide
                # MLM decoder bias, which torch's reduction ran at ~1.8 TB/s)
                dyc = dy2.contiguous()
                ws = torch.empty(_K.bf16_col_sum_ws_floats(o), device=x.device,
                                 dtype=torch.float32)
                _K.bf16_col_sum(dyc.data_ptr(), T, o, ws.data_ptr(), out.data_ptr(),
                                int(tb is not None), _st())
            elif tb is not None:
                out.add_(torch.sum(dy2, 0, dtype=torch.float32))
            else:
                out = torch.sum(dy2, 0, dtype=torch.float32)
            if tb is not None:
                _grad_ready(ctx.b_param)
            else:
                db = out.to(ctx.b_param.dtype)
        ctx.w_param = ctx.b_param = None
        return dx, dw, None, db, None


class _BiasGeluDense(torch.autograd.Function):
    """o = gelu(a + b1) @ W2^T -- BERT's FFN after its first GEMM (``a`` = x @ W1^T): the
    bias + GELU runs in our fused kernel and the second GEMM on hipBLASLt as before; in backward
    the data gradient d(a) = (do @ W2) * gelu'(a + b1) is ONE pass of our MFMA GEMM with the
    GELU derivative and the b1 column sums in its epilogue (csrc/kernels/gemm.hip gelu_a), so the
    d(gelu output) tensor [T, 3072] is never written or re-read (replaces hipBLASLt's data
    gradient + the bias_gelu backward pass).  The hidden activation is internal to the op, so no
    other consumer can add to its gradient."""

    @staticmethod
    def forward(ctx, a, b1, w_master, wb, h=None):
        N = a.shape[-1]
        a2 = a.reshape(-1, N).contiguous()
        if h is None:
            b32 = b1.detach().float().contiguous()
            h = torch.empty_like(a2)
            _K.bias_gelu_fwd(a2.data_ptr(), b32.data_ptr(), h.data_ptr(), a2.shape[0], N, _st())
        else:
            # the producer GEMM already applied bias + GELU (dense_gelu_dense): a is the
            # pre-activation a + b1 itself, so the backward's GELU derivative takes no bias
            b32 = None
            h = h.reshape(-1, N)
        o, i = wb.shape
        if wb.is_contiguous():
            _register_dgrad_filter(wb.view(o, 1, 1, i))
        ctx.has_b32 = b32 is not None
        ctx.save_for_backward(a2, b32 if b32 is not None else a2, h, wb)
        ctx.params = (b1, w_master)
        ctx.shape = a.shape
        if h.is_contiguous() and wb.is_contiguous() and _dense_gemm_native(h.shape[0], o, i):
            return gemm_nt(h, wb).view(*a.shape[:-1], o)
        return torch.nn.functional.linear(h, wb).view(*a.shape[:-1], o)

    @staticmethod
    def backward(ctx, do):
        a2, b32, h, wb = ctx.saved_tensors
        b32 = b32 if ctx.has_b32 else None
        b1, w_master = ctx.params
        ctx.params = None
        o, i = wb.shape
        M = a2.shape[0]
        do2 = do.reshape(M, o)
        do2 = do2.contiguous() if do2.dtype == _BF16 else do2.to(_BF16).contiguous()
        dw = da = db = None
        if ctx.needs_input_grad[2]:
            dw = _dense_weight_grad(w_master, h, do2)
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            wt = _transposed_bf16(wb)                                  # [i, o]
            da = torch.empty(M, i, device=do.device, dtype=_BF16)
            tiles = _K.gemm_tile_rows(M)
            colsum = torch.empty(tiles, i, device=do.device, dtype=torch.float32)
            _K.gemm_nt_gelu_bwd(do2.data_ptr(), wt.data_ptr(), da.data_ptr(), M, i, o,
                                do2.stride(0), wt.stride(0), a2.data_ptr(), _p(b32),
                                colsum.data_ptr(), _st())
            if ctx.needs_input_grad[1]:
                # the b1 gradient: the per-tile column sums' second level, in fixed order, added
                # straight into the flat gradient buffer (was a torch reduction + add: ~21 us)
                tb = _direct_grad(b1)
                out = tb if tb is not None else torch.empty(i, device=do.device,
                                                            dtype=torch.float32)
                _K.slab_reduce(colsum.data_ptr(), out.data_ptr(), i, tiles,
                               int(tb is not None), _st())
                if tb is not None:
                    _grad_ready(b1)
                else:
                    db = out.to(b1.dtype)
            da = da.view(ctx.shape)
        return da, db, dw, None, None


def bias_gelu_dense(a, b1, w):
    """gelu(a + b1) @ w^T with w [out, in] (fp32 master, bf16 shadow on the GEMM)."""
    _check_cuda_bf16(a)
    return _BiasGeluDense.apply(a, b1, w, _bf16_weight(w))


# BERT's FFN first GEMM on our MFMA GEMM with the bias + GELU epilogue (A/B knob, off by default:
# in the BERT-base b512 step it takes 441 us per layer against 268 us for hipBLASLt + 139 us for the
# bias_gelu_fwd pass, profiles/measurements/r4_bert_ffn1_fused_epilogue.jsonl)
# (on with DTF_DENSE_GEMM=native: the persistent kernel's interleaved epilogue writes z and h)
_FFN_GEMM_GELU = os.environ.get("DTF_FFN_GEMM_GELU",
                                "1" if _DENSE_GEMM == "native" else "0") == "1"


def dense_gelu_dense(x, w1, b1, w2):
    """gelu(x @ w1^T + b1) @ w2^T -- BERT's whole FFN (w [out, in], fp32 masters, bf16 shadows).
    The first GEMM runs on our MFMA GEMM with the bias + GELU in its epilogue, writing the
    pre-activation (for the GELU backward) and the activation (for the second GEMM) in one pass
    instead of a library GEMM followed by a bias + GELU pass over its output; the rest is
    _BiasGeluDense (the GELU derivative in the data-gradient GEMM's epilogue)."""
    _check_cuda_bf16(x)
    wb1 = _bf16_weight(w1)
    o, i = wb1.shape
    if (_FFN_GEMM_GELU and w1.dtype == torch.float32 and w1.requires_grad and wb1.is_contiguous()
            and x.is_contiguous() and o % 8 == 0 and i % 8 == 0):
        z, h = _Dense.apply(x, w1, wb1, None, b1.detach().float().contiguous())
        return _BiasGeluDense.apply(z, b1, w2, _bf16_weight(w2), h)
    return bias_gelu_dense(dense(x, w1, None, impl="library"), b1, w2)


def _transposed_bf16(wb):
    """[o, i] bf16 weight -> contiguous [i, o] (the data-gradient GEMM's B operand): the dense
    weights are registered with the conv filters in forward, so the first data gradient of the
    step transposes all of them in ONE batched launch (see _dgrad_filter)."""
    o, i = wb.shape
    return _dgrad_filter(wb.view(o, 1, i)).view(i, o)


class _NativeDense(torch.autograd.Function):
    """y = act(x W^T + b) on the hand-written MFMA GEMM (csrc/kernels/gemm.hip) with the bias and
    ReLU in its epilogue (reference ``tf.layers.dense(..., activation=tf.nn.relu)``,
    ``run_mnist_distributed.py:67-69``).  Backward: one fused pass for
    ReluGrad + BiasAddGrad (csrc/kernels/dense.hip), dX on the same GEMM with the transposed
    weight, dW (fp32, straight into the flat gradient buffer) on the conv weight-gradient
    kernel's TN form (a 1x1 conv over M = tokens).  Output widths that are not a multiple of 8
    (the 10-way logits) run zero-padded to the next multiple of 8."""

    @staticmethod
    def forward(ctx, x, w_master, b_master, relu):
        wb = _bf16_weight(w_master)
        o, i = wb.shape
        x2 = x.reshape(-1, i)
        x2 = x2 if x2.is_contiguous() else x2.contiguous()
        op = -(-o // 8) * 8
        bias = b_master
        if op != o:
            wp = torch.zeros(op, i, device=x.device, dtype=_BF16)
            wp[:o] = wb
            wb = wp
            if b_master is not None:
                bias = torch.zeros(op, device=x.device, dtype=torch.float32)
                bias[:o] = b_master.detach()
        elif x.requires_grad and wb.is_contiguous():
            _register_dgrad_filter(wb.view(o, 1, 1, i))
        y = gemm_nt(x2, wb, bias=bias, relu=relu)
        ctx.save_for_backward(x2, wb, y if relu else None)
        ctx.meta = (o, op, relu, x.shape)
        ctx.params = (w_master, b_master)
        ctx.x_ref = x     # a fused LayerNorm may leave d(x) here (residual_to_dense)
        out = y if op == o else y[:, :o]
        return out.view(*x.shape[:-1], o)

    @staticmethod
    def backward(ctx, dy):
        x2, wb, y = ctx.saved_tensors
        o, op, relu, xshape = ctx.meta
        w_master, b_master = ctx.params
        M, i = x2.shape
        dy2 = dy.reshape(M, o)
        if op != o:
            dp = torch.zeros(M, op, device=dy.device, dtype=_BF16)
            dp[:, :o] = dy2
            dy2 = dp
        dy2 = dy2.contiguous() if dy2.dtype == _BF16 else dy2.to(_BF16).contiguous()
        dx = dw = db = None
        need_b = b_master is not None and ctx.needs_input_grad[2]
        if relu or need_b:
            dz = torch.empty_like(dy2) if relu else dy2
            ws = torch.empty(_K.bias_relu_bwd_ws_floats(op), device=dy.device, dtype=torch.float32)
            tb = _direct_grad(b_master) if need_b and op == o else None
            dbuf = None
            if need_b:
                dbuf = tb if tb is not None else torch.empty(op, device=dy.device,
                                                             dtype=torch.float32)
            _K.bias_relu_bwd(dy2.data_ptr(), _p(y) if relu else dy2.data_ptr(), dz.data_ptr(), M,
                             op, ws.data_ptr(), _p(dbuf), int(tb is not None), int(relu), _st())
            if need_b:
                if tb is not None:
                    _grad_ready(b_master)
                else:
                    db = dbuf[:o].to(b_master.dtype)
        else:
            dz = dy2
        if ctx.needs_input_grad[1]:
            target = _direct_grad(w_master) if op == o else None
            if target is not None:
                conv2d_wgrad(x2.view(M, 1, 1, i), dz.view(M, 1, 1, op), (op, 1, 1, i), 1, 0,
                             out=target.view(op, 1, 1, i))
                _grad_ready(w_master)
            else:
                dw = conv2d_wgrad(x2.view(M, 1, 1, i), dz.view(M, 1, 1, op), (op, 1, 1, i), 1,
                                  0).view(op, i)[:o]
                tw = _direct_grad(w_master)
                if tw is not None:
                    tw.add_(dw)
                    _grad_ready(w_master)
                    dw = None
                else:
                    dw = dw.to(w_master.dtype)
        pending = getattr(ctx.x_ref, "_dtf_pending_grad", None)
        if pending is not None:
            del ctx.x_ref._dtf_pending_grad
        ctx.x_ref = None
        if ctx.needs_input_grad[0]:
            wt = _transposed_bf16(wb)                     # [i, op]
            if pending is not None and pending.dtype == _BF16 and pending.is_contiguous():
                # d(x) = d(residual) + dz W in one GEMM (beta = 1 epilogue)
                dx = gemm_nt(dz, wt, out=pending.view(M, i), cin=pending.view(M, i)).view(xshape)
            else:
                dx = gemm_nt(dz, wt).view(xshape)
                if pending is not None:
                    dx = dx + pending.view(xshape)
        ctx.params = None
        return dx, dw, db, None


def dense(x, w, b=None, relu=False, impl=None):
    """Dense layer.  ``impl``: "native" (default; the hand-written MFMA GEMM with fused
    bias / ReLU epilogues) or "library" -- the name is historical: the bias-in-epilogue form
    BERT uses (:class:`_Dense`), whose forward and data gradient also run on our persistent MFMA
    GEMM for every shape it takes (``DTF_DENSE_GEMM=native``, the default; the fp32 bias is added
    in the epilogue, so it is not bit-identical to the hipBLASLt + bf16-bias A/B arm
    ``DTF_DENSE_GEMM=library``) and on hipBLASLt only for other shapes.  Trainable fp32 masters
    get fp32 dW / db straight in the flat buffer."""
    impl = impl or _DENSE_IMPL
    if (impl == "native" and w.dtype == torch.float32 and x.dtype == _BF16 and x.is_cuda
            and w.dim() == 2 and x.shape[-1] % 8 == 0):
        return _NativeDense.apply(x, w, b, bool(relu))
    if w.dtype == torch.float32 and x.dtype == _BF16 and w.requires_grad and x.is_cuda:
        y = _Dense.apply(x, w, _bf16_weight(w), b)
        return torch.relu(y) if relu else y
    wb = _bf16_weight(w) if w.dtype != x.dtype else w
    if w.requires_grad and wb is not w:
        wb = _MasterCast.apply(w, wb)
    y = torch.nn.functional.linear(x, wb, None if b is None else b.to(x.dtype))
    return torch.relu(y) if relu else y


class _MasterCast(torch.autograd.Function):
    """Use the bf16 shadow forward; route the gradient to the fp32 master in fp32."""

    @staticmethod
    def forward(ctx, master, shadow):
        ctx.dt = master.dtype
        return shadow

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.dt), None


# ----------------------------------------------------------------------------- loss

class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        lg = logits.detach().float().contiguous()
        B, V = lg.shape
        lab = labels.contiguous()
        if lab.dtype not in (torch.int64, torch.int32):
            lab = lab.long()
        rows = torch.empty(B, device=lg.device, dtype=torch.float32)
        grad = torch.empty_like(lg)
        _K.softmax_xent(lg.data_ptr(), lab.data_ptr(), lab.element_size(), B, V, rows.data_ptr(),
                        grad.data_ptr(), 1.0 / B, _st())
        ctx.save_for_backward(grad)
        ctx.ldt = logits.dtype
        return rows.mean()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return (grad * g).to(ctx.ldt), None


def sparse_softmax_cross_entropy(logits, labels):
    if logits.dim() != 2:
        raise ValueError("logits must be [B, V]")
    return _SoftmaxXent.apply(logits, labels)


# ----------------------------------------------------------------------------- transformer ops
# (LayerNorm / GELU / attention for BERT live in .native_nlp to keep this file focused)

def layer_norm(x, gamma, beta, eps=1e-12):
    from . import native_nlp
    return native_nlp.layer_norm(x, gamma, beta, eps)


def gelu(x):
    from . import native_nlp
    return native_nlp.gelu(x)


def attention(q, k, v, mask=None, scale=None):
    from . import native_nlp
    return native_nlp.attention(q, k, v, mask, scale)


def kernels():
    """The loaded extension module (for optimizers / strategies)."""
    return _K


def extension_path():
    return os.path.abspath(_K.__file__)
