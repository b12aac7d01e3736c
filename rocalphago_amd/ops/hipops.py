"""Torch-facing wrappers over the gfx950 HIP kernels (C ABI via ctypes).

All functions take/return torch CUDA tensors and launch on the current HIP stream, so they can be
captured into HIP graphs (torch.cuda.graph). Activations use the padded channels-last bf16 layout
described in csrc/hip/conv.hip: ``[B, S+2H, S+2H, CP]`` with a zero halo of width ``H`` and
``CP = round_up(C, 32)`` channels.
"""
import ctypes

import torch

from .._native import hip as _hip_lib

_PAD = 32


def pad_channels(c):
    return (c + _PAD - 1) // _PAD * _PAD


def _lib():
    return _hip_lib(required=True)


# ctypes converts plain ints / None for c_void_p arguments: no per-argument wrapper objects
def _ptr(t):
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream of the current device as a raw handle. The C-level getters cost
    ~1 us; torch.cuda.current_stream() builds a Stream object (~8 us, a third of a self-play
    ply's host time went there: profiles/selfplay_host_r3.txt)."""
    if _raw_stream is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


def _check(rc, name):
    if rc != 0:
        raise RuntimeError("%s failed (rc=%d)" % (name, rc))


def alloc_padded(B, S, H, CP, device, dtype=torch.bfloat16):
    """Zero-initialised padded activation buffer (the halo is never written afterwards)."""
    return torch.zeros((B, S + 2 * H, S + 2 * H, CP), dtype=dtype, device=device)


def pack_weights(w, coutp, cinp, wf=None, wb=None):
    """OIHW fp32 -> bf16 forward [taps, coutp, cinp] (+ dgrad [taps, cinp, coutp] if wb given)."""
    cout, cin, ks, _ = w.shape
    taps = ks * ks
    if wf is None:
        wf = torch.empty((taps, coutp, cinp), dtype=torch.bfloat16, device=w.device)
    w = w.contiguous()
    _check(_lib().rag_pack_weights(_ptr(w), _ptr(wf), _ptr(wb), cout, cin, ks, coutp, cinp,
                                   _stream()), "pack_weights")
    return wf, wb


def pack_trunk(table, nrows, total, nfull=None, sgd=None):
    """Repack every layer of a trunk in one launch (table: device int64 [nrows, 11], see
    rag_pack_trunk in csrc/hip/conv.hip; ``total`` = 64x64 tap tiles of the largest layer). Rows
    past the first ``nfull`` (default: all) only pad their bias. ``sgd`` = (goff, lr, wd): step
    every fp32 master by SGD first (its gradient ``goff`` elements further), in the same pass."""
    nfull = nrows if nfull is None else nfull
    goff, lr, wd = sgd if sgd is not None else (0, 0.0, 0.0)
    _check(_lib().rag_pack_trunk(_ptr(table), nrows, nfull, int(total), _stream(), int(goff),
                                 float(lr), float(wd), 1 if sgd is not None else 0),
           "pack_trunk")


# (free function, handle buffer) of PendingReduction handles dropped during a stream capture
_DEFERRED_FREE = []


def _free_deferred():
    """Frees the handles whose owners died during a stream capture (called where a handle is
    created: never inside a capture, which a hipMalloc would invalidate as well)."""
    while _DEFERRED_FREE:
        free, buf = _DEFERRED_FREE.pop()
        free(ctypes.cast(buf, ctypes.c_void_p))


class PendingReduction(object):
    """Caller-owned handle of a deferred wgrad partial-slab reduction (conv.hip PendingRed):
    ``conv_wgrad(defer=True, pending=h)`` leaves the reduction in ``h``; the next
    ``conv_igemm(..., pending=h)`` on the same stream runs it in its free block slots, and
    ``wgrad_flush(h)`` launches it on its own. Launches without the handle never touch it."""

    def __init__(self):
        _free_deferred()
        self.buf = ctypes.create_string_buffer(int(_lib().rag_wgrad_pending_bytes()))
        # claim counters allocated now (a hipMalloc on first deferral synchronised the device
        # mid-step) and freed with the handle
        _check(_lib().rag_wgrad_pending_init(self.ptr), "wgrad_pending_init")
        self._free = _lib().rag_wgrad_pending_free

    def __del__(self):
        try:
            # the cyclic garbage collector can drop a dead trunk's handle in the middle of a HIP
            # graph capture on this thread (torch.cuda.graph does not collect first), and a
            # hipFree there invalidates the capture: keep it for the next safe point instead
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                _DEFERRED_FREE.append((self._free, self.buf))
                return
            self._free(self.ptr)
        except Exception:  # interpreter shutdown: the library may be gone already
            pass

    @property
    def ptr(self):
        return ctypes.cast(self.buf, ctypes.c_void_p)


def _hptr(pending):
    return None if pending is None else pending.ptr


_INT32_MAX = 2 ** 31 - 1


def _index_range_ok(*tensors):
    """The conv / BN / packing kernels index activations with 32-bit element offsets: refuse
    (loudly, before launch) a batch whose padded activation reaches 2^31 elements instead of
    faulting on a wrapped address. Callers split such batches (e.g. reinforcement.py)."""
    for t in tensors:
        if t is not None and t.numel() > _INT32_MAX:
            raise ValueError("activation of %d elements exceeds the kernels' 32-bit indexing; "
                             "split the batch (max rows ~ %d)" %
                             (t.numel(), _INT32_MAX // max(1, t[0].numel())))


def max_rows(S, halo, channels):
    """Largest batch whose padded [B, S+2h, S+2h, C] activation the kernels can index."""
    return _INT32_MAX // ((S + 2 * halo) ** 2 * channels)


def conv_igemm(x, wpack, bias, y, B, S, hi, ho, cinp, coutp, ks, relu, mask=None,
               mask_halo=None, residual=None, pending=None, cin=None):
    """y[pad ho] = act(conv_ks(x[pad hi]) + bias [+ residual]), or the dgrad form with a ReLU
    mask (the layer input: y's channel count, its own halo ``mask_halo``, default ho).
    ``residual`` (ResNet sum-merge) has y's layout and may be y itself. ``pending``: a
    PendingReduction whose deferred wgrad reduction rides along this launch."""
    _index_range_ok(x, y, mask, residual)
    hm = ho if mask_halo is None else mask_halo
    if mask is not None and (mask.shape[1] != S + 2 * hm or mask.shape[-1] != y.shape[-1]):
        raise ValueError("mask layout does not match (halo %d, %d channels)" % (hm, y.shape[-1]))
    if residual is not None and residual.shape[1:] != y.shape[1:]:
        raise ValueError("residual layout does not match the output")
    if cin is not None and cin < cinp:
        # the real input channel count lets the 5x5 input layer skip its zero channels
        _check(_lib().rag_conv_igemm_cin(_ptr(x), _ptr(wpack), _ptr(bias), _ptr(y), _ptr(mask),
                                         _ptr(residual), B, S, hi, ho, cinp, coutp, y.shape[-1],
                                         ks, int(relu), hm, _stream(), _hptr(pending), int(cin)),
               "conv_igemm")
        return y
    _check(_lib().rag_conv_igemm(_ptr(x), _ptr(wpack), _ptr(bias), _ptr(y), _ptr(mask),
                                 _ptr(residual), B, S, hi, ho, cinp, coutp, y.shape[-1], ks,
                                 int(relu), hm, _stream(), _hptr(pending)), "conv_igemm")
    return y


def conv_wino_ok(S, hi, kin, nout, ks):
    """True if conv_wino (Winograd F(2,3) along the width, csrc/hip/conv_wino.hip) runs this
    layer: 3x3, input halo 1, input channels a multiple of 32, output channels of 192."""
    return bool(_lib().rag_conv_wino_ok(S, hi, kin, nout, ks))


def conv_wino_prefer(B, S, kin, nout):
    """True if conv_wino should take this layer at batch B rather than the direct kernel: one
    board per block and a last wave of blocks that fills at least 7/8 of the CUs."""
    return bool(_lib().rag_conv_wino_prefer(B, S, kin, nout))


def conv_wino_mode(B, S, kin, nout):
    """How conv_wino runs batch B: 1 one-board blocks, 2 half-board blocks (two per board:
    batches whose one-board grid would leave the chip half idle), 0 not preferred."""
    return int(_lib().rag_conv_wino_mode(B, S, kin, nout))


def wino_pack(table, nlayers, max_tiles, sgd=None):
    """Winograd weights of 3x3 layers from their fp32 OIHW masters in one launch. ``table``:
    device int64 [nlayers, 8] = (W, cout, cin, coutp, cinp, Uf, Ub or 0, Wd or 0); Uf (forward,
    N = coutp, K = cinp) and Ub (dgrad, N = cinp, K = coutp) each 12 * N * K bf16, stored
    fragment-major [12][K/32][N/16][64][8] (conv_wino.hip); Wd: the direct dgrad layout
    [9, cinp, coutp] (pack_trunk's); ``max_tiles``: 64x64 (n, c) tiles of the widest layer.
    ``sgd`` = (goff, lr, wd): the optimizer step folded in (pack_trunk)."""
    goff, lr, wd = sgd if sgd is not None else (0, 0.0, 0.0)
    _check(_lib().rag_wino_pack(_ptr(table), nlayers, int(max_tiles), _stream(), int(goff),
                                float(lr), float(wd), 1 if sgd is not None else 0), "wino_pack")


def pack_step(wtable, nwino, ttable, nrows, nfull, max_taps, width, sgd=None, flat=None,
              rest=()):
    """A fused trunk's whole weight update in one launch (rag_pack_step, csrc/hip/conv_wino.hip):
    the ``nwino`` Winograd rows of ``wtable`` (wino_pack's table), the pack_trunk rows of
    ``ttable`` (``nrows``, ``nfull``: pack_trunk's; kernels up to ``max_taps`` taps) on a grid
    ``width`` blocks wide, and with ``sgd`` = (goff, lr, wd) the optimizer step folded in plus
    plain SGD over the (at most two) [start, end) element ranges ``rest`` of ``flat``."""
    if len(rest) > 2:
        raise ValueError("pack_step steps at most two rest ranges, got %d" % len(rest))
    goff, lr, wd = sgd if sgd is not None else (0, 0.0, 0.0)
    rr = [(a, b - a) for a, b in rest] + [(0, 0)] * (2 - len(rest))
    _check(_lib().rag_pack_step(_ptr(wtable), int(nwino), _ptr(ttable), int(nrows), int(nfull),
                                int(max_taps), int(width), _stream(), int(goff), float(lr),
                                float(wd), 1 if sgd is not None else 0, _ptr(flat),
                                rr[0][0], rr[0][1], rr[1][0], rr[1][1]), "pack_step")


def wino_weights(w, coutp, cinp, dgrad=True):
    """(Uf, Ub) Winograd weights of one OIHW fp32 3x3 weight tensor (tests, one-off layers)."""
    cout, cin = w.shape[:2]
    w = w.contiguous()
    uf = torch.empty((12, coutp, cinp), dtype=torch.bfloat16, device=w.device)
    ub = torch.empty((12, cinp, coutp), dtype=torch.bfloat16, device=w.device) if dgrad else None
    table = torch.tensor([[w.data_ptr(), cout, cin, coutp, cinp, uf.data_ptr(),
                           0 if ub is None else ub.data_ptr(), 0]], dtype=torch.int64)
    table = table.to(w.device)
    wino_pack(table, 1, -(-coutp // 64) * -(-cinp // 64))
    torch.cuda.current_stream(w.device).synchronize()  # the table is a temporary
    return uf, ub


def conv_wino(x, u, bias, y, B, S, kin, nout, ho, relu, mask=None, mask_halo=None,
              pending=None, half=False):
    """y[pad ho] = act(conv3x3(x[pad 1]) + bias) through the Winograd kernel with the layer's
    Winograd weights ``u`` [12, nout, kin] (wino_pack), or the dgrad form with a ReLU mask (the
    layer input, y's channel count, halo ``mask_halo``). ``pending``: a PendingReduction whose
    deferred wgrad reduction rides along the launch. ``half``: half-board blocks whenever the
    shape has them (launches sharing the chip with resident kernels, e.g. GPU rollouts)."""
    _index_range_ok(x, y, mask)
    hm = ho if mask_halo is None else mask_halo
    if x.shape[1] != S + 2 or x.shape[-1] != kin:
        raise ValueError("conv_wino input must have halo 1 and %d channels" % kin)
    if mask is not None and (mask.shape[1] != S + 2 * hm or mask.shape[-1] != y.shape[-1]):
        raise ValueError("mask layout does not match (halo %d, %d channels)" % (hm, y.shape[-1]))
    _check(_lib().rag_conv_wino_p(_ptr(x), _ptr(u), _ptr(bias), _ptr(y), _ptr(mask), B, S, kin,
                                  nout, ho, y.shape[-1], int(relu), hm, _stream(),
                                  _hptr(pending), int(bool(half))), "conv_wino")
    return y


def conv_wino_bn_ok(B, S, kin, nout):
    """True if conv_wino_bn (the Winograd kernel with the residual trunk's fused BatchNorm) runs
    a batch of B: 128 -> 128 channels, one board per block, a grid that fills the chip."""
    return bool(_lib().rag_conv_wino_bn_ok(B, S, kin, nout))


def conv_wino_bn(x, u, bias, y, B, S, kin, nout, relu, bn_coef=None, mask=None, mask_coef=None,
                 residual=None, pending=None, stat_part=None, stat_mean=None):
    """conv_igemm_bn's two forms on the Winograd kernel (conv_wino.hip WinoBN) with the layer's
    Winograd weights ``u``: forward (``bn_coef``: x is the BN input, U = ReLU(bn_coef[0][col] x +
    bn_coef[2][col]) is built in the input transform; optional ``residual``) or dgrad
    (``mask`` = x and ``mask_coef``). ``stat_part`` [B, 2, S]: one partial row pair per board
    (bn_finalize_fwd / bn_finalize_bwd with nblk = B). Needs conv_wino_bn_ok(B, ...)."""
    _index_range_ok(x, y, mask, residual)
    if x.shape[1] != S + 2 or x.shape[-1] != kin or y.shape[1] != S + 2:
        raise ValueError("conv_wino_bn input and output have halo 1 (%d input channels)" % kin)
    if residual is not None and residual.shape[1:] != y.shape[1:]:
        raise ValueError("residual layout does not match the output")
    if mask is not None and (mask.shape[1] != S + 2 or mask.shape[-1] != y.shape[-1]):
        raise ValueError("mask layout does not match (halo 1, %d channels)" % y.shape[-1])
    if (mask is None) != (mask_coef is None) or (bn_coef is None) == (mask_coef is None):
        raise ValueError("conv_wino_bn: bn_coef (forward) or mask + mask_coef (dgrad)")
    if stat_part is not None and stat_part.shape[0] < B:
        raise ValueError("stat_part needs one row pair per board")
    _check(_lib().rag_conv_wino_bn(_ptr(x), _ptr(u), _ptr(bias), _ptr(y), _ptr(mask),
                                   _ptr(residual), B, S, kin, nout, 1, y.shape[-1], int(relu), 1,
                                   _stream(), _hptr(pending), _ptr(bn_coef), _ptr(mask_coef),
                                   _ptr(stat_part), _ptr(stat_mean)), "conv_wino_bn")
    return y


def conv_bn_fusable(B, S, hi, cinp, coutp, ks):
    """True if a layer of this shape can take its input as BN input x + column coefficients
    (conv_igemm_bn / conv_wgrad(xcoef=...)): 3x3, 128 channels, a grid that fills the chip."""
    return bool(_lib().rag_conv_bn_fusable(B, S, hi, cinp, coutp, ks))


def conv_bn_stat_blocks(B, S, coutp):
    """Partial rows [n][2][S] a statistics-producing conv_igemm_bn writes (its block count)."""
    return int(_lib().rag_conv_bn_stat_blocks(B, S, coutp))


def conv_igemm_bn(x, wpack, bias, y, B, S, cinp, coutp, relu, bn_coef=None, mask=None,
                  mask_coef=None, residual=None, pending=None, stat_part=None, stat_mean=None):
    """3x3 conv whose input is U = ReLU(bn_coef[0][col] * x + bn_coef[2][col]) computed while
    staging (x = the BN input, halo 1; U is never stored), and/or the dgrad form whose ReLU mask
    U > 0 is recomputed from ``mask`` = x and ``mask_coef``. Only shapes with
    conv_bn_fusable(...) have a kernel. ``residual``: as conv_igemm (forward form only).
    ``stat_part`` [conv_bn_stat_blocks, 2, S] fp32: the output's BN column statistics as per-block
    partials for bn_finalize_fwd (sum, sum of squares), or, with ``stat_mean`` (the BN mean) in the
    dgrad form, for bn_finalize_bwd (sum dU, sum dU (x - mean))."""
    _index_range_ok(x, y, mask, residual)
    if residual is not None and residual.shape[1:] != y.shape[1:]:
        raise ValueError("residual layout does not match the output")
    if mask is not None and (mask.shape[1] != S + 2 or mask.shape[-1] != y.shape[-1]):
        raise ValueError("mask layout does not match (halo 1, %d channels)" % y.shape[-1])
    if (mask is None) != (mask_coef is None):
        raise ValueError("mask and mask_coef go together")
    _check(_lib().rag_conv_igemm_bn(_ptr(x), _ptr(wpack), _ptr(bias), _ptr(y), _ptr(mask),
                                    _ptr(residual), B, S, 1, 1, cinp, coutp, y.shape[-1],
                                    int(relu), 1, _stream(),
                                    _hptr(pending), _ptr(bn_coef), _ptr(mask_coef),
                                    _ptr(stat_part), _ptr(stat_mean)),
           "conv_igemm_bn")
    return y


# ---- column BatchNorm (bn.hip; ResnetPolicy). Activations use the padded layout above; every
# per-column vector (gamma, beta, running mean / var, stats [2, S], coef [3, S]) is fp32.

def _halo(t, S):
    return (t.shape[1] - S) // 2


def bn_workspace(B, S, device):
    n = _lib().rag_bn_workspace(B, S)
    key = ("bn", device)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(n + 256, dtype=torch.float32, device=device)
        _ws_cache[key] = buf
    return buf


def bn_train_fwd(x, B, S, C, gamma, beta, rmean, rvar, eps, momentum, stats, coef):
    """Batch statistics of x [pad] per column -> stats (mean, rstd), coef (affine), running
    averages updated in place (skipped when rmean is None)."""
    _check(_lib().rag_bn_train_fwd(_ptr(x), _halo(x, S), B, S, C, x.shape[-1], _ptr(gamma),
                                   _ptr(beta), _ptr(rmean), _ptr(rvar), float(eps),
                                   float(momentum), _ptr(stats), _ptr(coef),
                                   _ptr(bn_workspace(B, S, x.device)), _stream()), "bn_train_fwd")


def bn_infer_coef(gamma, beta, rmean, rvar, eps, S, coef):
    _check(_lib().rag_bn_infer_coef(_ptr(gamma), _ptr(beta), _ptr(rmean), _ptr(rvar),
                                    float(eps), S, _ptr(coef), _stream()), "bn_infer_coef")


def bn_finalize_fwd(part, nblk, B, S, C, gamma, beta, rmean, rvar, eps, momentum, stats, coef):
    """bn_train_fwd from per-block partials a fused conv epilogue wrote (conv_igemm_bn
    ``stat_part``)."""
    _check(_lib().rag_bn_finalize_fwd(_ptr(part), nblk, B, S, C, _ptr(gamma), _ptr(beta),
                                      _ptr(rmean), _ptr(rvar), float(eps), float(momentum),
                                      _ptr(stats), _ptr(coef), _stream()), "bn_finalize_fwd")


def bn_finalize_bwd(part, nblk, B, S, C, gamma, stats, dgamma, dbeta, coef):
    """bn_bwd_coef from per-block partials of a fused dgrad epilogue (conv_igemm_bn
    ``stat_part`` + ``stat_mean``)."""
    _check(_lib().rag_bn_finalize_bwd(_ptr(part), nblk, B, S, C, _ptr(gamma), _ptr(stats),
                                      _ptr(dgamma), _ptr(dbeta), _ptr(coef), _stream()),
           "bn_finalize_bwd")


def bn_bwd_coef(x, dy, B, S, C, gamma, stats, dgamma, dbeta, coef):
    _check(_lib().rag_bn_bwd_coef(_ptr(x), _halo(x, S), _ptr(dy), _halo(dy, S), B, S, C,
                                  x.shape[-1], _ptr(gamma), _ptr(stats), _ptr(dgamma),
                                  _ptr(dbeta), _ptr(coef), _ptr(bn_workspace(B, S, x.device)),
                                  _stream()), "bn_bwd_coef")


def bn_apply(x, out, B, S, C, coef=None, relu=True, dy=None, residual=None):
    """out = act(coef[0]*x + coef[1]*dy + coef[2] + residual) (interior; padded channels 0)."""
    CP = x.shape[-1]
    for t in (out, dy, residual):
        if t is not None and t.shape[-1] != CP:
            raise ValueError("bn_apply channel mismatch")
    _check(_lib().rag_bn_apply(_ptr(x), _halo(x, S), _ptr(dy), 0 if dy is None else _halo(dy, S),
                               _ptr(residual), 0 if residual is None else _halo(residual, S),
                               _ptr(out), _halo(out, S), _ptr(coef), int(relu), B, S, C, CP,
                               _stream()), "bn_apply")
    return out


def bn_apply_bwd_part(part, nblk, x, out, B, S, C, gamma, stats, dgamma, dbeta, dy,
                      residual=None):
    """bn_finalize_bwd + bn_apply(dy, coef) in one launch: out = dL/dx [+ residual] of a BN
    whose backward statistics are the per-block partials ``part`` [nblk, 2, S] (each block of
    the apply derives the column coefficients itself); dgamma / dbeta as bn_finalize_bwd."""
    CP = x.shape[-1]
    for t in (out, dy, residual):
        if t is not None and t.shape[-1] != CP:
            raise ValueError("bn_apply channel mismatch")
    _check(_lib().rag_bn_apply_bwd_part(
        _ptr(part), int(nblk), _ptr(gamma), _ptr(stats), _ptr(dgamma), _ptr(dbeta), _ptr(x),
        _halo(x, S), _ptr(dy), _halo(dy, S), _ptr(residual),
        0 if residual is None else _halo(residual, S), _ptr(out), _halo(out, S), B, S, C, CP,
        _stream()), "bn_apply_bwd_part")
    return out


_ws_cache = {}


def wgrad_workspace(B, S, coutp, cinp, ks, device):
    n = _lib().rag_conv_wgrad_workspace(B, S, coutp, cinp, ks, None)
    key = (device, )
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(int(n * 1.25) + 1024, dtype=torch.float32, device=device)
        _ws_cache[key] = buf
    return buf


def conv_wgrad(g, x, dw, db, B, S, hi, cout, coutp, cin, cinp, ks, accumulate=False, work=None,
               hg=None, reduce_stream=None, defer=False, pending=None, xcoef=None):
    """dW (OIHW fp32) and db from dL/dpre g [pad hg] and the layer input x [pad hi].
    ``reduce_stream`` (a torch stream): run the partial-slab reduction there, ordered after the
    wgrad kernel by an event, so it overlaps the following kernels of the current stream; the
    caller then owns the ordering of ``work`` reuse and of ``dw``/``db`` consumers.
    ``defer``: leave an fp16 partial-slab reduction pending in ``pending`` (a PendingReduction,
    required); the next ``conv_igemm(..., pending=pending)`` on this stream runs it in its free
    block slots (or ``wgrad_flush(pending)`` launches it). ``dw``/``db`` are final only after
    that. ``xcoef`` (BN prologue, conv_bn_fusable shapes): x is the BN input and the layer input
    is U = ReLU(xcoef[0][col] * x + xcoef[2][col]), applied while staging."""
    _index_range_ok(g, x)
    if work is None:
        work = wgrad_workspace(B, S, coutp, cinp, ks, g.device)
    if hg is None:
        hg = (g.shape[1] - S) // 2
    if xcoef is not None:
        if reduce_stream is not None:
            raise ValueError("conv_wgrad(xcoef=...) has no reduce-stream form")
        _check(_lib().rag_conv_wgrad_deferred_bn(_ptr(g), _ptr(x), _ptr(dw), _ptr(db), _ptr(work),
                                                 B, S, hi, hg, g.shape[-1], cout, coutp, cin,
                                                 cinp, ks, int(accumulate), _stream(),
                                                 _hptr(pending) if defer else None, _ptr(xcoef)),
               "conv_wgrad_bn")
        return
    if defer and reduce_stream is None:
        if pending is None:
            raise ValueError("conv_wgrad(defer=True) needs a PendingReduction handle")
        _check(_lib().rag_conv_wgrad_deferred(_ptr(g), _ptr(x), _ptr(dw), _ptr(db), _ptr(work), B,
                                              S, hi, hg, g.shape[-1], cout, coutp, cin, cinp, ks,
                                              int(accumulate), _stream(), pending.ptr),
               "conv_wgrad_deferred")
        return
    rs = ctypes.c_void_p(reduce_stream.cuda_stream) if reduce_stream is not None else None
    _check(_lib().rag_conv_wgrad(_ptr(g), _ptr(x), _ptr(dw), _ptr(db), _ptr(work), B, S, hi, hg,
                                 g.shape[-1], cout, coutp, cin, cinp, ks, int(accumulate),
                                 _stream(), rs), "conv_wgrad")


def wgrad_flush(pending):
    """Launch the reduction left in ``pending`` by ``conv_wgrad(defer=True)`` (no-op if none)."""
    _check(_lib().rag_wgrad_flush(_stream(), pending.ptr), "wgrad_flush")


def pack_input(features, out, H, index=None, transforms=None, nplanes=None):
    """[N, F, S, S] uint8/float32 planes (the first ``nplanes`` of them when given), or
    bit-packed int64 words [N, S, S] with ``nplanes`` (training/replay.py), optionally gathered
    by ``index`` [B] and dihedral-transformed by ``transforms`` [B] int32 -> padded bf16 ``out``
    [B, S+2H, S+2H, CP]."""
    B = out.shape[0]
    S = features.shape[-1]
    CP = out.shape[-1]
    if features.dtype == torch.int64:
        if nplanes is None:
            raise ValueError("bit-packed input needs nplanes")
        _check(_lib().rag_pack_input_bits(_ptr(features), _ptr(index), _ptr(transforms),
                                          _ptr(out), B, int(nplanes), S, H, CP, _stream()),
               "pack_input_bits")
        return out
    FS = features.shape[1]  # planes per position in the source
    NF = FS if nplanes is None else min(FS, int(nplanes))  # planes packed
    if features.dtype not in (torch.uint8, torch.float32):
        features = features.float()
    if not features.is_contiguous():
        features = features.contiguous()
    fn = _lib().rag_pack_input_u8 if features.dtype == torch.uint8 else _lib().rag_pack_input_f32
    _check(fn(_ptr(features), _ptr(index), _ptr(transforms), _ptr(out), B, NF, FS, S, H, CP,
              _stream()), "pack_input")
    return out


def unpack(x, C, H):
    """padded channels-last bf16 -> NCHW fp32 (first C channels)."""
    B, WP, _, CP = x.shape
    S = WP - 2 * H
    out = torch.empty((B, C, S, S), dtype=torch.float32, device=x.device)
    _check(_lib().rag_unpack(_ptr(x), _ptr(out), B, C, S, H, CP, _stream()), "unpack")
    return out


def pack_nchw(t, H, CP, out=None):
    B, C, S, _ = t.shape
    if out is None:
        out = alloc_padded(B, S, H, CP, t.device)
    t = t.contiguous().float()
    _check(_lib().rag_pack_nchw(_ptr(t), _ptr(out), B, C, S, H, CP, _stream()), "pack_nchw")
    return out


def policy_head_fwd(h, w, b0, pbias, probs, K, labels=None, sweight=None, loss=None, dz=None,
                    hit=None, mode=0, gscale=1.0, pass_w=None, pass_b=None, zout=None,
                    dpass=None, acc=None, dzsum=None):
    """Fused 1x1 conv + bias + softmax (+ loss / dL/dz). With ``pass_w``/``pass_b`` (PassLogit)
    probs are [B, S*S + 1] (pass last), ``zout`` gets the position logits and ``dpass`` the
    pass-logit gradient for the PassLogit weight gradients. ``acc`` (fp32 [2], optional): the
    batch's loss sum and top-1 hit count are added to it in the kernel."""
    B, WP, _, KP = h.shape
    S = WP - 2
    if acc is not None and (acc.dtype != torch.float32 or acc.numel() < 2):
        raise ValueError("acc must be an fp32 tensor of >= 2 elements")
    if pass_w is not None:
        _check(_lib().rag_policy_head_pass_fwd(
            _ptr(h), _ptr(w), _ptr(b0), _ptr(pbias), _ptr(pass_w), _ptr(pass_b), _ptr(probs),
            _ptr(labels), _ptr(sweight), _ptr(loss), _ptr(dz), _ptr(hit), _ptr(zout),
            _ptr(dpass), _ptr(acc), B, S, KP, K, mode, float(gscale), _stream()),
            "policy_head_pass_fwd")
        return
    if dzsum is not None:  # + each board's sum of dz (head_bwd's fixed-order db0)
        _check(_lib().rag_policy_head_fwd_s(_ptr(h), _ptr(w), _ptr(b0), _ptr(pbias), _ptr(probs),
                                            _ptr(labels), _ptr(sweight), _ptr(loss), _ptr(dz),
                                            _ptr(hit), _ptr(acc), _ptr(dzsum), B, S, KP, K, mode,
                                            float(gscale), _stream()), "policy_head_fwd")
        return
    _check(_lib().rag_policy_head_fwd(_ptr(h), _ptr(w), _ptr(b0), _ptr(pbias), _ptr(probs),
                                      _ptr(labels), _ptr(sweight), _ptr(loss), _ptr(dz),
                                      _ptr(hit), _ptr(acc), B, S, KP, K, mode, float(gscale),
                                      _stream()), "policy_head_fwd")


def pass_grads(zout, dpass, dW, db):
    """PassLogit weight gradients on the GPU: dW = dpass^T zout ([S*S]), db = sum(dpass)."""
    B, P = zout.shape
    if dpass.numel() != B or dW.numel() != P or db.numel() != 1 or not zout.is_contiguous():
        raise ValueError("pass_grads: zout [B, P] contiguous, dpass [B], dW [P], db [1]")
    _check(_lib().rag_pass_grads(_ptr(zout), _ptr(dpass), _ptr(dW), _ptr(db), B, P, _stream()),
           "pass_grads")


_head_ws = {}


def head_bwd(h, w, dz, dh, dw, db0, dpbias, K, relu_mask=True, work=None, metrics=None,
             dzsum=None):
    """dH (ReLU-masked) + dw / db0 / dpbias (all overwritten, not accumulated). ``metrics``:
    (loss [B], hit [B], acc fp32 [2]) -- the head forward's per-board values, added to the
    running sums acc by the reduce launch (policy_head_fwd then runs with acc=None)."""
    B, WP, _, KP = h.shape
    S = WP - 2
    if work is None:
        need = _lib().rag_head_bwd_workspace(B, S, KP)
        work = _head_ws.get(h.device)
        if work is None or work.numel() < need:
            work = torch.empty(need, dtype=torch.float32, device=h.device)
            _head_ws[h.device] = work
    ml = mh = acc = None
    if metrics is not None:
        ml, mh, acc = metrics
        if acc.dtype != torch.float32 or acc.numel() < 2 or ml.numel() < B or mh.numel() < B:
            raise ValueError("head_bwd metrics: loss [B], hit [B], fp32 acc [2]")
    if dzsum is not None and dzsum.numel() < B:
        raise ValueError("head_bwd dzsum: [B] per-board sums expected")
    # db0 in a fixed summation order (from dzsum, or from dz itself when the forward gave none)
    _check(_lib().rag_head_bwd_m(_ptr(h), _ptr(w), _ptr(dz), _ptr(dh), _ptr(dw), _ptr(db0),
                                 _ptr(dpbias), _ptr(work), B, S, KP, K, int(relu_mask),
                                 _ptr(ml), _ptr(mh), _ptr(acc), _ptr(dzsum), _stream()),
           "head_bwd")


def head_linear(h, w, b0, z, K):
    B, WP, _, KP = h.shape
    S = WP - 2
    _check(_lib().rag_head_linear(_ptr(h), _ptr(w), _ptr(b0), _ptr(z), B, S, KP, K, _stream()),
           "head_linear")


MLP_ACTS = {"linear": 0, "relu": 1, "tanh": 2}
_mlp_ws = {}


def value_mlp_fwd(z, W1, b1, W2, b2, act="linear", out=None, hout=None):
    """tanh(act(z @ W1 + b1) @ W2 + b2) for fp32 z [B, P], W1 [P, H], W2 [H, 1] -> [B, 1].
    ``hout`` (fp32 [B, H], optional) receives the pre-activation z @ W1 + b1 (training)."""
    B, P = z.shape
    H = W1.shape[1]
    if (W1.shape != (P, H) or b1.numel() != H or W2.numel() != H or b2.numel() != 1
            or act not in MLP_ACTS):
        raise ValueError("value_mlp_fwd: bad shapes/activation %s %s %s" %
                         (tuple(z.shape), tuple(W1.shape), act))
    for t in (z, W1, b1, W2, b2):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("value_mlp_fwd expects contiguous fp32 tensors")
    if hout is not None and (hout.shape != (B, H) or hout.dtype != torch.float32
                             or not hout.is_contiguous()):
        raise ValueError("value_mlp_fwd: hout must be contiguous fp32 [B, H]")
    if out is None:
        out = torch.empty((B, 1), dtype=torch.float32, device=z.device)
    need = _lib().rag_value_mlp_workspace(B, H)
    stream = _stream()
    key = (z.device, stream)  # per stream: pipelined evaluations may run concurrently
    work = _mlp_ws.get(key)
    if work is None or work.numel() < need:
        work = torch.empty(need, dtype=torch.float32, device=z.device)
        _mlp_ws[key] = work
    _check(_lib().rag_value_mlp_fwd(_ptr(z), _ptr(W1), _ptr(b1), _ptr(W2), _ptr(b2), _ptr(out),
                                    _ptr(work), _ptr(hout), B, P, H, MLP_ACTS[act], stream),
           "value_mlp_fwd")
    return out


def sl_batch(index, labels, tf_table, sym, seed, step, tf_out=None, lab_out=None):
    """One launch per SL step (batch.hip): a random allowed dihedral transform per sampled row
    (int32 [B]) and the transformed target index (int64 [B])."""
    B = index.numel()
    dev = index.device
    for t, dt in ((index, torch.int64), (labels, torch.int64), (tf_table, torch.int64),
                  (sym, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError("sl_batch: bad dtype / layout")
    if tf_out is None:
        tf_out = torch.empty(B, dtype=torch.int32, device=dev)
    if lab_out is None:
        lab_out = torch.empty(B, dtype=torch.int64, device=dev)
    _check(_lib().rag_sl_batch(_ptr(index), _ptr(labels), _ptr(tf_table), tf_table.shape[1],
                               _ptr(sym), sym.numel(), ctypes.c_uint(seed & 0xFFFFFFFF),
                               ctypes.c_uint(step & 0xFFFFFFFF), _ptr(tf_out), _ptr(lab_out), B,
                               _stream()), "sl_batch")
    return tf_out, lab_out


def value_batch(index, values, sym, seed, step, tf_out=None, y_out=None):
    """One launch per value-net step (batch.hip): a random allowed dihedral transform per sampled
    row (int32 [B]) and its target outcome values[index] (float [B, 1])."""
    B = index.numel()
    dev = index.device
    for t, dt in ((index, torch.int64), (values, torch.float32), (sym, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError("value_batch: bad dtype / layout")
    if tf_out is None:
        tf_out = torch.empty(B, dtype=torch.int32, device=dev)
    if y_out is None:
        y_out = torch.empty((B, 1), dtype=torch.float32, device=dev)
    _check(_lib().rag_value_batch(_ptr(index), _ptr(values), _ptr(sym), sym.numel(),
                                  ctypes.c_uint(seed & 0xFFFFFFFF),
                                  ctypes.c_uint(step & 0xFFFFFFFF), _ptr(tf_out), _ptr(y_out),
                                  B, _stream()), "value_batch")
    return tf_out, y_out


_mlp_train_ws = {}


def value_mlp_train(z, W1, b1, W2, b2, y, sw, act, dW1, db1, dW2, db2, dz=None, vout=None):
    """Forward + backward of the value MLP head under the MSE loss, all on HIP kernels
    (head.hip value_mlp_part_kernel, value_bwd.hip): writes dW1 [P, H], db1 [H], dW2 [H],
    db2 [1] and (optional) dz [B, P] = dL/dz; returns the per-board loss terms [B] (their sum is
    the batch loss). y: targets [B] or [B, 1]; sw: optional sample weights [B]."""
    B, P = z.shape
    H = W1.shape[1]
    if (W1.shape != (P, H) or b1.numel() != H or W2.numel() != H or b2.numel() != 1
            or act not in MLP_ACTS or y.numel() != B or (sw is not None and sw.numel() != B)):
        raise ValueError("value_mlp_train: bad shapes/activation %s %s %s" %
                         (tuple(z.shape), tuple(W1.shape), act))
    for t in (z, W1, b1, W2, b2, y, sw, dW1, db1, dW2, db2, dz, vout):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("value_mlp_train expects contiguous fp32 tensors")
    if dW1.numel() != P * H or db1.numel() != H or dW2.numel() != H or db2.numel() != 1 or \
            (dz is not None and dz.shape != (B, P)) or (vout is not None and vout.numel() != B):
        raise ValueError("value_mlp_train: bad gradient shapes")
    lib = _lib()
    stream = _stream()
    key = (z.device, stream)
    ws = _mlp_train_ws.get(key)
    npart, nbwd = lib.rag_value_mlp_workspace(B, H), lib.rag_value_mlp_bwd_workspace(B, H)
    if ws is None or ws[0].numel() < npart or ws[1].numel() < B * H or ws[2].numel() < nbwd \
            or ws[3].numel() < B:
        ws = tuple(torch.empty(n, dtype=torch.float32, device=z.device)
                   for n in (npart, B * H, nbwd, B))
        _mlp_train_ws[key] = ws
    part, hpre, work, loss = ws
    _check(lib.rag_value_mlp_fwd(_ptr(z), _ptr(W1), _ptr(b1), _ptr(W2), _ptr(b2), _ptr(None),
                                 _ptr(part), _ptr(hpre), B, P, H, MLP_ACTS[act], stream),
           "value_mlp_fwd")
    _check(lib.rag_value_mlp_bwd(_ptr(z), _ptr(W1), _ptr(W2), _ptr(b2), _ptr(hpre), _ptr(part),
                                 _ptr(y), _ptr(sw), _ptr(work), _ptr(loss), _ptr(vout),
                                 _ptr(dW1), _ptr(db1), _ptr(dW2), _ptr(db2), _ptr(dz), B, P, H,
                                 MLP_ACTS[act], stream), "value_mlp_bwd")
    return loss[:B]


def sample_moves(probs, mask, beta=1.0, greedy=None, seed=0, out=None, seed_dev=None):
    """Per row: a move drawn from probs^beta restricted to ``mask`` (uint8 [B, >=P]), or the
    masked argmax where ``greedy`` (uint8 [B]) is set; -1 for rows without candidates
    (sample.hip, Gumbel-max). Returns int32 [B] on the device. ``seed_dev`` (int64 [1] on the
    device, optional) is XORed into the seed when the kernel runs (captured graphs)."""
    B, P = probs.shape
    probs = probs.contiguous().float()
    mask = mask.reshape(B, -1)
    if mask.dtype != torch.uint8:
        mask = mask.to(torch.uint8)
    mask = mask.contiguous()
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=probs.device)
    _check(_lib().rag_sample_moves(_ptr(probs), _ptr(mask), mask.shape[1], _ptr(greedy), B, P,
                                   float(beta), int(seed) & ((1 << 64) - 1), _ptr(seed_dev),
                                   _ptr(out), _stream()), "sample_moves")
    return out


def sgd_(p, g, lr, momentum=0.0, v=None, wd=0.0, nesterov=False):
    """In-place Keras-style SGD on a flat fp32 buffer."""
    _check(_lib().rag_sgd(_ptr(p), _ptr(g), _ptr(v), p.numel(), float(lr), float(momentum),
                          float(wd), int(nesterov), _stream()), "sgd")
