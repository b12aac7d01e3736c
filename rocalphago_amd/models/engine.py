"""HIP network engine: the GPU execution path of the convolutional policy / value networks.

A ``HipTrunk`` executes a sequential stack of 'same' convolutions (+bias, optional ReLU) on
preallocated padded channels-last bf16 activations (layout: csrc/hip/conv.hip), with

  * forward    : one implicit-GEMM MFMA launch per layer (bias + ReLU fused in the epilogue);
                 3x3 192 -> 192 layers at full-chip batches: the Winograd F(2,3) kernel
                 (conv_wino.hip, 2/3 of the MFMA work) instead (and in dgrad when no deferred
                 wgrad reduction rides in it)
  * backward   : per layer one wgrad launch (+ slab reduce) and one dgrad launch whose epilogue
                 applies the ReLU derivative of the layer below (so no separate mask pass)
  * weights    : fp32 OIHW master parameters (views of one flat buffer owned by the model) are
                 repacked to the two bf16 GEMM layouts only when they change.

Heads: ``PolicyHeadEngine`` (1x1 conv -> per-position Bias -> softmax, with the cross-entropy /
REINFORCE loss fused into the same kernel) and ``ValueHeadEngine`` (1x1 conv on HIP, then the two
dense layers + tanh in csrc/hip/head.hip ``value_mlp_*`` for inference and csrc/hip/value_bwd.hip
for training: forward, MSE tail and all head gradients in two launches, no library GEMMs).

No autograd graph is built on the hot path; ``models/kerasish.py`` exposes these engines through
torch.autograd.Function wrappers for generic use and calls ``train_step`` directly for speed.
"""
import os

import torch

from ..ops import hipops as ops


class ConvSpec(object):
    __slots__ = ("ks", "cin", "cout", "relu", "cinp", "coutp", "halo_in", "bias")

    def __init__(self, ks, cin, cout, relu, bias=True):
        self.ks, self.cin, self.cout, self.relu, self.bias = ks, cin, cout, relu, bias
        self.cinp, self.coutp = ops.pad_channels(cin), ops.pad_channels(cout)
        self.halo_in = max(1, ks // 2)


def complement(ranges, n):
    """The [start, end) ranges of [0, n) that none of ``ranges`` covers, in order."""
    out, pos = [], 0
    for a, b in sorted(ranges) + [(n, n)]:
        if a > pos:
            out.append((pos, a))
        pos = max(pos, b)
    return out


def pack_grid_width(specs):
    """Grid width of the pack_trunk rows (csrc/hip/pack.h pack_trunk_block): the 16x16 (n, c)
    all-tap tiles of the widest layer, rounded up to a multiple of 8 (each block grid-strides over
    its layer's tiles)."""
    return max(8 * -(-((-(-s.coutp // 16)) * (-(-s.cinp // 16))) // 8) for s in specs)


class _PackedConvs(object):
    """bf16 GEMM layouts (+ padded fp32 biases) of a list of convolutions, repacked from the fp32
    OIHW masters in one launch whenever the model's weight version changes."""

    def _init_packing(self, specs, device, wino=None):
        # pack.h pack_trunk_block stages a 16x16 tile of all taps in LDS: kernels up to 7x7
        if any(s.ks > 7 for s in specs):
            raise ValueError("fused HIP trunks take kernels up to 7x7, got %s"
                             % sorted({s.ks for s in specs}))
        self._wf = [None] * len(specs)
        self._wb = [None] * len(specs)
        self._bias = [torch.zeros(s.coutp, device=device) for s in specs]
        self._packed_version = None
        # Winograd layers (conv_wino.hip): their fragment-major forward Winograd weights are
        # packed on every weight change, and either their dgrad Winograd weights (wino_dgrad) or
        # the direct dgrad layout; the direct forward layout only when a batch the Winograd
        # kernel does not take (conv_wino_prefer) needs it (_direct_layouts)
        self._wino = list(wino) if wino is not None else [False] * len(specs)
        self._uf = [None] * len(specs)
        self._ub = [None] * len(specs)
        self._direct_version = None
        self._ub_version = None
        self.wino_dgrad = False

    def sync_weights(self, weights, biases, version):
        """Repack bf16 GEMM layouts from fp32 OIHW masters when ``version`` changed."""
        if version == self._packed_version:
            return
        for l, s in enumerate(self.specs):
            taps = s.ks * s.ks
            if self._wf[l] is None:
                self._wf[l] = torch.empty((taps, s.coutp, s.cinp), dtype=torch.bfloat16,
                                          device=self.device)
                # the trunk input takes no gradient: layer 0 has no dgrad layout
                if l > 0:
                    self._wb[l] = torch.empty((taps, s.cinp, s.coutp), dtype=torch.bfloat16,
                                              device=self.device)
            if self._wino[l] and self._uf[l] is None:
                self._uf[l] = torch.empty((12, s.coutp, s.cinp), dtype=torch.bfloat16,
                                          device=self.device)
                if self.wino_dgrad:
                    self._ub[l] = torch.empty((12, s.cinp, s.coutp), dtype=torch.bfloat16,
                                              device=self.device)
        # one launch repacks all layers (GEMM layouts + padded biases; Winograd layers: their
        # Winograd weights, bias in the pack_trunk rows); the pointer tables are rebuilt only
        # when a parameter tensor moved
        ws = [w.contiguous() for w in weights]
        key = tuple(w.data_ptr() for w in ws) + \
            tuple(0 if b is None else b.data_ptr() for b in biases)
        if getattr(self, "_pack_key", None) != key:
            rows, drows, wrows, start = [], [], [], 0
            for l, s in enumerate(self.specs):
                b = biases[l]
                wbp = 0 if self._wb[l] is None else self._wb[l].data_ptr()
                row = [ws[l].data_ptr(), 0 if b is None else b.data_ptr(), s.cout, s.cin, s.ks,
                       s.coutp, s.cinp, self._wf[l].data_ptr(), wbp,
                       self._bias[l].data_ptr(), start]
                start += s.ks * s.ks * s.coutp * s.cinp + s.coutp
                if self._wino[l]:
                    drows.append(row)
                    ub = self._ub[l].data_ptr() if self.wino_dgrad else 0
                    # the direct dgrad layout (unless the dgrad runs Winograd too) comes out of
                    # wino_pack's tiles: the pack_trunk row keeps only the bias
                    wd = 0 if self.wino_dgrad else wbp
                    wrows.append([ws[l].data_ptr(), s.cout, s.cin, s.coutp, s.cinp,
                                  self._uf[l].data_ptr(), ub, wd])
                    row = row[:7] + [0, 0] + row[9:]
                rows.append(row)
            # the rows that pack weights first; the bias-only rows share one grid row
            full = [l for l, r in enumerate(rows) if r[7] or r[8]]
            rows = [rows[l] for l in full] + [r for r in rows if not (r[7] or r[8])]
            self._pack_nfull = len(full)
            self._pack_table = torch.tensor(rows, dtype=torch.int64).to(self.device)
            self._pack_total = pack_grid_width([self.specs[l] for l in full]) if full else 8
            self._pack_taps = max([self.specs[l].ks ** 2 for l in full] or [1])
            wsp = [s for l, s in enumerate(self.specs) if self._wino[l]]
            if wsp:
                self._dpack_table = torch.tensor(drows, dtype=torch.int64).to(self.device)
                self._dpack_total = pack_grid_width(wsp)
                self._wpack_table = torch.tensor(wrows, dtype=torch.int64).to(self.device)
                self._wpack_tiles = max(-(-s.coutp // 64) * -(-s.cinp // 64) for s in wsp)
            self._pack_key = key
            self._pack_keep = ws  # keep contiguous copies alive while the table points at them
        self._launch_pack()
        self._packed_version = version
        # once any batch has run a Winograd layer on the direct kernel, its direct layout stays
        # fresh on every weight change: a captured graph replayed after sync_weights() never
        # re-enters wino_plan() (the Python forward that would repack it lazily)
        if self._direct_version is not None:
            self._direct_layouts()

    # ONE_LAUNCH: the repack (+ folded optimizer step) of all layers in one pack_step launch;
    # False: the separate wino_pack + pack_trunk (+ sgd_kernel) launches (the A/B)
    ONE_LAUNCH = True

    def _launch_pack(self, sgd=None, flat=None, rest=()):
        """Repack every layer from its fp32 master (with ``sgd``: stepped first, and the
        ``rest`` ranges of ``flat`` stepped by plain SGD in the same launch; ONE_LAUNCH only)."""
        wino = sum(self._wino)
        if self.ONE_LAUNCH:
            width = max(8 * self._wpack_tiles, self._pack_total) if wino else self._pack_total
            ops.pack_step(self._wpack_table if wino else None, wino, self._pack_table,
                          len(self.specs), self._pack_nfull, self._pack_taps, width, sgd=sgd,
                          flat=flat, rest=rest)
            return
        if wino:
            ops.wino_pack(self._wpack_table, wino, self._wpack_tiles, sgd=sgd)
        ops.pack_trunk(self._pack_table, len(self.specs), self._pack_total, self._pack_nfull,
                       sgd=sgd)

    def sgd_pack(self, weights, biases, flat, flat_grad, lr, version, max_gaps=None,
                 step_rest=False):
        """The optimizer step of this trunk's parameters folded into their repacking (round 6:
        pack_trunk + wino_pack re-read the fp32 masters right after sgd_kernel had): wino_pack
        and pack_trunk read each master and its gradient once, write back w - lr g and pack
        that. Returns the [start, end) element ranges of ``flat`` it stepped (the caller steps
        the rest), or None when the packing tables do not point into ``flat`` or the rest of
        ``flat`` would take more than ``max_gaps`` separate ranges (then nothing was done).
        ``step_rest``: the rest too, in the same launch, when it is at most two ranges (the
        returned ranges then cover all of ``flat``)."""
        if self._packed_version is None or getattr(self, "_pack_key", None) is None:
            return None
        ws = [w.contiguous() for w in weights]
        key = tuple(w.data_ptr() for w in ws) + \
            tuple(0 if b is None else b.data_ptr() for b in biases)
        if key != self._pack_key:
            return None
        base, esz = flat.data_ptr(), flat.element_size()
        end = base + flat.numel() * esz
        ranges = []
        for t in list(weights) + [b for b in biases if b is not None]:
            p = t.data_ptr()
            if not t.is_contiguous() or p < base or p + t.numel() * esz > end:
                return None
            ranges.append(((p - base) // esz, (p - base) // esz + t.numel()))
        if flat_grad.numel() != flat.numel():
            return None
        if max_gaps is not None and len(complement(ranges, flat.numel())) > max_gaps:
            return None
        sgd = ((flat_grad.data_ptr() - base) // esz, lr, 0.0)
        rest = complement(ranges, flat.numel()) if step_rest and self.ONE_LAUNCH else []
        if len(rest) > 2:
            rest = []
        self._launch_pack(sgd=sgd, flat=flat, rest=rest)
        ranges = ranges + rest
        self._packed_version = version
        if self._direct_version is not None:
            self._direct_layouts()
        return ranges

    def _dgrad_wino_layouts(self):
        """Winograd dgrad weights of the Winograd layers when the dgrad normally runs the direct
        kernel (a large batch takes Winograd, see HipTrunk.backward): packed once per weight
        version, on first use."""
        if self.wino_dgrad or self._ub_version == self._packed_version:
            return
        if getattr(self, "_ubpack_table", None) is None or self._ubpack_key != self._pack_key:
            rows = []
            for l, s in enumerate(self.specs):
                if not self._wino[l]:
                    continue
                if self._ub[l] is None:
                    self._ub[l] = torch.empty((12, s.cinp, s.coutp), dtype=torch.bfloat16,
                                              device=self.device)
                rows.append([self._pack_keep[l].data_ptr(), s.cout, s.cin, s.coutp, s.cinp, 0,
                             self._ub[l].data_ptr(), 0])
            self._ubpack_table = torch.tensor(rows, dtype=torch.int64).to(self.device)
            self._ubpack_key = self._pack_key
        ops.wino_pack(self._ubpack_table, sum(self._wino), self._wpack_tiles)
        self._ub_version = self._packed_version

    def _direct_layouts(self):
        """Direct GEMM layouts of the Winograd layers, for a batch that runs them on the direct
        kernel: packed once per weight version, on first use."""
        if self._direct_version != self._packed_version:
            ops.pack_trunk(self._dpack_table, sum(self._wino), self._dpack_total)
            self._direct_version = self._packed_version


class HipTrunk(_PackedConvs):
    # wgrad slab reductions ride along the next dgrad launch (False: their own reduce kernels,
    # and the dgrads of the Winograd layers run Winograd too)
    DEFER_REDUCE = True

    def __init__(self, specs, board, device):
        assert specs, "empty trunk"
        self.specs = specs
        self.S = board
        self.device = device
        self.L = len(specs)
        for a, b in zip(specs[:-1], specs[1:]):
            assert a.cout == b.cin, "channel mismatch in trunk"
        self._B = 0
        self.acts = []
        self._gbufs = {}
        # 3x3 192 -> 192 layers run the Winograd F(2,3) kernel (conv_wino.hip) forward at
        # batches that fill its grid (RAG_WINO=0: direct kernel only)
        wino_on = device.type == "cuda" and os.environ.get("RAG_WINO", "1") != "0"
        wino = [wino_on and s.ks == 3 and ops.conv_wino_ok(board, 1, s.cinp, s.coutp, 3)
                and ops.conv_wino_ok(board, 1, s.coutp, s.cinp, 3) for s in specs]
        self._init_packing(specs, device, wino)
        self._wino_plans = {}
        # half-board Winograd blocks at every batch (a search whose GPU rollouts share the chip
        # may set it)
        self.wino_half = False
        self._work = None
        self.defer_reduce = self.DEFER_REDUCE
        # The dgrad of a Winograd layer runs the direct kernel while it carries a deferred
        # reduction: the Winograd grid is exactly one wave of blocks (one per CU), so the
        # reduction's ~28 MB of partial slabs stream after every block's epilogue (+6-8 us in
        # the step), while the direct kernel's ragged last wave absorbs them (+1-2 us); without
        # deferral (own reduce kernels) the dgrad runs Winograd as well. (Overlapping the
        # reductions with the dgrad on a second stream measured slower, 78.1k vs 80.8k
        # positions/s, and was deleted in round 6: docs/KERNELS.md.)
        self.wino_dgrad = not self.defer_reduce
        self.wino_dgrad_min_batch = 512
        self._pending = ops.PendingReduction() if device.type == "cuda" else None

    # ------------------------------------------------------------------ buffers
    def _halos(self):
        """halo[b] of activation boundary b: the smallest halo layer b's kernel needs (1 for
        1x1/3x3, 2 for the 5x5 input layer); the trunk output (read by the heads) has halo 1.

        The gradient g_l (w.r.t. layer l's pre-activation) is stored with the halo of layer l's
        INPUT, halo[l], not of its output: then G and X of layer l's wgrad share one padded
        geometry and the all-taps wgrad kernel (wgrad.hip) applies to every layer. The dgrad
        that produces g_{l-1} reads its ReLU mask (acts[l]) with that tensor's own halo."""
        sp = self.specs
        h = [max(1, s.ks // 2) for s in sp]
        assert sp[-1].ks <= 3, "last trunk layer must be 1x1 or 3x3 (heads read halo 1)"
        h.append(1)
        return h

    def ensure_batch(self, B):
        if B <= self._B:
            return
        self.gen = getattr(self, "gen", 0) + 1  # buffers moved (captured graphs)
        B = max(B, 1)
        S = self.S
        self.halo = self._halos()
        acts = [ops.alloc_padded(B, S, self.halo[0], self.specs[0].cinp, self.device)]
        for l, s in enumerate(self.specs):
            acts.append(ops.alloc_padded(B, S, self.halo[l + 1], s.coutp, self.device))
        self.acts = acts
        self._gbufs = {}
        for l, s in enumerate(self.specs):
            key = (s.coutp, self.halo[l])
            if key not in self._gbufs:
                self._gbufs[key] = [ops.alloc_padded(B, S, key[1], key[0], self.device)
                                    for _ in range(2)]
        self._B = B
        need = 0
        for s in self.specs:
            need = max(need, ops._lib().rag_conv_wgrad_workspace(B, S, s.coutp, s.cinp, s.ks,
                                                                 None))
        self._work = torch.empty(need + 1024, dtype=torch.float32, device=self.device)

    def input_buffer(self, B):
        self.ensure_batch(B)
        return self.acts[0][:B]

    def output(self, B):
        return self.acts[-1][:B]

    def grad_buffer(self, l, which, B):
        """g_l = dL/d(pre-activation of layer l), stored with the halo of layer l's input."""
        s = self.specs[l]
        return self._gbufs[(s.coutp, self.halo[l])][which][:B]

    # ------------------------------------------------------------------ compute
    @property
    def top_relu(self):
        return self.specs[-1].relu

    def top_grad(self, B):
        """Where the head writes dL/d(trunk output) (ReLU-masked if top_relu)."""
        return self.grad_buffer(self.L - 1, 0, B)

    def wino_plan(self, B):
        """Per layer: True if it runs the Winograd kernel at batch B (forward and dgrad)."""
        plan = self._wino_plans.get(B)
        if plan is None:
            plan = [w and ops.conv_wino_prefer(B, self.S, s.cinp, s.coutp)
                    for w, s in zip(self._wino, self.specs)]
            self._wino_plans[B] = plan
        if any(w and not p for w, p in zip(self._wino, plan)):
            self._direct_layouts()
        return plan

    def forward(self, B, training=False):
        S = self.S
        wino = self.wino_plan(B)
        for l, s in enumerate(self.specs):
            x, y = self.acts[l][:B], self.acts[l + 1][:B]
            if wino[l]:
                ops.conv_wino(x, self._uf[l], self._bias[l], y, B, S, s.cinp, s.coutp,
                              self.halo[l + 1], s.relu, half=self.wino_half)
            else:
                ops.conv_igemm(x, self._wf[l], self._bias[l], y, B, S, self.halo[l],
                               self.halo[l + 1], s.cinp, s.coutp, s.ks, s.relu, cin=s.cin)
        return self.acts[-1][:B]

    def backward(self, B, dws, dbs, top_which=0, accumulate=False, on_layer_done=None):
        """Backprop from grad_buffer(L-1, top_which) (= dL/d pre-activation of the last layer,
        already ReLU-masked) down to the first layer; writes fp32 OIHW grads into dws/dbs.
        ``on_layer_done(l)`` fires right after layer l's wgrad is queued (DP bucket overlap)."""
        S = self.S
        which = top_which
        wino = self.wino_plan(B)
        for l in range(self.L - 1, -1, -1):
            s = self.specs[l]
            g = self.grad_buffer(l, which, B)
            x = self.acts[l][:B]
            # layer l's slab reduction is deferred into the free block slots of its own dgrad
            # launch (this trunk's PendingReduction handle, passed to that launch explicitly);
            # dW[l] is final after that
            defer = self.defer_reduce
            ops.conv_wgrad(g, x, dws[l], dbs[l], B, S, self.halo[l], s.cout, s.coutp, s.cin,
                           s.cinp, s.ks, accumulate=accumulate, work=self._work,
                           hg=self.halo[l], defer=defer,
                           pending=self._pending if defer else None)
            if l > 0:
                below = self.specs[l - 1]
                which ^= 1
                gout = self.grad_buffer(l - 1, which, B)
                # batches of two or more block waves (the RL learner's 8192-position chunks) run
                # the dgrad on Winograd too: a riding reduction costs a few us there, not a wave
                big = wino[l] and not self.wino_dgrad and B >= self.wino_dgrad_min_batch
                if big:
                    self._dgrad_wino_layouts()
                if wino[l] and (self.wino_dgrad or big):
                    ops.conv_wino(g, self._ub[l], None, gout, B, S, s.coutp, s.cinp,
                                  self.halo[l - 1], False, mask=x if below.relu else None,
                                  mask_halo=self.halo[l],
                                  pending=self._pending if defer else None)
                else:
                    ops.conv_igemm(g, self._wb[l], None, gout, B, S, self.halo[l],
                                   self.halo[l - 1], s.coutp, s.cinp, s.ks, False,
                                   mask=x if below.relu else None, mask_halo=self.halo[l],
                                   pending=self._pending if defer else None)
            elif defer:
                ops.wgrad_flush(self._pending)
            if on_layer_done is not None:
                on_layer_done(l)
        if self.defer_reduce:
            ops.wgrad_flush(self._pending)


class BNSpec(object):
    """One column BatchNormalization (Keras-1 axis=-1 on (B, C, H, W) tensors: S statistics)."""
    __slots__ = ("eps", "momentum", "gamma", "beta", "rmean", "rvar", "dgamma", "dbeta")

    def __init__(self, eps, momentum, params, grads):
        self.eps, self.momentum = eps, momentum
        self.gamma, self.beta, self.rmean, self.rvar = params
        self.dgamma, self.dbeta = grads[0], grads[1]


class ResTrunk(_PackedConvs):
    # 3x3 128 -> 128 layers whose input BN is fused run the Winograd BN kernel: "0" off, "1"
    # forward only (default), "2" forward and dgrad (see __init__)
    WINO_MODE = "1"
    DEFER_REDUCE = True

    """Residual trunk of ResnetPolicy (reference policy.py:196-244) on the HIP engine:

        A_0 = conv0(x)                                       (linear, 5x5 by default)
        unit u: X = A_u; n_skip x [U = ReLU(BN(X)); X = conv(U)]; A_{u+1} = A_u + X
        H = ReLU(A_U)                                        (read by the policy head)

    Forward: the column BN statistics (summed in the epilogue of the fused conv that produced
    the BN input, else a bn.hip pass) + a finalize launch, then BN+ReLU fused into the next
    conv's prologue (the ping-pong kernel stages the BN input x and turns it into U while
    staging; ``_prologue_ok``) or, for shapes without that kernel (5x5, small batches), one BN+ReLU
    pass; the MFMA conv adds the residual in its epilogue (conv.hip ``res``). Backward, per conv:
    wgrad (fused layers rebuild U from x while staging), dgrad with the ReLU mask of U in the
    epilogue (fused: recomputed from x, and the BN backward sums taken in the same epilogue),
    then the BN backward (reduction unless fused + one elementwise pass that also adds the skip
    gradient, in place when the halos agree).

    Halos: A_u / X / H use halo 1. U_j (conv l = j+1's input) and every gradient consumed by
    conv l use halo hin[l] = max(1, ks_l // 2), so wgrad always runs the all-taps kernel and the
    dgrad input is wide enough (the reference's filter_width_1 also sets the FIRST unit's conv,
    5x5 by default). Memory: (units + BNs + ~4) activations of B x (S+2)^2 x K bf16 (29 MB each
    at B=256, K=128) — trivial against 288 GB of HBM."""

    def __init__(self, specs, units, bns, board, device):
        assert specs and len(specs) == 1 + sum(units) == 1 + len(bns)
        self.specs, self.units, self.bns = specs, list(units), bns
        self.S = board
        self.device = device
        self.L = len(specs)
        K = specs[0].cout
        for s in specs[1:]:
            assert s.cin == K and s.cout == K, "residual trunk needs constant width"
        self.K, self.KP = K, specs[0].coutp
        self._B = 0
        # 3x3 128 -> 128 layers whose input BN is fused (_prologue_ok) run the Winograd kernel
        # with the BN built into its input transform (conv_wino.hip WinoBN) at batches that fill
        # its grid; WINO_MODE: 0 off, 1 (default) forward only, 2 forward and dgrad. The dgrad
        # carries the deferred wgrad reduction: one wave of Winograd blocks pays for it in full
        # (51.6 vs 48.6 us on the direct kernel; standalone it is 37.4 us + a 16.6 us reduction,
        # and riding in the BN backward apply made that pass 47.9 instead of 18.5 us). ResNet
        # 71.6 k (1) / 70.9 k (2) / 69.7 k (2, no deferral) / 68.0 k (0) positions/s on one box.
        mode = str(self.WINO_MODE) if device.type == "cuda" else "0"
        wino = [mode != "0" and l > 0 and s.ks == 3 and s.cinp == s.coutp == 128
                and ops.conv_wino_ok(board, 1, s.cinp, s.coutp, 3) for l, s in enumerate(specs)]
        self._init_packing(specs, device, wino)
        self.wino_dgrad = mode == "2"
        self._wino_plans = {}
        self.hin = [max(1, s.ks // 2) for s in specs]
        self.halo = [self.hin[0]]
        # last conv of each unit, and the gradient halo each unit's output gradient needs
        ends, j = [], 0
        for n in self.units:
            j += n
            ends.append(j)
        self._unit_last = ends
        self._work = None
        # 3x3 wgrad slab reductions ride along the dgrad launch that follows them (as HipTrunk)
        self.defer_reduce = self.DEFER_REDUCE
        self._pending = ops.PendingReduction() if device.type == "cuda" else None
        self.bn_prologue = True
        # fused BNs: the backward finalize folded into the apply (False: two launches)
        self.fold_bwd_finalize = self.S <= 32
        self._fused = []  # per BN: fused into the next conv on the last forward

    # ------------------------------------------------------------------ buffers
    def ensure_batch(self, B):
        if B <= self._B:
            return
        self.gen = getattr(self, "gen", 0) + 1  # buffers moved (captured graphs)
        B = max(B, 1)
        S, KP, dev = self.S, self.KP, self.device
        alloc = ops.alloc_padded
        self.xin = alloc(B, S, self.hin[0], self.specs[0].cinp, dev)
        self.A = [alloc(B, S, 1, KP, dev) for _ in range(len(self.units) + 1)]
        nb = len(self.bns)
        self.U = [alloc(B, S, self.hin[j + 1], KP, dev) for j in range(nb)]
        # inner conv outputs of units with n_skip > 1 (BN j's input when it is not A_u)
        self.Xin = [None] * nb
        inner_h = set()
        j = 0
        for n in self.units:
            for i in range(1, n):
                self.Xin[j + i] = alloc(B, S, 1, KP, dev)
                inner_h.add(self.hin[j + i])
            j += n
        self.H = alloc(B, S, 1, KP, dev)
        self.G = {h: alloc(B, S, h, KP, dev) for h in set(self.hin) | {1}}
        self.gI = {h: alloc(B, S, h, KP, dev) for h in inner_h}
        self.dU = alloc(B, S, 1, KP, dev)
        self.stats = torch.zeros((nb, 2, S), dtype=torch.float32, device=dev)
        self.coef = torch.zeros((nb, 3, S), dtype=torch.float32, device=dev)
        self.bcoef = torch.zeros((3, S), dtype=torch.float32, device=dev)
        # BN column-statistics partials written by the fused conv epilogues (forward: one per
        # BN, whose input that conv produced; backward: one, reused layer by layer)
        # (the Winograd kernel writes one partial per board)
        nblk = max(ops.conv_bn_stat_blocks(B, S, KP), B) if KP % 128 == 0 and KP % 192 else 1
        self.spart = torch.zeros((nb, nblk, 2, S), dtype=torch.float32, device=dev)
        self.bpart = torch.zeros((nblk, 2, S), dtype=torch.float32, device=dev)
        need = max(ops._lib().rag_conv_wgrad_workspace(B, S, s.coutp, s.cinp, s.ks, None)
                   for s in self.specs)
        self._work = torch.empty(need + 1024, dtype=torch.float32, device=dev)
        self._B = B

    def input_buffer(self, B):
        self.ensure_batch(B)
        return self.xin[:B]

    def output(self, B):
        return self.H[:B]

    top_relu = True

    def top_grad(self, B):
        return self.G[1][:B]

    def _bn_input(self, j, u, B):
        return self.A[u][:B] if self.Xin[j] is None else self.Xin[j][:B]

    def _prologue_ok(self, j, B):
        """BN j + ReLU fused into conv j+1 (conv prologue): that conv stages the BN
        input x and applies U = ReLU(cx[col] x + cc[col]) while staging, its wgrad does the same,
        and its dgrad recomputes the ReLU mask from x; U is never materialised. Needs the
        128-channel ping-pong / slab kernels (3x3, unpadded width, a grid that fills the chip);
        other layers keep the bn_apply pass. bn_prologue = False disables it."""
        sp = self.specs[j + 1]
        return (self.bn_prologue and sp.ks == 3 and self.hin[j + 1] == 1 and self.K == self.KP
                and ops.conv_bn_fusable(B, self.S, 1, sp.cinp, sp.coutp, sp.ks))

    def _plan(self, B):
        """(fused, wino) at batch B: per BN j, fused into conv j+1's prologue; per conv l, runs
        the Winograd BN kernel (its input BN fused, a grid that fills the chip)."""
        plan = self._wino_plans.get(B)
        if plan is None:
            fused = [self._prologue_ok(j, B) for j in range(len(self.bns))]
            wino = [w and l > 0 and fused[l - 1] and ops.conv_wino_bn_ok(B, self.S, self.KP,
                                                                         self.KP)
                    for l, w in enumerate(self._wino)]
            plan = self._wino_plans[B] = (fused, wino)
        if any(w and not p for w, p in zip(self._wino, plan[1])):
            self._direct_layouts()
        return plan

    def _stat_blocks(self, l, B, dgrad=False):
        """Partial rows of the BN statistics conv l's forward (or dgrad) epilogue writes."""
        wino = self._plan(B)[1][l] and (self.wino_dgrad or not dgrad)
        return B if wino else ops.conv_bn_stat_blocks(B, self.S, self.KP)

    # ------------------------------------------------------------------ compute
    def forward(self, B, training=False):
        S, K = self.S, self.K
        s0 = self.specs[0]
        ops.conv_igemm(self.xin[:B], self._wf[0], self._bias[0], self.A[0][:B], B, S,
                       self.hin[0], 1, s0.cinp, s0.coutp, s0.ks, False, cin=s0.cin)
        j = 0
        nb = len(self.bns)
        fused, wino = self._plan(B)
        self._fused = list(fused)
        stat_ready = [False] * nb  # BN j's input statistics came out of the conv producing it
        for u, n in enumerate(self.units):
            for i in range(n):
                bn, x, U = self.bns[j], self._bn_input(j, u, B), self.U[j][:B]
                if training and stat_ready[j]:
                    ops.bn_finalize_fwd(self.spart[j], self._stat_blocks(j, B), B, S, K,
                                        bn.gamma, bn.beta,
                                        bn.rmean, bn.rvar, bn.eps, bn.momentum, self.stats[j],
                                        self.coef[j])
                elif training:
                    ops.bn_train_fwd(x, B, S, K, bn.gamma, bn.beta, bn.rmean, bn.rvar, bn.eps,
                                     bn.momentum, self.stats[j], self.coef[j])
                else:
                    ops.bn_infer_coef(bn.gamma, bn.beta, bn.rmean, bn.rvar, bn.eps, S,
                                      self.coef[j])
                l, sp = j + 1, self.specs[j + 1]
                last = i == n - 1
                y = self.A[u + 1][:B] if last else self.Xin[j + 1][:B]
                res = self.A[u][:B] if last else None
                if self._fused[j]:
                    # this conv's output is BN l's input: its epilogue also sums BN l's stats
                    sp_out = self.spart[l] if training and l < nb else None
                    if wino[l]:
                        ops.conv_wino_bn(x, self._uf[l], self._bias[l], y, B, S, sp.cinp,
                                         sp.coutp, False, bn_coef=self.coef[j], residual=res,
                                         stat_part=sp_out)
                    else:
                        ops.conv_igemm_bn(x, self._wf[l], self._bias[l], y, B, S, sp.cinp,
                                          sp.coutp, False, bn_coef=self.coef[j], residual=res,
                                          stat_part=sp_out)
                    if sp_out is not None:
                        stat_ready[l] = True
                else:
                    ops.bn_apply(x, U, B, S, K, coef=self.coef[j], relu=True)
                    ops.conv_igemm(U, self._wf[l], self._bias[l], y, B, S, self.hin[l], 1,
                                   sp.cinp, sp.coutp, sp.ks, False, residual=res)
                j += 1
        ops.bn_apply(self.A[-1][:B], self.H[:B], B, S, K, coef=None, relu=True)
        return self.H[:B]

    def backward(self, B, dws, dbs, top_which=0, accumulate=False, on_layer_done=None):
        """Backprop from top_grad (dL/dA_U, already ReLU-masked by the head) to conv0; writes
        conv grads into dws/dbs and BN grads into each BNSpec's dgamma/dbeta (batch-statistics
        BN, i.e. the training learning phase). ``on_layer_done(l)`` fires after conv l's wgrad
        (BN j's grads, which sit between conv j and conv j+1 in the flat buffer, are complete
        by then)."""
        S, K = self.S, self.K
        wino = self._plan(B)[1]
        cur, hcur = self.G[1][:B], 1  # dL/dA_{u+1}
        for u in range(len(self.units) - 1, -1, -1):
            n, jend = self.units[u], self._unit_last[u]
            need = self.hin[jend]
            if hcur != need:  # only the top unit (the head writes halo 1): re-pad once
                ops.bn_apply(cur, self.G[need][:B], B, S, K, coef=None, relu=False)
                cur, hcur = self.G[need][:B], need
            gx = cur
            for i in range(n - 1, -1, -1):
                j = jend - n + i
                l, sp, bn = j + 1, self.specs[j + 1], self.bns[j]
                U, x = self.U[j][:B], self._bn_input(j, u, B)
                defer = self._pending is not None and self.defer_reduce
                fused = self._fused[j] if j < len(self._fused) else False
                dU = self.dU[:B]
                if fused:  # U never stored: both kernels rebuild it from x and BN j's coefs
                    ops.conv_wgrad(gx, x, dws[l], dbs[l], B, S, 1, sp.cout, sp.coutp, sp.cin,
                                   sp.cinp, sp.ks, accumulate=accumulate, work=self._work, hg=1,
                                   defer=defer, pending=self._pending if defer else None,
                                   xcoef=self.coef[j])
                    # its epilogue also sums BN j's backward statistics (dU, dU (x - mean))
                    if wino[l] and self.wino_dgrad:
                        ops.conv_wino_bn(gx, self._ub[l], None, dU, B, S, sp.coutp, sp.cinp,
                                         False, mask=x, mask_coef=self.coef[j],
                                         pending=self._pending if defer else None,
                                         stat_part=self.bpart, stat_mean=self.stats[j])
                    else:
                        ops.conv_igemm_bn(gx, self._wb[l], None, dU, B, S, sp.coutp, sp.cinp,
                                          False, mask=x, mask_coef=self.coef[j],
                                          pending=self._pending if defer else None,
                                          stat_part=self.bpart, stat_mean=self.stats[j])
                else:
                    ops.conv_wgrad(gx, U, dws[l], dbs[l], B, S, self.hin[l], sp.cout, sp.coutp,
                                   sp.cin, sp.cinp, sp.ks, accumulate=accumulate,
                                   work=self._work, hg=self.hin[l], defer=defer,
                                   pending=self._pending if defer else None)
                    # the dgrad runs the pending slab reduction in its free block slots: dW[l]
                    # is final after it
                    ops.conv_igemm(gx, self._wb[l], None, dU, B, S, self.hin[l], 1, sp.coutp,
                                   sp.cinp, sp.ks, False, mask=U, mask_halo=self.hin[l],
                                   pending=self._pending if defer else None)
                # i > 0: gradient of the inner conv output Xin[j] = conv j's gx; i == 0:
                # dL/dA_u = BN'(dU) + skip gradient (in place when halos agree)
                if i > 0:
                    out, res = self.gI[self.hin[j]][:B], None
                else:
                    hn = self.hin[self._unit_last[u - 1]] if u > 0 else self.hin[0]
                    out, res = self.G[hn][:B], cur
                if fused and self.fold_bwd_finalize:
                    # the finalize folded into the apply (each block sums the dgrad's partials)
                    ops.bn_apply_bwd_part(self.bpart, self._stat_blocks(l, B, True), x,
                                          out, B, S, K, bn.gamma, self.stats[j], bn.dgamma,
                                          bn.dbeta, dU, residual=res)
                else:
                    if fused:
                        ops.bn_finalize_bwd(self.bpart, self._stat_blocks(l, B, True),
                                            B, S, K, bn.gamma, self.stats[j], bn.dgamma,
                                            bn.dbeta, self.bcoef)
                    else:
                        ops.bn_bwd_coef(x, dU, B, S, K, bn.gamma, self.stats[j], bn.dgamma,
                                        bn.dbeta, self.bcoef)
                    ops.bn_apply(x, out, B, S, K, coef=self.bcoef, relu=False, dy=dU,
                                 residual=res)
                if on_layer_done is not None:  # dW[l] final (its reduction ran by now)
                    on_layer_done(l)
                if i > 0:
                    gx = out
                else:
                    cur, hcur = out, hn
        s0 = self.specs[0]
        ops.conv_wgrad(cur, self.xin[:B], dws[0], dbs[0], B, S, self.hin[0], s0.cout,
                       s0.coutp, s0.cin, s0.cinp, s0.ks, accumulate=accumulate, work=self._work,
                       hg=self.hin[0])
        if self._pending is not None:
            ops.wgrad_flush(self._pending)
        if on_layer_done is not None:
            on_layer_done(0)


class PolicyHeadEngine(object):
    """1x1 conv (K->1, scalar bias) -> Flatten -> per-position Bias -> softmax."""

    def __init__(self, trunk, K, pass_logit=False):
        self.trunk = trunk
        self.K = K
        self.S = trunk.S
        self.pass_logit = pass_logit
        self._B = 0

    def ensure(self, B):
        if B <= self._B:
            return
        self.gen = getattr(self, "gen", 0) + 1  # buffers moved (captured graphs)
        dev = self.trunk.device
        S2 = self.S * self.S
        self.probs = torch.empty((B, S2 + (1 if self.pass_logit else 0)), device=dev)
        self.dz = torch.empty((B, S2), device=dev)
        self.loss = torch.empty((B,), device=dev)
        self.hit = torch.empty((B,), device=dev)
        self.dzsum = torch.empty((B,), device=dev)
        if self.pass_logit:
            self.zpos = torch.empty((B, S2), device=dev)
            self.dpass = torch.empty((B,), device=dev)
        self._B = B

    def forward(self, B, w, b0, pbias, labels=None, sweight=None, mode=0, gscale=1.0,
                pass_params=None, acc=None):
        """pass_params: (W [S*S], b [1]) of a PassLogit layer, or None. acc: fp32 [2] running
        (loss sum, hit count). In a training forward (mode > 0) the sums are added by the
        matching backward() (its reduce launch sums the per-board loss / hit arrays), so every
        training forward that passes ``acc`` must be followed by backward() before the next
        one; a second such forward raises instead of silently dropping the first's metrics."""
        if mode and acc is not None and getattr(self, "_macc", None) is not None:
            raise RuntimeError("PolicyHeadEngine: training forward with acc= while the previous "
                               "one's metrics are still pending (backward() not called)")
        self.ensure(B)
        h = self.trunk.output(B)
        pk = {}
        if pass_params is not None:
            pk = dict(pass_w=pass_params[0], pass_b=pass_params[1], zout=self.zpos[:B],
                      dpass=self.dpass[:B] if mode else None)
        # running metrics: summed by the backward's reduce launch from the per-board loss / hit
        # (acc in the forward kernel meant two contended device atomics per board)
        # (set only once the launch succeeded: a failed forward leaves nothing pending)
        self._macc = None
        ops.policy_head_fwd(h, w, b0, pbias, self.probs[:B], self.K, labels=labels,
                            sweight=sweight, loss=self.loss[:B] if mode else None,
                            dz=self.dz[:B] if mode else None, hit=self.hit[:B] if mode else None,
                            mode=mode, gscale=gscale, acc=None if mode else acc,
                            dzsum=self.dzsum[:B] if (mode and not pk) else None, **pk)
        self._macc = acc if mode else None
        self._dzsum = bool(mode and not pk)
        return self.probs[:B]

    def reset_metrics(self):
        """Drop a training forward's pending metrics (a caller that recovers from an error
        raised between forward() and backward())."""
        self._macc = None

    def pass_grads(self, B, dW, db):
        """PassLogit weight gradients after a training forward: dW = dpass^T z, db = sum dpass
        (head.hip pass_grads_kernel)."""
        ops.pass_grads(self.zpos[:B], self.dpass[:B], dW, db)

    def backward(self, B, w, dz, dw, db0, dpbias):
        """dz [B, S*S] -> head param grads + trunk top gradient (ReLU-masked) in grad buffer 0."""
        h = self.trunk.output(B)
        acc, self._macc = getattr(self, "_macc", None), None
        ops.head_bwd(h, w, dz, self.trunk.top_grad(B), dw, db0, dpbias, self.K,
                     relu_mask=self.trunk.top_relu,
                     metrics=(self.loss[:B], self.hit[:B], acc) if acc is not None else None,
                     dzsum=self.dzsum[:B] if getattr(self, "_dzsum", False) else None)


class ValueHeadEngine(object):
    """1x1 conv (K->1) on HIP; Dense(S*S->H) + act; Dense(H->1) + tanh: inference through the
    fused value_mlp_fwd HIP kernel (fused.ValuePlan.forward), training through
    ops.value_mlp_train (head.hip + value_bwd.hip: loss and every head gradient on HIP)."""

    def __init__(self, trunk, K):
        self.trunk = trunk
        self.K = K
        self.S = trunk.S
        self._B = 0

    def ensure(self, B):
        if B <= self._B:
            return
        self.gen = getattr(self, "gen", 0) + 1  # buffers moved (captured graphs)
        self.z = torch.empty((B, self.S * self.S), device=self.trunk.device)
        self.dz = torch.empty((B, self.S * self.S), device=self.trunk.device)
        self._B = B

    def dz_buffer(self, B):
        self.ensure(B)
        return self.dz[:B]

    def conv_out(self, B, w, b0):
        self.ensure(B)
        ops.head_linear(self.trunk.output(B), w, b0, self.z[:B], self.K)
        return self.z[:B]

    def backward_conv(self, B, w, dz, dw, db0):
        h = self.trunk.output(B)
        ops.head_bwd(h, w, dz.contiguous(), self.trunk.top_grad(B), dw, db0, None, self.K,
                     relu_mask=self.trunk.top_relu)
