"""ResnetPolicy on the HIP engine (bn.hip column BatchNorm, residual conv epilogue, ResnetPlan)
against plain PyTorch fp32 references: the kernels one by one, then the whole fused plan against
the generic executor (reference policy.py:141-271; Keras-1 BN axis=-1 on 'th' tensors)."""
import numpy as np

from rocalphago_amd.models.engine import ResTrunk
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.ops import hipops
    return hipops


def col_bn_ref(x, gamma, beta, eps):
    """Keras-1 BN over axis=-1 of (B, C, H, W): one statistic per column w."""
    mean = x.mean(dim=(0, 1, 2))
    var = x.var(dim=(0, 1, 2), unbiased=False)
    return (x - mean) / torch.sqrt(var + eps) * gamma + beta, mean, var


def bfr(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("B,C,S", [(5, 40, 9), (3, 128, 19), (2, 192, 13)])
def test_bn_forward_backward(ops, B, C, S):
    dev = "cuda"
    torch.manual_seed(0)
    CP = ops.pad_channels(C)
    x = bfr(torch.randn(B, C, S, S, device=dev) * 2 + 0.5)
    gamma = torch.rand(S, device=dev) + 0.5
    beta = torch.randn(S, device=dev) * 0.2
    rmean, rvar = torch.zeros(S, device=dev), torch.ones(S, device=dev)
    eps, mom = 1e-3, 0.99
    xp = ops.pack_nchw(x, 1, CP)
    stats = torch.zeros(2, S, device=dev)
    coef = torch.zeros(3, S, device=dev)
    ops.bn_train_fwd(xp, B, S, C, gamma, beta, rmean, rvar, eps, mom, stats, coef)
    U = ops.alloc_padded(B, S, 1, CP, dev)
    ops.bn_apply(xp, U, B, S, C, coef=coef, relu=True)
    y_ref, mean, var = col_bn_ref(x, gamma, beta, eps)
    got = ops.unpack(U, C, 1)
    assert torch.allclose(got, F.relu(y_ref), atol=3e-2, rtol=1e-2)
    assert torch.allclose(stats[0], mean, atol=1e-4)
    assert torch.allclose(rmean, (1 - mom) * mean, atol=1e-5)
    assert torch.allclose(rvar, mom + (1 - mom) * var, atol=1e-4)
    # padded channels stay zero
    if C < CP:
        assert U[..., C:].abs().max().item() == 0
    # backward: dx = BN'(dy) + residual
    xr = x.clone().requires_grad_()
    yr, _, _ = col_bn_ref(xr, gamma, beta, eps)
    dy = bfr(torch.randn_like(x))
    res = bfr(torch.randn_like(x))
    yr.backward(dy)
    dgamma, dbeta = torch.zeros(S, device=dev), torch.zeros(S, device=dev)
    bcoef = torch.zeros(3, S, device=dev)
    dyp = ops.pack_nchw(dy, 1, CP)
    ops.bn_bwd_coef(xp, dyp, B, S, C, gamma, stats, dgamma, dbeta, bcoef)
    out = ops.alloc_padded(B, S, 2, CP, dev)  # other output halo (the conv0 gradient case)
    ops.bn_apply(xp, out, B, S, C, coef=bcoef, relu=False, dy=dyp,
                 residual=ops.pack_nchw(res, 1, CP))
    g_ref = xr.grad + res
    got = ops.unpack(out, C, 2)
    scale = g_ref.abs().max().item()
    assert (got - g_ref).abs().max().item() < 2e-2 * scale
    xn = (x - mean) / torch.sqrt(var + eps)
    assert torch.allclose(dbeta, dy.sum(dim=(0, 1, 2)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(dgamma, (dy * xn).sum(dim=(0, 1, 2)), rtol=1e-3, atol=1e-2)
    # inference coefficients from running statistics
    ops.bn_infer_coef(gamma, beta, rmean, rvar, eps, S, coef)
    ops.bn_apply(xp, U, B, S, C, coef=coef, relu=True)
    inf_ref = F.relu((x - rmean) / torch.sqrt(rvar + eps) * gamma + beta)
    assert torch.allclose(ops.unpack(U, C, 1), inf_ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("C,ks", [(64, 3), (192, 3), (32, 3), (128, 1)])
def test_conv_residual_epilogue(ops, C, ks):
    dev = "cuda"
    torch.manual_seed(1)
    B, S = 4, 19
    CP = ops.pad_channels(C)
    x = bfr(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, ks, ks, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = bfr(torch.randn(B, C, S, S, device=dev))
    wf, _ = ops.pack_weights(w, CP, CP)
    bias = torch.zeros(CP, device=dev)
    bias[:C] = b
    xp = ops.pack_nchw(x, 1, CP)
    rp = ops.pack_nchw(r, 1, CP)
    y = ops.alloc_padded(B, S, 1, CP, dev)
    ops.conv_igemm(xp, wf, bias, y, B, S, 1, 1, CP, CP, ks, False, residual=rp)
    ref = F.conv2d(x, bfr(w), b, padding=ks // 2) + r
    got = ops.unpack(y, C, 1)
    assert (got - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    # in place: y = conv(x) + y
    ops.conv_igemm(xp, wf, bias, rp, B, S, 1, 1, CP, CP, ks, False, residual=rp)
    assert (ops.unpack(rp, C, 1) - ref).abs().max().item() < 3e-2 * ref.abs().max().item()


def _pair(K, layers, board, n_skip, seed=3):
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models.policy import ResnetPolicy
    kw = dict(board=board, filters_per_layer=K, layers=layers, seed=seed)
    kw.update(n_skip)
    cpu = ResnetPolicy(DEFAULT_FEATURES, device="cpu", **kw)
    gpu = ResnetPolicy(DEFAULT_FEATURES, device="cuda", **kw)
    rng = np.random.RandomState(seed)
    ws = []
    for (lname, wname, shape), v in zip(cpu.model.net.weight_names, cpu.model.get_weights()):
        if "running_std" in wname:
            v = (rng.rand(*shape) * 2 + 0.5).astype(np.float32)
        elif "running_mean" in wname or "beta" in wname:
            v = (rng.randn(*shape) * 0.1).astype(np.float32)
        elif "gamma" in wname:
            v = (rng.rand(*shape) + 0.5).astype(np.float32)
        elif "param_0" in wname:
            v = (rng.randn(*shape) * 0.1).astype(np.float32)
        ws.append(v)
    cpu.model.set_weights(ws)
    gpu.model.set_weights(ws)
    return cpu, gpu


def _planes(n, board, seed=0):
    rng = np.random.RandomState(seed)
    return (rng.rand(n, 48, board, board) > 0.6).astype(np.uint8)


@pytest.mark.parametrize("K,layers,board,n_skip", [(64, 5, 19, {}), (32, 4, 9, {"n_skip_1": 2}),
                                                   (128, 7, 19, {"n_skip_3": 3})])
def test_resnet_plan_forward_matches_generic(ops, K, layers, board, n_skip):
    from rocalphago_amd.models.fused import ResnetPlan
    cpu, gpu = _pair(K, layers, board, n_skip)
    plan = gpu.model._plan_for()
    assert isinstance(plan, ResnetPlan)
    X = _planes(6, board)
    ref = cpu.model.predict(X)
    got = gpu.model.predict(X)
    lr, lg = np.log(ref + 1e-12), np.log(got + 1e-12)
    # bf16 activations through every layer: compare log-probabilities of the likely moves
    sel = ref > 1e-3
    assert np.abs(lr - lg)[sel].max() < 0.15
    assert np.abs(ref - got).max() < 2e-2


@pytest.mark.parametrize("K,layers,board,n_skip", [(64, 5, 19, {}), (32, 4, 9, {"n_skip_1": 2})])
def test_resnet_plan_train_step_matches_generic(ops, K, layers, board, n_skip):
    from rocalphago_amd.models import kerasish as KZ
    cpu, gpu = _pair(K, layers, board, n_skip)
    B = 16
    X = _planes(B, board, 1)
    lab = np.random.RandomState(2).randint(0, board * board, B)
    Y = np.zeros((B, board * board), np.float32)
    Y[np.arange(B), lab] = 1
    for m in (cpu.model, gpu.model):
        m.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
    r_cpu = cpu.model.train_on_batch(X, Y)
    r_gpu = gpu.model.train_on_batch(X, Y)
    assert abs(r_cpu - r_gpu) < 0.05 * abs(r_cpu)
    net_c, net_g = cpu.model.net, gpu.model.net
    for (lname, wname, shape), gc, gg, pc, pg in zip(net_c.weight_names, net_c._gviews,
                                                     net_g._gviews, net_c._views, net_g._views):
        gc, gg = gc.detach().reshape(-1), gg.detach().cpu().reshape(-1)
        if "running" in wname:
            # running statistics: updated from the batch statistics, no gradient
            assert torch.allclose(pc.detach().cpu(), pg.detach().cpu(), rtol=1e-2, atol=2e-3), \
                wname
            continue
        nc = gc.norm().item()
        if nc < 1e-6:
            assert gg.norm().item() < 1e-3, wname
            continue
        cos = torch.dot(gc, gg).item() / (nc * gg.norm().item() + 1e-12)
        assert cos > 0.98, (wname, cos)
        assert abs(gg.norm().item() / nc - 1) < 0.08, (wname, gg.norm().item(), nc)


def test_pass_grads_kernel_matches_torch(ops):
    """head.hip pass_grads_kernel: dW = dpass^T z, db = sum dpass (fp32 torch reference)."""
    g = torch.Generator().manual_seed(0)
    for B, P in [(1, 49), (7, 81), (256, 361)]:
        z = torch.randn(B, P, generator=g).cuda()
        dp = torch.randn(B, generator=g).cuda()
        dW = torch.full((P,), 9.0, device="cuda")
        db = torch.full((1,), 9.0, device="cuda")
        ops.pass_grads(z, dp, dW, db)
        torch.cuda.synchronize()
        ref = (z.double().t() @ dp.double()).float()
        assert torch.allclose(dW, ref, rtol=1e-5, atol=1e-4 * max(1.0, ref.abs().max().item()))
        assert abs(db.item() - dp.double().sum().item()) < 1e-4 * B


def test_resnet_plan_with_pass_logit_matches_generic(ops):
    """ResnetPlan carries the PassLogit head (softmax over S*S + 1) in forward and training,
    with the PassLogit gradients on HIP; the update matches the generic fp32 executor."""
    from rocalphago_amd.models import kerasish as KZ
    from rocalphago_amd.models.fused import ResnetPlan
    cpu, gpu = _pair(32, 4, 9, {"pass_logit": True})
    assert isinstance(gpu.model._plan_for(), ResnetPlan)
    assert gpu.model._plan_for().pass_name is not None
    rs = np.random.RandomState(4)
    w = cpu.model.get_weights()
    w[-2] = (rs.randn(81) * 0.05).astype(np.float32)
    w[-1] = np.array([0.4], np.float32)
    cpu.model.set_weights(w)
    gpu.model.set_weights(w)
    X = _planes(12, 9, 3)
    pc, pg = cpu.model.predict(X), gpu.model.predict(X)
    assert pg.shape == (12, 82) and np.abs(pg - pc).max() < 2e-2
    Y = np.zeros((12, 82), np.float32)
    Y[np.arange(12), rs.randint(0, 82, 12)] = 1
    Y[:4, :] = 0
    Y[:4, 81] = 1  # pass targets
    for m in (cpu.model, gpu.model):
        m.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
    lc, lg = cpu.model.train_on_batch(X, Y), gpu.model.train_on_batch(X, Y)
    assert abs(lc - lg) < 0.05 * abs(lc)
    net_c, net_g = cpu.model.net, gpu.model.net
    names = [wn for _, wn, _ in net_c.weight_names]
    for wname, gc, gg in zip(names, net_c._gviews, net_g._gviews):
        if "running" in wname:
            continue
        gc, gg = gc.detach().reshape(-1), gg.detach().cpu().reshape(-1)
        nc = gc.norm().item()
        if nc < 1e-6:
            continue
        cos = torch.dot(gc, gg).item() / (nc * gg.norm().item() + 1e-12)
        assert cos > 0.98, (wname, cos)
    # the PassLogit tensors are the last two weights
    for gc, gg in zip(net_c._gviews[-2:], net_g._gviews[-2:]):
        gc, gg = gc.detach().reshape(-1), gg.detach().cpu().reshape(-1)
        assert (gc - gg).abs().max().item() < 5e-2 * max(gc.abs().max().item(), 1e-3)


def test_bn_prologue_kernels_match_torch(ops):
    """K13: BN + ReLU fused into the 128-channel conv kernels. The layer input
    U = ReLU(cx[col] * x + cc[col]) (zero on the halo) is built while staging from the BN input x:
    forward with the residual epilogue, dgrad with the ReLU mask recomputed from x, and the slab
    wgrad (reduction deferred into that dgrad) -- each against fp32 PyTorch on the materialised
    U."""
    dev = "cuda"
    torch.manual_seed(7)
    B, C, S = 256, 128, 19
    assert ops.conv_bn_fusable(B, S, 1, C, C, 3)
    x = bfr(torch.randn(B, C, S, S, device=dev) * 1.5)
    coef = torch.zeros(3, S, device=dev)
    coef[0] = torch.rand(S, device=dev) + 0.5
    coef[2] = torch.randn(S, device=dev) * 0.3
    U = bfr(F.relu(x * coef[0] + coef[2]))  # per column w (last axis)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = bfr(torch.randn(B, C, S, S, device=dev))
    g = bfr(torch.randn(B, C, S, S, device=dev))
    xp, rp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(r, 1, C), ops.pack_nchw(g, 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    y = ops.alloc_padded(B, S, 1, C, dev)
    nblk = ops.conv_bn_stat_blocks(B, S, C)
    part = torch.full((nblk, 2, S), 7.0, device=dev)
    ops.conv_igemm_bn(xp, wf, b, y, B, S, C, C, False, bn_coef=coef, residual=rp, stat_part=part)
    ref = F.conv2d(U, bfr(w), b, padding=1) + r
    got = ops.unpack(y, C, 1)
    assert (got - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    # the epilogue's column statistics are those of the stored output
    sums = part.double().sum(0)
    assert torch.allclose(sums[0], got.double().sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert torch.allclose(sums[1], (got.double() ** 2).sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert y[:, 0].abs().max().item() == 0 and y[:, :, -1].abs().max().item() == 0
    Ur, wr = U.clone().requires_grad_(), bfr(w).requires_grad_()
    (F.conv2d(Ur, wr, padding=1) * g).sum().backward()
    h = ops.PendingReduction()
    dw, db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
    ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=h,
                   xcoef=coef)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    mean = torch.randn(S, device=dev) * 0.1
    ops.conv_igemm_bn(gp, wb, None, dx, B, S, C, C, False, mask=xp, mask_coef=coef, pending=h,
                      stat_part=part, stat_mean=mean)
    torch.cuda.synchronize()
    ref_dx = Ur.grad * (U > 0)
    d = ops.unpack(dx, C, 1).double()
    sums = part.double().sum(0)
    assert torch.allclose(sums[0], d.sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert torch.allclose(sums[1], (d * (x.double() - mean.double())).sum((0, 1, 2)), rtol=1e-4,
                          atol=1e-1)
    err = (ops.unpack(dx, C, 1) - ref_dx).abs().max().item()
    assert err < 2e-2 * ref_dx.abs().max().item()
    assert (dw - wr.grad).abs().max().item() < 1e-2 * wr.grad.abs().max().item()
    assert torch.allclose(db, g.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


def test_wino_bn_kernels_match_torch(ops):
    """K13 on the Winograd kernel (conv_wino.hip WinoBN): the 128-channel residual trunk's
    forward builds U = ReLU(cx[col] x + cc[col]) (zero on the halo) in the input transform and adds
    the residual in its epilogue; the dgrad recomputes the ReLU mask from x while a deferred wgrad
    reduction rides in it; both sum their column statistics per board. Against fp32 PyTorch on the
    materialised U, and the statistics against the stored outputs."""
    dev = "cuda"
    torch.manual_seed(17)
    B, C, S = 256, 128, 19
    # one wave of one-board blocks at any batch up to the CU count; a ragged second wave: direct
    assert ops.conv_wino_bn_ok(B, S, C, C) and ops.conv_wino_bn_ok(100, S, C, C)
    assert not ops.conv_wino_bn_ok(300, S, C, C)
    x = bfr(torch.randn(B, C, S, S, device=dev) * 1.5)
    coef = torch.zeros(3, S, device=dev)
    coef[0] = torch.rand(S, device=dev) + 0.5
    coef[2] = torch.randn(S, device=dev) * 0.3
    U = F.relu(x * coef[0] + coef[2])
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = bfr(torch.randn(B, C, S, S, device=dev))
    g = bfr(torch.randn(B, C, S, S, device=dev))
    xp, rp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(r, 1, C), ops.pack_nchw(g, 1, C)
    uf, ub = ops.wino_weights(w, C, C)
    y = ops.alloc_padded(B, S, 1, C, dev)
    part = torch.full((B, 2, S), 7.0, device=dev)
    ops.conv_wino_bn(xp, uf, b, y, B, S, C, C, False, bn_coef=coef, residual=rp, stat_part=part)
    ref = F.conv2d(U, w, b, padding=1) + r
    got = ops.unpack(y, C, 1)
    assert (got - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    assert (got - ref).norm().item() < 6e-3 * ref.norm().item()
    sums = part.double().sum(0)
    assert torch.allclose(sums[0], got.double().sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert torch.allclose(sums[1], (got.double() ** 2).sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert y[:, 0].abs().max().item() == 0 and y[:, :, -1].abs().max().item() == 0
    # dgrad with a deferred wgrad reduction riding in the launch
    Ur, wr = U.clone().requires_grad_(), w.clone().requires_grad_()
    (F.conv2d(Ur, wr, padding=1) * g).sum().backward()
    h = ops.PendingReduction()
    dw, db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
    ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=h,
                   xcoef=coef)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    mean = torch.randn(S, device=dev) * 0.1
    ops.conv_wino_bn(gp, ub, None, dx, B, S, C, C, False, mask=xp, mask_coef=coef, pending=h,
                     stat_part=part, stat_mean=mean)
    torch.cuda.synchronize()
    ref_dx = Ur.grad * (U > 0)
    d = ops.unpack(dx, C, 1).double()
    sums = part.double().sum(0)
    assert torch.allclose(sums[0], d.sum((0, 1, 2)), rtol=1e-4, atol=1e-1)
    assert torch.allclose(sums[1], (d * (x.double() - mean.double())).sum((0, 1, 2)), rtol=1e-4,
                          atol=1e-1)
    err = (ops.unpack(dx, C, 1) - ref_dx).abs().max().item()
    assert err < 2e-2 * ref_dx.abs().max().item()
    assert (dw - wr.grad).abs().max().item() < 1e-2 * wr.grad.abs().max().item()
    assert torch.allclose(db, g.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("wino", ["0", "2"])
def test_resnet_bn_prologue_train_step_matches_unfused(ops, monkeypatch, wino):
    """A 128-filter ResnetPolicy train step at B = 256 with BN+ReLU fused into the conv
    prologues gives the same loss and gradients as the bn_apply path (bn_prologue = False): on the
    direct kernels (WINO_MODE 0), and with the fused layers on the Winograd kernel (forward and
    dgrad, WINO_MODE 2; its transform roundings put the gradients' cosine at 0.997-0.999)."""
    from rocalphago_amd.models import kerasish as KZ
    monkeypatch.setattr(ResTrunk, "WINO_MODE", wino)
    _, fused = _pair(128, 5, 19, {})
    _, plain = _pair(128, 5, 19, {})
    plain.model._plan_for().trunk.bn_prologue = False
    B = 256
    X = _planes(B, 19, 5)
    lab = np.random.RandomState(6).randint(0, 361, B)
    Y = np.zeros((B, 361), np.float32)
    Y[np.arange(B), lab] = 1
    for m in (fused.model, plain.model):
        m.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
    lf, lp = fused.model.train_on_batch(X, Y), plain.model.train_on_batch(X, Y)
    assert any(fused.model._plan_for().trunk._fused)
    assert not any(plain.model._plan_for().trunk._fused)
    assert any(fused.model._plan_for().trunk._plan(B)[1]) == (wino == "2")
    assert abs(lf - lp) < 1e-3 * abs(lp)
    # Winograd: the transform roundings go through nine BN backwards. The conv biases in front of
    # a column BN have small gradients that sum every pixel's error (cosine 0.9969, norm +-2 %
    # measured), so they are checked only as part of the whole gradient; the kernels themselves
    # are pinned against fp32 in test_wino_bn_kernels_match_torch.
    min_cos, norm_tol = (0.999, 1e-2) if wino == "0" else (0.995, 2e-2)
    flat_f, flat_p = [], []
    for (lname, wname, shape), gf, gp in zip(fused.model.net.weight_names,
                                             fused.model.net._gviews, plain.model.net._gviews):
        if "running" in wname:
            continue
        flat_f.append(gf.detach().reshape(-1).float())
        flat_p.append(gp.detach().reshape(-1).float())
        if wino != "0" and wname.endswith("_b"):
            continue
        gf, gp = gf.detach().reshape(-1).float(), gp.detach().reshape(-1).float()
        n = gp.norm().item()
        if n < 1e-6:
            continue
        cos = torch.dot(gf, gp).item() / (n * gf.norm().item() + 1e-12)
        assert cos > min_cos, (wname, cos)
        assert abs(gf.norm().item() / n - 1) < norm_tol, (wname, gf.norm().item(), n)
    gf, gp = torch.cat(flat_f), torch.cat(flat_p)
    cos = torch.dot(gf, gp).item() / (gf.norm().item() * gp.norm().item())
    assert cos > (0.999 if wino == "0" else 0.998), cos


def _cos(a, b):
    a, b = a.detach().reshape(-1).double().cpu(), b.detach().reshape(-1).double().cpu()
    return torch.dot(a, b).item() / (a.norm().item() * b.norm().item() + 1e-30)


def test_resnet_wino_train_step_vs_fp32(ops, monkeypatch):
    """The Winograd BN path is as close to the fp32 generic executor as the direct kernels: one
    128-filter ResnetPolicy train step at B = 256 (the fused 3x3 layers on conv_wino's WinoBN
    forward + dgrad vs on the ping-pong kernels), weight-gradient cosines against the CPU fp32
    step per tensor and over the whole gradient."""
    from rocalphago_amd.models import kerasish as KZ
    monkeypatch.setattr(ResTrunk, "WINO_MODE", "0")
    cpu, direct = _pair(128, 5, 19, {})
    direct.model._plan_for()  # (the trunk reads WINO_MODE when the plan is built)
    monkeypatch.setattr(ResTrunk, "WINO_MODE", "2")
    _, wino = _pair(128, 5, 19, {})
    wino.model._plan_for()
    B = 256
    X = _planes(B, 19, 7)
    lab = np.random.RandomState(8).randint(0, 361, B)
    Y = np.zeros((B, 361), np.float32)
    Y[np.arange(B), lab] = 1
    models = (cpu.model, direct.model, wino.model)
    for m in models:
        m.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
    losses = [m.train_on_batch(X, Y) for m in models]
    assert any(wino.model._plan_for().trunk._plan(B)[1])
    assert not any(direct.model._plan_for().trunk._plan(B)[1])
    assert abs(losses[2] - losses[0]) < 2e-3 * abs(losses[0])
    names = [wn for _, wn, _ in cpu.model.net.weight_names]
    views = [m.net._gviews for m in models]
    keep = [i for i, wn in enumerate(names) if "running" not in wn]
    for i in keep:
        if not names[i].endswith("_W"):
            continue
        cd, cw = _cos(views[1][i], views[0][i]), _cos(views[2][i], views[0][i])
        assert cw > cd - 2e-3, (names[i], cd, cw)
    flat = [torch.cat([v[i].detach().reshape(-1).double().cpu() for i in keep]) for v in views]
    cd, cw = _cos(flat[1], flat[0]), _cos(flat[2], flat[0])
    assert cw > cd - 1e-3, (cd, cw)


@pytest.mark.gpu
@pytest.mark.parametrize("residual", [False, True])
def test_bn_apply_with_folded_finalize_matches_two_launches(ops, residual):
    """bn_apply_bwd_part (every block derives the column coefficients from the dgrad partials)
    equals bn_finalize_bwd + bn_apply: dgamma / dbeta and dL/dx (+ the skip gradient)."""
    dev = torch.device("cuda")
    torch.manual_seed(8)
    B, C, S, nblk = 64, 128, 19, 61
    part = torch.randn(nblk, 2, S, device=dev) * 3.0
    gamma = torch.rand(S, device=dev) + 0.5
    stats = torch.stack([torch.randn(S, device=dev) * 0.1, torch.rand(S, device=dev) + 0.5])
    x = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C)
    dy = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C)
    res = ops.pack_nchw(torch.randn(B, C, S, S, device=dev), 1, C) if residual else None
    dg0, db0 = torch.zeros(S, device=dev), torch.zeros(S, device=dev)
    coef = torch.zeros(3, S, device=dev)
    ops.bn_finalize_bwd(part, nblk, B, S, C, gamma, stats, dg0, db0, coef)
    ref = ops.alloc_padded(B, S, 1, C, dev)
    ops.bn_apply(x, ref, B, S, C, coef=coef, relu=False, dy=dy, residual=res)
    dg1, db1 = torch.zeros(S, device=dev), torch.zeros(S, device=dev)
    out = ops.alloc_padded(B, S, 1, C, dev)
    ops.bn_apply_bwd_part(part, nblk, x, out, B, S, C, gamma, stats, dg1, db1, dy, residual=res)
    torch.cuda.synchronize()
    assert torch.allclose(dg1, dg0, rtol=1e-6, atol=1e-6)
    assert torch.allclose(db1, db0, rtol=1e-6, atol=1e-6)
    d = (out.float() - ref.float()).abs()
    assert d.max().item() <= 1e-2 * ref.float().abs().max().item()
    assert out[:, 0].abs().max().item() == 0 and out[:, :, -1].abs().max().item() == 0


@pytest.mark.parametrize("knob,val,C", [("tap_mode", 6, 192), ("tap_mode", 6, 128)])
def test_conv_pp_variants_bit_identical(ops, knob, val, C):
    """The ping-pong conv's A/B alternative keeps every accumulator's MFMA order, so its outputs
    equal the default kernel's bit for bit (the BN statistics partials to fp32 atomic-order
    rounding): dispatch mode 6 (all slab loads at tap 0, per-segment priority flips) against the
    default 12 -- forward with bias+ReLU, with a residual, masked dgrad, and at 128 channels the
    BN-prologue forward / dgrad with their column statistics; the forward also against fp32
    PyTorch. (Round 4's K2 / register-staging variants were deleted in round 5.)"""
    from rocalphago_amd.ops.hipops import _lib
    setter = getattr(_lib(), "rag_conv_" + knob)
    dev = "cuda"
    torch.manual_seed(11)
    B, S = 256, 19
    x = bfr(torch.randn(B, C, S, S, device=dev)).relu()
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    xp = ops.pack_nchw(x, 1, C)
    rp = ops.pack_nchw(bfr(torch.randn(B, C, S, S, device=dev)), 1, C)
    gp = ops.pack_nchw(bfr(torch.randn(B, C, S, S, device=dev)), 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    coef = torch.zeros(3, S, device=dev)
    coef[0] = torch.rand(S, device=dev) + 0.5
    coef[2] = torch.randn(S, device=dev) * 0.3
    mean = torch.randn(S, device=dev) * 0.1
    nblk = ops.conv_bn_stat_blocks(B, S, C) if C == 128 else 1

    def run():
        outs = []
        for form in range(5 if C == 128 else 3):
            y = ops.alloc_padded(B, S, 1, C, dev)
            part = torch.zeros(nblk, 2, S, device=dev)
            if form == 0:
                ops.conv_igemm(xp, wf, b, y, B, S, 1, 1, C, C, 3, True)
            elif form == 1:
                ops.conv_igemm(xp, wf, None, y, B, S, 1, 1, C, C, 3, False, residual=rp)
            elif form == 2:
                ops.conv_igemm(gp, wb, None, y, B, S, 1, 1, C, C, 3, False, mask=xp)
            elif form == 3:
                ops.conv_igemm_bn(xp, wf, b, y, B, S, C, C, False, bn_coef=coef, residual=rp,
                                  stat_part=part)
            else:
                ops.conv_igemm_bn(gp, wb, None, y, B, S, C, C, False, mask=xp, mask_coef=coef,
                                  stat_part=part, stat_mean=mean)
            outs.append((y.clone(), part.clone()))
        torch.cuda.synchronize()
        return outs

    old = setter(12)
    try:
        ref = run()
        setter(val)
        got = run()
    finally:
        setter(old)
    for form, ((yr, pr), (yg, pg)) in enumerate(zip(ref, got)):
        assert torch.equal(yr, yg), form
        # column statistics: LDS atomics in the epilogue, order-dependent in the last bits
        assert torch.allclose(pr, pg, rtol=1e-5, atol=1e-3), form
    want = F.relu(F.conv2d(x, bfr(w), b, padding=1))
    got0 = ops.unpack(got[0][0], C, 1)
    assert (got0 - want).abs().max().item() < 2e-2 * want.abs().max().item()
