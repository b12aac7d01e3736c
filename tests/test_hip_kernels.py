"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references (GPU only)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def bf(t):
    return t.to(torch.bfloat16).float()


def rel_err(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.ops import hipops
    return hipops


@pytest.mark.parametrize("B,cin,cout,ks,S", [(3, 192, 192, 3, 19), (5, 48, 192, 5, 19),
                                             (2, 16, 16, 3, 19), (7, 128, 128, 3, 13),
                                             (4, 192, 32, 1, 19), (1, 12, 16, 5, 9),
                                             (2, 64, 96, 3, 7), (130, 192, 192, 3, 19),
                                             (128, 48, 192, 5, 19), (256, 48, 192, 5, 19),
                                             (256, 40, 192, 5, 19), (256, 48, 128, 5, 19)])
def test_conv_forward(ops, B, cin, cout, ks, S):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(B, cin, S, S, device=dev)
    w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
    b = torch.randn(cout, device=dev) * 0.1
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=ks // 2))
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    hi = ks // 2 if ks > 1 else 1
    xp = ops.pack_nchw(x, hi, cinp)
    wf, _ = ops.pack_weights(w, coutp, cinp)
    bias = torch.zeros(coutp, device=dev)
    bias[:cout] = b
    y = ops.alloc_padded(B, S, 1, coutp, dev)
    ops.conv_igemm(xp, wf, bias, y, B, S, hi, 1, cinp, coutp, ks, relu=True, cin=cin)
    out = ops.unpack(y, cout, 1)
    assert rel_err(out, ref) < 2e-2
    # halo stays zero
    assert y[:, 0].abs().max().item() == 0 and y[:, :, -1].abs().max().item() == 0


# (hi, hg) = input / gradient halos; hi == hg selects the all-taps wgrad kernel (wgrad.hip)
@pytest.mark.parametrize("B,cin,cout,ks,hi,hg,S", [
    (3, 192, 192, 3, 1, 1, 19), (2, 16, 16, 3, 1, 1, 19), (4, 64, 128, 3, 1, 1, 19),
    (3, 32, 192, 5, 2, 1, 19), (3, 64, 192, 5, 2, 2, 19), (2, 128, 64, 1, 1, 1, 19),
    (37, 192, 192, 3, 1, 1, 19), (5, 64, 64, 3, 2, 2, 9), (6, 128, 192, 3, 1, 1, 13),
    (128, 192, 192, 3, 1, 1, 19)])
def test_conv_backward(ops, B, cin, cout, ks, hi, hg, S):
    dev = torch.device("cuda")
    torch.manual_seed(1)
    x = F.relu(torch.randn(B, cin, S, S, device=dev))
    w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
    g = torch.randn(B, cout, S, S, device=dev)
    xr, wr = bf(x).requires_grad_(), bf(w).requires_grad_()
    y = F.conv2d(xr, wr, padding=ks // 2)
    (y * bf(g)).sum().backward()
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    xp = ops.pack_nchw(x, hi, cinp)
    gp = ops.pack_nchw(g, hg, coutp)
    wf, wb = ops.pack_weights(w, coutp, cinp,
                              wb=torch.empty(ks * ks, cinp, coutp, dtype=torch.bfloat16,
                                             device=dev))
    if ks == 3 and hg == 1:
        # dgrad with fused ReLU mask of the layer input
        xm = ops.pack_nchw(x, 1, cinp)
        dx = ops.alloc_padded(B, S, 1, cinp, dev)
        ops.conv_igemm(gp, wb, None, dx, B, S, 1, 1, coutp, cinp, ks, relu=False, mask=xm)
        ref_dx = xr.grad * (x > 0)
        assert rel_err(ops.unpack(dx, cin, 1), ref_dx) < 2e-2
    dw = torch.zeros(cout, cin, ks, ks, device=dev)
    db = torch.zeros(cout, device=dev)
    ops.conv_wgrad(gp, xp, dw, db, B, S, hi, cout, coutp, cin, cinp, ks, hg=hg)
    assert rel_err(dw, wr.grad) < 2e-2
    assert rel_err(db, bf(g).sum((0, 2, 3))) < 2e-2


def test_conv_residual_halo2_ragged_batch(ops):
    """The default 3x3 dispatch at a ragged batch (B = 131: the 192-pixel kernels) vs fp32
    PyTorch: residual sum-merge epilogue, output halo 2 (stays zero), boards past B untouched,
    and dgrad. (The opt-in one-board-per-block slab kernel it used to force was deleted in
    round 5.)"""
    dev = torch.device("cuda")
    torch.manual_seed(3)
    B, C, S = 131, 192, 19
    x = torch.randn(B, C, S, S, device=dev)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = torch.randn(B, C, S, S, device=dev)
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=1) + bf(r))
    xp = ops.pack_nchw(x, 1, C)
    wf, _ = ops.pack_weights(w, C, C)
    y = ops.alloc_padded(B + 1, S, 2, C, dev)
    y[B:] = 7.0
    rp = ops.alloc_padded(B, S, 2, C, dev)
    rp[:, 2:-2, 2:-2] = ops.pack_nchw(r, 2, C)[:, 2:-2, 2:-2]
    ops.conv_igemm(xp, wf, b, y[:B], B, S, 1, 2, C, C, 3, relu=True, residual=rp)
    # dgrad form (ReLU mask of the layer input)
    wf2, wb2 = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16,
                                                          device=dev))
    g = torch.randn(B, C, S, S, device=dev)
    xr = bf(F.relu(x)).requires_grad_()
    F.conv2d(xr, bf(w), padding=1).mul(bf(g)).sum().backward()
    xm = ops.pack_nchw(F.relu(x), 1, C)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(ops.pack_nchw(g, 1, C), wb2, None, dx, B, S, 1, 1, C, C, 3, relu=False,
                   mask=xm)
    assert rel_err(ops.unpack(dx, C, 1), xr.grad * (x > 0)) < 2e-2
    assert rel_err(ops.unpack(y[:B], C, 2), ref) < 2e-2
    assert y[:B, :2].abs().max().item() == 0 and y[:B, :, -2:].abs().max().item() == 0
    assert (y[B:] == 7.0).all()


def test_pack_input_transforms(ops):
    dev = torch.device("cuda")
    S, NF, B = 19, 48, 8
    feats = (torch.rand(10, NF, S, S, device=dev) > 0.5).to(torch.uint8)
    idx = torch.tensor([3, 1, 4, 1, 5, 9, 2, 6], device=dev, dtype=torch.int64)
    tf = torch.arange(8, device=dev, dtype=torch.int32)
    out = ops.alloc_padded(B, S, 2, 64, dev)
    ops.pack_input(feats, out, 2, index=idx, transforms=tf)
    got = ops.unpack(out, NF, 2).cpu().numpy()
    fn = [lambda a: a, lambda a: np.rot90(a, 1), lambda a: np.rot90(a, 2), lambda a: np.rot90(a, 3),
          np.fliplr, np.flipud, np.transpose, lambda a: np.fliplr(np.rot90(a, 1))]
    src = feats.cpu().numpy()
    for b in range(B):
        for c in (0, 7, 47):
            assert np.array_equal(got[b, c], fn[b](src[idx[b].item(), c]).astype(np.float32))


def test_policy_head_and_backward(ops):
    dev = torch.device("cuda")
    torch.manual_seed(2)
    B, K, S = 6, 192, 19
    h = F.relu(torch.randn(B, K, S, S, device=dev))
    w = torch.randn(K, device=dev) * 0.1
    b0 = torch.tensor([0.3], device=dev)
    pb = torch.randn(S * S, device=dev) * 0.1
    lab = torch.randint(0, S * S, (B,), device=dev)
    hp = ops.pack_nchw(h, 1, K)
    probs = torch.empty(B, S * S, device=dev)
    loss = torch.empty(B, device=dev)
    dz = torch.empty(B, S * S, device=dev)
    hit = torch.empty(B, device=dev)
    ops.policy_head_fwd(hp, w, b0, pb, probs, K, labels=lab, loss=loss, dz=dz, hit=hit, mode=1,
                        gscale=1.0 / B)
    hr = bf(h).requires_grad_()
    wr, br = w.clone().requires_grad_(), b0.clone().requires_grad_()
    pbr = pb.clone().requires_grad_()
    z = (hr * wr.view(1, K, 1, 1)).sum(1).flatten(1) + br + pbr
    ref = F.softmax(z, dim=1)
    assert rel_err(probs, ref) < 1e-2
    l = F.cross_entropy(z, lab)
    l.backward()
    assert abs(loss.mean().item() - l.item()) < 1e-2 * max(1.0, l.item())
    assert torch.equal(hit.bool(), z.argmax(1) == lab)
    dh = ops.alloc_padded(B, S, 1, K, dev)
    dw = torch.zeros(K, device=dev)
    db0 = torch.zeros(1, device=dev)
    dpb = torch.zeros(S * S, device=dev)
    ops.head_bwd(hp, w, dz, dh, dw, db0, dpb, K, relu_mask=True)
    assert rel_err(ops.unpack(dh, K, 1), hr.grad * (h > 0)) < 2e-2
    assert rel_err(dw, wr.grad) < 2e-2
    assert abs(db0.item() - br.grad.item()) < 1e-4  # both ~0: sum of (p - y)
    assert rel_err(dpb, pbr.grad) < 2e-2


@pytest.mark.parametrize("B", [256, 7])
def test_head_bwd_bias_gradient_sums_all_of_dz(ops, B):
    """Without per-board sums (the value head) head_bwd's db0 is the sum of all B x 361 dz values
    (16-byte loads, four sums per thread; B = 7: 2527 values, not a multiple of 4)."""
    dev = torch.device("cuda")
    torch.manual_seed(3)
    K, S = 192, 19
    h = F.relu(torch.randn(B, K, S, S, device=dev))
    hp = ops.pack_nchw(h, 1, K)
    w = torch.randn(K, device=dev) * 0.1
    dz = torch.randn(B, S * S, device=dev)
    dh = ops.alloc_padded(B, S, 1, K, dev)
    dw = torch.zeros(K, device=dev)
    db0 = torch.zeros(1, device=dev)
    ops.head_bwd(hp, w, dz, dh, dw, db0, None, K, relu_mask=True)
    ref = dz.double().sum().item()
    assert abs(db0.item() - ref) < 1e-5 * dz.abs().sum().item()
    ref_dw = (bf(h) * dz.view(B, 1, S, S)).sum((0, 2, 3))
    assert rel_err(dw, ref_dw) < 1e-2


def test_sgd(ops):
    dev = torch.device("cuda")
    p = torch.randn(1001, device=dev)
    g = torch.randn(1001, device=dev)
    ref = p - 0.1 * g
    ops.sgd_(p, g, 0.1)
    assert torch.allclose(p, ref, atol=1e-6)
    v = torch.zeros(1001, device=dev)
    p2 = p.clone()
    ops.sgd_(p, g, 0.1, momentum=0.9, v=v)
    assert torch.allclose(p, p2 - 0.1 * g, atol=1e-6)


def test_dgrad_mixed_halos(ops):
    """dgrad writing g_{l-1} with the halo of layer l-1's input (2, a 5x5 layer below) while the
    ReLU mask (layer l's input) keeps halo 1 — the layout the engine uses below the 5x5 layer."""
    dev = torch.device("cuda")
    torch.manual_seed(3)
    B, S, cin, cout, ks = 3, 19, 192, 192, 3
    x = F.relu(torch.randn(B, cin, S, S, device=dev))
    w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
    g = torch.randn(B, cout, S, S, device=dev)
    xr, wr = bf(x).requires_grad_(), bf(w)
    (F.conv2d(xr, wr, padding=1) * bf(g)).sum().backward()
    _, wb = ops.pack_weights(w, cout, cin, wb=torch.empty(9, cin, cout, dtype=torch.bfloat16,
                                                          device=dev))
    gp = ops.pack_nchw(g, 1, cout)
    xm = ops.pack_nchw(x, 1, cin)
    dx = ops.alloc_padded(B, S, 2, cin, dev)
    ops.conv_igemm(gp, wb, None, dx, B, S, 1, 2, cout, cin, ks, False, mask=xm, mask_halo=1)
    assert rel_err(ops.unpack(dx, cin, 2), xr.grad * (x > 0)) < 2e-2
    assert dx[:, :2].abs().max().item() == 0 and dx[:, :, -2:].abs().max().item() == 0


def test_pack_input_bits_matches_uint8(ops):
    from rocalphago_amd.training.replay import pack_bits
    dev = torch.device("cuda")
    S, NF, B = 19, 49, 16
    feats = (torch.rand(40, NF, S, S, device=dev) > 0.5).to(torch.uint8)
    bits = pack_bits(feats)
    idx = torch.randint(0, 40, (B,), device=dev)
    tf = torch.randint(0, 8, (B,), device=dev, dtype=torch.int32)
    a = ops.alloc_padded(B, S, 2, 64, dev)
    b = ops.alloc_padded(B, S, 2, 64, dev)
    ops.pack_input(feats, a, 2, index=idx, transforms=tf)
    ops.pack_input(bits, b, 2, index=idx, transforms=tf, nplanes=NF)
    assert torch.equal(a, b)


def test_packed_dataset_training_matches_plain(ops):
    from rocalphago_amd.models import kerasish as K
    from rocalphago_amd.models.policy import CNNPolicy
    from rocalphago_amd.training.data import DeviceDataset
    from rocalphago_amd.training.replay import PackedDataset
    from rocalphago_amd.training.supervised import SupervisedTrainer
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    rs = np.random.RandomState(4)
    st = (rs.rand(64, 48, 19, 19) > 0.6).astype(np.uint8)
    acts = rs.randint(0, 361, 64)
    losses = []
    for cls in (DeviceDataset, PackedDataset):
        pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=64, layers=3, device="cuda", seed=9)
        pol.model.compile(loss="categorical_crossentropy", optimizer=K.SGD(lr=0.05))
        tr = SupervisedTrainer(pol.model, cls(st, acts, "cuda"), 32, ["noop", "rot90"], None,
                               seed=1)
        for s in range(3):
            tr.step(torch.arange(s * 16, s * 16 + 32, device="cuda") % 64)
        losses.append(tr.pop_metrics()[0])
    assert abs(losses[0] - losses[1]) < 1e-5


@pytest.mark.parametrize("B,P,H,act", [(256, 361, 256, "linear"), (5, 49, 64, "relu"),
                                       (3, 81, 300, "tanh"), (1, 361, 256, "linear")])
def test_value_mlp_fwd(ops, B, P, H, act):
    dev = torch.device("cuda")
    torch.manual_seed(3)
    z = torch.randn(B, P, device=dev)
    W1 = torch.randn(P, H, device=dev) * 0.05
    b1 = torch.randn(H, device=dev) * 0.1
    W2 = torch.randn(H, 1, device=dev) * 0.1
    b2 = torch.randn(1, device=dev) * 0.1
    h = z.double() @ W1.double() + b1.double()
    h = {"linear": h, "relu": torch.relu(h), "tanh": torch.tanh(h)}[act]
    ref = torch.tanh(h @ W2.double() + b2.double()).float()
    hout = torch.empty(B, H, device=dev)
    out = ops.value_mlp_fwd(z, W1, b1, W2, b2, act=act, hout=hout)
    torch.cuda.synchronize()
    assert out.shape == (B, 1)
    assert (out - ref).abs().max().item() < 1e-4
    href = (z.double() @ W1.double() + b1.double()).float()
    assert rel_err(hout, href) < 1e-5


@pytest.mark.parametrize("B,P,H,act,weighted", [(256, 361, 256, "relu", False),
                                                (100, 361, 256, "tanh", True),
                                                (7, 49, 200, "linear", True),
                                                (1, 81, 64, "relu", False),
                                                (130, 361, 300, "tanh", False)])
def test_value_mlp_train(ops, B, P, H, act, weighted):
    """Loss and every head gradient of the HIP value-MLP training path vs fp64 autograd."""
    dev = torch.device("cuda")
    torch.manual_seed(5)
    z = torch.randn(B, P, device=dev)
    W1 = torch.randn(P, H, device=dev) * 0.05
    b1 = torch.randn(H, device=dev) * 0.1
    W2 = torch.randn(H, 1, device=dev) * 0.1
    b2 = torch.randn(1, device=dev) * 0.1
    y = torch.rand(B, device=dev) * 2 - 1
    sw = None
    if weighted:
        sw = torch.rand(B, device=dev) * 2 - 1
        sw[::3] = 0
    ps = [t.double().requires_grad_() for t in (z, W1, b1, W2, b2)]
    h = ps[0] @ ps[1] + ps[2]
    h = {"linear": h, "relu": torch.relu(h), "tanh": torch.tanh(h)}[act]
    v = torch.tanh(h @ ps[3] + ps[4]).reshape(-1)
    per = (v - y.double()) ** 2
    if sw is not None:
        per = per * sw.double() / (sw != 0).double().mean()
    lref = per.mean()
    grads = torch.autograd.grad(lref, ps)
    g = [torch.full(t.shape, float("nan"), device=dev) for t in (W1, b1, W2, b2)]
    dz = torch.full((B, P), float("nan"), device=dev)
    vout = torch.empty(B, device=dev)
    loss = ops.value_mlp_train(z, W1, b1, W2, b2, y, sw, act, *g, dz=dz, vout=vout)
    torch.cuda.synchronize()
    assert abs(loss.sum().item() - lref.item()) < 1e-5 * max(1.0, abs(lref.item()))
    assert (vout - v.detach().float()).abs().max().item() < 1e-5
    for name, got, want in zip(["dz", "dW1", "db1", "dW2", "db2"], [dz] + g, grads):
        assert torch.isfinite(got).all(), name
        assert rel_err(got.reshape(want.shape), want.float()) < 1e-4, name


def test_sl_batch_prep(ops):
    """Fused per-step transform draw + transformed labels (batch.hip) vs torch indexing."""
    from rocalphago_amd.training.data import label_transform_table, transform_ids
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    labels = torch.randint(0, 361, (5000,), generator=g, device=dev)
    index = torch.randint(0, 5000, (256,), generator=g, device=dev)
    table = torch.from_numpy(label_transform_table(19)).to(dev)
    sym = torch.tensor(transform_ids(["noop", "rot90", "fliplr"]), dtype=torch.int32, device=dev)
    tf, lab = ops.sl_batch(index, labels, table, sym, seed=7, step=11)
    torch.cuda.synchronize()
    assert set(tf.cpu().tolist()) <= set(sym.cpu().tolist())
    assert len(set(tf.cpu().tolist())) == 3  # 256 draws hit every allowed transform
    assert torch.equal(lab, table[tf.long(), labels[index]])
    tf2, _ = ops.sl_batch(index, labels, table, sym, seed=7, step=11)
    tf3, _ = ops.sl_batch(index, labels, table, sym, seed=7, step=12)
    assert torch.equal(tf, tf2) and not torch.equal(tf, tf3)


@pytest.mark.gpu
@pytest.mark.parametrize("wmap", [0, 1])
def test_wgrad_slab_fp16_partials_match_fp32(ops, wmap):
    """wgrad_slab's default block-scaled fp16 partial slabs (MFMA C layout + reduce) vs the
    fp32 part[chunk][tap][n][c] path and fp32 PyTorch, accumulating, for both wave->tile maps."""
    dev = torch.device("cuda")
    torch.manual_seed(5)
    B, C, S = 64, 192, 19
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    g = torch.randn(B, C, S, S, device=dev)
    ref = torch.nn.grad.conv2d_weight(bf(x), (C, C, 3, 3), bf(g), padding=1)
    xp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(g, 1, C)
    lib = ops._lib()
    out = {}
    prev_map = lib.rag_wgrad_slab_map(wmap)
    for mode in (1, 0):
        prev = lib.rag_wgrad_slab_part_bf16(mode)
        try:
            dw = torch.full((C, C, 3, 3), 0.5, device=dev)
            db = torch.full((C,), 0.5, device=dev)
            ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, accumulate=True, hg=1)
            ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, accumulate=True, hg=1)
            torch.cuda.synchronize()
            out[mode] = (dw - 0.5, db - 0.5)
        finally:
            lib.rag_wgrad_slab_part_bf16(prev)
    lib.rag_wgrad_slab_map(prev_map)
    for mode in (1, 0):
        assert rel_err(out[mode][0], 2 * ref) < 1e-2
        assert rel_err(out[mode][1], 2 * bf(g).sum((0, 2, 3))) < 1e-2
    print("fp16-vs-fp32 partials rel err", rel_err(out[1][0], out[0][0]))
    assert rel_err(out[1][0], out[0][0]) < 1e-3


@pytest.mark.gpu
def test_deferred_wgrad_reduce_fused_into_dgrad(ops):
    """conv_wgrad(defer=True) leaves the bf16 partial-slab reduction pending; the next conv_igemm
    (a tap-slab dgrad) runs it in extra blocks, or wgrad_flush() launches it. dW / db equal the
    standalone reduction and the dgrad output is unchanged."""
    dev = torch.device("cuda")
    torch.manual_seed(9)
    B, C, S = 64, 192, 19
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    g = torch.randn(B, C, S, S, device=dev)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    xp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(g, 1, C)
    _, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    ref_dw, ref_db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
    ops.conv_wgrad(gp, xp, ref_dw, ref_db, B, S, 1, C, C, C, C, 3, hg=1)
    ref_dx = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(gp, wb, None, ref_dx, B, S, 1, 1, C, C, 3, False, mask=xp)
    # fused into the dgrad launch
    h = ops.PendingReduction()
    dw, db = torch.full((C, C, 3, 3), 7.0, device=dev), torch.full((C,), 7.0, device=dev)
    ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=h)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(gp, wb, None, dx, B, S, 1, 1, C, C, 3, False, mask=xp, pending=h)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)
    assert rel_err(dw, ref_dw) < 1e-5 and rel_err(db, ref_db) < 1e-5
    # explicit flush, accumulating on top
    ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, accumulate=True, hg=1, defer=True,
                   pending=h)
    ops.wgrad_flush(h)
    ops.wgrad_flush(h)  # nothing pending: no-op
    torch.cuda.synchronize()
    assert rel_err(dw, 2 * ref_dw) < 1e-5 and rel_err(db, 2 * ref_db) < 1e-5


@pytest.mark.gpu
def test_deferred_reductions_of_two_trunks_interleave_on_one_stream(ops):
    """Each trunk owns its pending-reduction handle: launches of another network (or without a
    handle) on the same stream neither run nor drop it."""
    dev = torch.device("cuda")
    torch.manual_seed(11)
    B, C, S = 32, 192, 19
    nets = []
    for k in range(2):
        x = F.relu(torch.randn(B, C, S, S, device=dev))
        g = torch.randn(B, C, S, S, device=dev)
        w = torch.randn(C, C, 3, 3, device=dev) * 0.05
        xp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(g, 1, C)
        _, wb = ops.pack_weights(w, C, C,
                                 wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
        rdw, rdb = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
        ops.conv_wgrad(gp, xp, rdw, rdb, B, S, 1, C, C, C, C, 3, hg=1)
        nets.append((xp, gp, wb, rdw, rdb))
    torch.cuda.synchronize()
    ha, hb = ops.PendingReduction(), ops.PendingReduction()
    (xa, ga, wba, rdwa, rdba), (xb, gb, wbb, rdwb, rdbb) = nets
    dwa, dba = torch.zeros_like(rdwa), torch.zeros_like(rdba)
    dwb, dbb = torch.zeros_like(rdwb), torch.zeros_like(rdbb)
    wsa = ops.wgrad_workspace(B, S, C, C, 3, dev).clone()  # separate partial-slab workspaces
    wsb = ops.wgrad_workspace(B, S, C, C, 3, dev).clone()
    ops.conv_wgrad(ga, xa, dwa, dba, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=ha,
                   work=wsa)
    # trunk B's wgrad + dgrad and a handle-less launch run in between: A's reduction waits
    ops.conv_wgrad(gb, xb, dwb, dbb, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=hb,
                   work=wsb)
    dxb = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(gb, wbb, None, dxb, B, S, 1, 1, C, C, 3, False, mask=xb, pending=hb)
    ops.conv_igemm(ga, wba, None, ops.alloc_padded(B, S, 1, C, dev), B, S, 1, 1, C, C, 3, False)
    torch.cuda.synchronize()
    assert rel_err(dwb, rdwb) < 1e-5 and rel_err(dbb, rdbb) < 1e-5
    assert float(dwa.abs().max()) == 0.0, "A's reduction must still be pending"
    dxa = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(ga, wba, None, dxa, B, S, 1, 1, C, C, 3, False, mask=xa, pending=ha)
    torch.cuda.synchronize()
    assert rel_err(dwa, rdwa) < 1e-5 and rel_err(dba, rdba) < 1e-5


@pytest.mark.gpu
def test_trunk_repack_matches_per_layer_packer(ops):
    """pack_trunk (one launch, 16x16 all-tap tiles through LDS) equals pack_weights per layer for
    both bf16 GEMM layouts and the padded biases: a 7x7 and a 5x5 input layer, odd widths, 3x3
    layers, a 1x1 head."""
    from rocalphago_amd.models.engine import ConvSpec, HipTrunk
    dev = torch.device("cuda")
    torch.manual_seed(4)
    specs = [ConvSpec(7, 48, 48, True), ConvSpec(5, 48, 192, True),
             ConvSpec(3, 192, 192, True), ConvSpec(3, 192, 40, True),
             ConvSpec(3, 40, 64, True), ConvSpec(1, 64, 1, False)]
    tr = HipTrunk(specs, 19, dev)
    ws = [torch.randn(s.cout, s.cin, s.ks, s.ks, device=dev) for s in specs]
    bs = [torch.randn(s.cout, device=dev) for s in specs]
    tr.sync_weights(ws, bs, 1)
    # the 192 -> 192 layer is a Winograd layer: its fragment-major Winograd weights come with
    # every repack (and its direct dgrad layout while the dgrad carries deferred reductions),
    # its direct forward layout on first demand
    assert tr._wino == [False, False, True, False, False, False]
    for l in (2,):
        uf, ub = ops.wino_weights(ws[l], 192, 192)
        assert torch.equal(tr._uf[l], uf)
        assert (tr._ub[l] is None) if not tr.wino_dgrad else torch.equal(tr._ub[l], ub)
    tr._direct_layouts()
    torch.cuda.synchronize()
    for l, s in enumerate(specs):
        wb = torch.empty(s.ks * s.ks, s.cinp, s.coutp, dtype=torch.bfloat16, device=dev)
        wf, wb = ops.pack_weights(ws[l], s.coutp, s.cinp, wb=wb)
        assert torch.equal(tr._wf[l], wf), l
        # the trunk input takes no gradient: no dgrad layout for layer 0
        assert (tr._wb[l] is None) if l == 0 else torch.equal(tr._wb[l], wb), l
        ref_b = torch.zeros(s.coutp, device=dev)
        ref_b[:s.cout] = bs[l]
        assert torch.equal(tr._bias[l], ref_b), l


@pytest.mark.gpu
def test_one_launch_repack_matches_separate_launches(ops):
    """pack_step (conv_wino.hip: the Winograd rows, the pack_trunk rows and the rest of the flat
    buffer's SGD in one launch) writes bit for bit what wino_pack + pack_trunk + sgd_kernel write:
    the packed layouts and biases, and the stepped fp32 masters, with and without the fold."""
    from rocalphago_amd.models.engine import ConvSpec, HipTrunk, complement
    dev = torch.device("cuda")
    specs = [ConvSpec(5, 48, 192, True), ConvSpec(3, 192, 192, True), ConvSpec(3, 192, 192, True),
             ConvSpec(3, 192, 40, True), ConvSpec(1, 40, 4, False)]
    sizes = [s.cout * s.cin * s.ks * s.ks for s in specs]

    def packed(tr):
        # what a repack writes: the direct layouts of the non-Winograd layers (a Winograd layer's
        # direct forward layout is packed on first demand only), the Winograd weights, the direct
        # dgrad layouts of layers 1.. (the Winograd layers' out of their wino_pack rows), biases
        d = {}
        for l in range(len(specs)):
            if not tr._wino[l]:
                d["wf%d" % l] = tr._wf[l].clone()
            else:
                d["uf%d" % l] = tr._uf[l].clone()
            if l > 0:
                d["wb%d" % l] = tr._wb[l].clone()
            d["b%d" % l] = tr._bias[l].clone()
        return d

    out = []
    for one in (True, False):
        torch.manual_seed(5)
        # flat buffer: a head-like block in front, the trunk's weights and biases, a tail block
        # (every range 16-byte aligned: sgd_kernel's float4 accesses)
        n = 780 + sum(sizes) + sum(s.cout for s in specs) + 332
        flat = torch.randn(n, device=dev)
        grad = torch.randn(n, device=dev)
        ws, bs, p = [], [], 780
        for s, k in zip(specs, sizes):
            ws.append(flat[p:p + k].view(s.cout, s.cin, s.ks, s.ks))
            p += k
            bs.append(flat[p:p + s.cout])
            p += s.cout
        tr = HipTrunk(specs, 19, dev)
        tr.ONE_LAUNCH = one
        assert tr._wino == [False, True, True, False, False]
        tr.sync_weights(ws, bs, 1)
        torch.cuda.synchronize()
        p1 = packed(tr)
        ranges = tr.sgd_pack(ws, bs, flat, grad, 0.05, 2, step_rest=True)
        rest = complement(ranges, n)
        assert rest == ([] if one else [(0, 780), (n - 332, n)])
        for a, b in rest:  # what fused.sgd_fold does with the rest
            ops.sgd_(flat[a:b], grad[a:b], 0.05)
        torch.cuda.synchronize()
        assert tr._wb[0] is None
        out.append((p1, flat.clone(), packed(tr)))
    (pa, fa, qa), (pb, fb, qb) = out
    for k in pa:
        assert torch.equal(pa[k], pb[k]), k
    assert torch.equal(fa, fb)
    for k in qa:
        assert torch.equal(qa[k], qb[k]), k


@pytest.mark.gpu
def test_wgrad_denormal_scale_gradients_stay_finite(ops):
    """Block-scaled fp16 partial slabs with a block max near 2^-110 (dead / vanishing channels):
    the scale exponent is floored, so dW stays finite and proportional (2^(14-e)
    overflowed to inf, turning zeros into NaN)."""
    dev = torch.device("cuda")
    torch.manual_seed(13)
    B, C, S = 16, 192, 19
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    g = torch.randn(B, C, S, S, device=dev)
    g[:, :64] = 0.0  # exact zeros next to tiny values
    xp = ops.pack_nchw(x, 1, C)
    ref_dw, ref_db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
    ops.conv_wgrad(ops.pack_nchw(g, 1, C), xp, ref_dw, ref_db, B, S, 1, C, C, C, C, 3, hg=1)
    tiny = 2.0 ** -112
    dw, db = torch.zeros_like(ref_dw), torch.zeros_like(ref_db)
    ops.conv_wgrad(ops.pack_nchw(g * tiny, 1, C), xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1)
    torch.cuda.synchronize()
    assert torch.isfinite(dw).all() and torch.isfinite(db).all()
    assert rel_err(dw / tiny, ref_dw) < 5e-2


@pytest.mark.gpu
def test_width128_pingpong_conv_and_wgrad_slab(ops):
    """128-channel 3x3 layers (ResnetPolicy / the reference CNNPolicy default width) at B = 256:
    the ping-pong tap kernel with 96 x 64 wave tiles (forward with bias + ReLU, residual
    sum-merge, dgrad with the ReLU mask) and the 8-wave wgrad slab kernel with its reduction
    deferred into that dgrad, each against fp32 PyTorch on bf16-rounded operands."""
    dev = torch.device("cuda")
    torch.manual_seed(11)
    B, C, S = 256, 128, 19
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = torch.randn(B, C, S, S, device=dev)
    g = torch.randn(B, C, S, S, device=dev)
    xp, gp = ops.pack_nchw(x, 1, C), ops.pack_nchw(g, 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    y = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(xp, wf, b, y, B, S, 1, 1, C, C, 3, relu=True)
    assert rel_err(ops.unpack(y, C, 1), F.relu(F.conv2d(bf(x), bf(w), b, padding=1))) < 2e-2
    assert y[:, 0].abs().max().item() == 0 and y[:, :, -1].abs().max().item() == 0
    rp = ops.pack_nchw(r, 1, C)
    yr = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(xp, wf, None, yr, B, S, 1, 1, C, C, 3, relu=False, residual=rp)
    assert rel_err(ops.unpack(yr, C, 1), F.conv2d(bf(x), bf(w), padding=1) + bf(r)) < 2e-2
    # wgrad (deferred) + dgrad with the ReLU mask of the layer input, twice on one handle: the
    # claimed reduction's counters must be back at zero for the second launch (a
    # missed reset would skip the whole second reduction and leave dw / db at their NaN fill)
    xr, wr = bf(x).requires_grad_(), bf(w).requires_grad_()
    (F.conv2d(xr, wr, padding=1) * bf(g)).sum().backward()
    h = ops.PendingReduction()
    for rnd in range(2):
        dw = torch.full((C, C, 3, 3), float("nan"), device=dev)
        db = torch.full((C,), float("nan"), device=dev)
        ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=h)
        dx = ops.alloc_padded(B, S, 1, C, dev)
        ops.conv_igemm(gp, wb, None, dx, B, S, 1, 1, C, C, 3, relu=False, mask=xp, pending=h)
        torch.cuda.synchronize()
        assert rel_err(ops.unpack(dx, C, 1), xr.grad * (x > 0)) < 2e-2
        assert rel_err(dw, wr.grad) < 1e-2, "round %d" % rnd
        assert rel_err(db, bf(g).sum((0, 2, 3))) < 1e-2, "round %d" % rnd


@pytest.mark.gpu
@pytest.mark.parametrize("B,cin,cout", [(256, 48, 192), (256, 128, 128), (7, 48, 192)])
def test_wgrad_slab_5x5_rows(ops, B, cin, cout):
    """5x5 weight gradients on the slab kernel (one kernel row per block, fp16 partials; the
    SL input layer 48->192 and ResnetPolicy's first unit 128->128) against fp32 PyTorch and the
    all-taps kernel (RAG_WGRAD_SLAB5 path off), standalone and deferred into a dgrad."""
    dev = torch.device("cuda")
    torch.manual_seed(17)
    S = 19
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    x = F.relu(torch.randn(B, cin, S, S, device=dev))
    g = torch.randn(B, cout, S, S, device=dev)
    ref = torch.nn.grad.conv2d_weight(bf(x), (cout, cin, 5, 5), bf(g), padding=2)
    xp, gp = ops.pack_nchw(x, 2, cinp), ops.pack_nchw(g, 2, coutp)
    dw = torch.full((cout, cin, 5, 5), 0.25, device=dev)
    db = torch.full((cout,), 0.25, device=dev)
    ops.conv_wgrad(gp, xp, dw, db, B, S, 2, cout, coutp, cin, cinp, 5, accumulate=True, hg=2)
    h = ops.PendingReduction()
    ops.conv_wgrad(gp, xp, dw, db, B, S, 2, cout, coutp, cin, cinp, 5, accumulate=True, hg=2,
                   defer=True, pending=h)
    ops.wgrad_flush(h)
    torch.cuda.synchronize()
    assert rel_err(dw - 0.25, 2 * ref) < 1e-2
    assert rel_err(db - 0.25, 2 * bf(g).sum((0, 2, 3))) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout", [(48, 192), (128, 128)])
def test_pingpong_conv_5x5(ops, cin, cout):
    """5x5 layers at B = 256 on the ping-pong kernel (25 taps per channel chunk): the SL input
    layer 48->192 (bias + ReLU) and ResnetPolicy's first unit 128->128 (residual forward, dgrad
    with the ReLU mask), against fp32 PyTorch on bf16-rounded operands."""
    dev = torch.device("cuda")
    torch.manual_seed(19)
    B, S = 256, 19
    cinp, coutp = ops.pad_channels(cin), ops.pad_channels(cout)
    x = F.relu(torch.randn(B, cin, S, S, device=dev))
    w = torch.randn(cout, cin, 5, 5, device=dev) * 0.03
    b = torch.randn(cout, device=dev) * 0.1
    xp = ops.pack_nchw(x, 2, cinp)
    wf, wb = ops.pack_weights(w, coutp, cinp, wb=torch.empty(25, cinp, coutp,
                                                              dtype=torch.bfloat16, device=dev))
    bias = torch.zeros(coutp, device=dev)
    bias[:cout] = b
    y = ops.alloc_padded(B, S, 1, coutp, dev)
    ops.conv_igemm(xp, wf, bias, y, B, S, 2, 1, cinp, coutp, 5, relu=True)
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=2))
    assert rel_err(ops.unpack(y, cout, 1), ref) < 2e-2
    assert y[:, 0].abs().max().item() == 0 and y[:, :, -1].abs().max().item() == 0
    if cin == cout:
        r = torch.randn(B, cout, S, S, device=dev)
        rp = ops.pack_nchw(r, 1, coutp)
        yr = ops.alloc_padded(B, S, 1, coutp, dev)
        ops.conv_igemm(xp, wf, None, yr, B, S, 2, 1, cinp, coutp, 5, relu=False, residual=rp)
        assert rel_err(ops.unpack(yr, cout, 1), F.conv2d(bf(x), bf(w), padding=2) + bf(r)) < 2e-2
        g = torch.randn(B, cout, S, S, device=dev)
        xr = bf(x).requires_grad_()
        (F.conv2d(xr, bf(w), padding=2) * bf(g)).sum().backward()
        gp = ops.pack_nchw(g, 2, coutp)
        dx = ops.alloc_padded(B, S, 1, cinp, dev)
        xm = ops.pack_nchw(x, 1, cinp)
        ops.conv_igemm(gp, wb, None, dx, B, S, 2, 1, coutp, cinp, 5, relu=False, mask=xm)
        assert rel_err(ops.unpack(dx, cin, 1), xr.grad * (x > 0)) < 2e-2


@pytest.mark.gpu
def test_pingpong_conv_192px_blocks_residual_and_dgrad(ops):
    """B = 128 (a self-play pipeline group): 121 blocks of 384 pixels would leave half the chip
    idle, so the 3x3 layers run the ping-pong kernel on 192-pixel blocks (MT = 3). Forward with
    the residual sum-merge (register epilogue) and the masked dgrad (LDS epilogue) vs fp32."""
    dev = torch.device("cuda")
    torch.manual_seed(21)
    B, C, S = 128, 192, 19
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    r = torch.randn(B, C, S, S, device=dev)
    xp = ops.pack_nchw(x, 1, C)
    wf, wb = ops.pack_weights(w, C, C, wb=torch.empty(9, C, C, dtype=torch.bfloat16, device=dev))
    y = ops.pack_nchw(r, 1, C)  # residual in place
    ops.conv_igemm(xp, wf, b.contiguous(), y, B, S, 1, 1, C, C, 3, relu=True, residual=y)
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=1) + bf(r))
    assert rel_err(ops.unpack(y, C, 1), ref) < 2e-2
    g = torch.randn(B, C, S, S, device=dev)
    gp = ops.pack_nchw(g, 1, C)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_igemm(gp, wb, None, dx, B, S, 1, 1, C, C, 3, relu=False, mask=xp)
    xr = bf(x).requires_grad_()
    (F.conv2d(xr, bf(w), padding=1) * bf(g)).sum().backward()
    assert rel_err(ops.unpack(dx, C, 1), xr.grad * (x > 0)) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("K,KP,B", [(192, 192, 256), (128, 128, 64), (256, 256, 3), (40, 40, 7),
                                    (36, 40, 5)])
def test_head_linear_matches_fp32(ops, K, KP, B):
    """The value head's 1x1 convolution (head.hip head_linear_kernel: weights held in registers
    for K a multiple of 8 up to 256, the generic loop otherwise) against fp32 PyTorch on the
    same bf16-rounded inputs, including the padded channels past K."""
    dev = torch.device("cuda")
    torch.manual_seed(21)
    S = 19
    h = F.relu(torch.randn(B, K, S, S, device=dev))
    hp = ops.pack_nchw(h, 1, KP)
    if KP > K:  # garbage in the padded channels must not leak into z
        hp[..., K:] = 1.0
    w = torch.randn(K, device=dev)
    b0 = torch.randn(1, device=dev)
    z = torch.empty(B, S * S, device=dev)
    ops.head_linear(hp, w, b0, z, K)
    hb = h.to(torch.bfloat16).float()
    ref = (hb * w.view(1, K, 1, 1)).sum(1).reshape(B, S * S) + b0
    assert torch.allclose(z, ref, rtol=1e-4, atol=1e-3), (z - ref).abs().max().item()


@pytest.mark.gpu
def test_pending_handle_dropped_inside_capture_keeps_the_capture_valid(ops):
    """A PendingReduction whose owner dies during a HIP graph capture (the cyclic GC dropping a
    dead trunk mid-capture) defers its hipFree: the capture stays valid, and the next handle
    created frees it."""
    from rocalphago_amd.ops import hipops
    h = ops.PendingReduction()
    x = torch.zeros(4, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
            x.add_(1)
            del h
            x.add_(1)
    assert len(hipops._DEFERRED_FREE) == 1
    g.replay()
    torch.cuda.synchronize()
    assert x.tolist() == [2.0] * 4
    ops.PendingReduction()
    assert not hipops._DEFERRED_FREE

