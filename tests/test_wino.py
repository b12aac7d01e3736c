"""Winograd F(2,3) 3x3 convolution (csrc/hip/conv_wino.hip) against fp32 PyTorch (GPU only).

The kernel computes the reference's 3x3 Convolution2D (policy.py:96-136) as four width-wise
Winograd GEMMs: the inputs are bf16, the transformed inputs V = d_a +- d_b are rounded to bf16
once, the weights U = G g once, and everything accumulates in fp32. That adds one rounding per
operand to the direct kernel's arithmetic: ~0.3 % relative (norm) error against an fp32
convolution of the same bf16 inputs, against ~0.2 % for the bf16 output rounding alone."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def bf(t):
    return t.to(torch.bfloat16).float()


def rel_max(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def rel_norm(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rocalphago_amd.ops import hipops
    return hipops


@pytest.mark.parametrize("B,S,ho,C", [(1, 19, 1, 192), (3, 19, 2, 192), (256, 19, 1, 192),
                                      (3, 13, 1, 192), (5, 9, 1, 192), (7, 7, 2, 192),
                                      (3, 19, 1, 128), (256, 19, 2, 128), (128, 19, 1, 192),
                                      (120, 19, 2, 192), (200, 19, 1, 192)])
def test_wino_forward_matches_fp32(ops, B, S, ho, C):
    """192-wide tiles (one or several boards per block), the 128-wide tile (CNNPolicy's
    default width: 48 pairs x 64 channels per wave) and half-board blocks (B <= 128 at 19x19 on
    256 CUs: two 96-pair blocks per board; B = 200: one wave of one-board blocks)."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    assert ops.conv_wino_ok(S, 1, C, C, 3)
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=1))
    if B in (120, 128) and ops.conv_wino_mode(B, S, C, C) != 2:
        pytest.skip("half-board blocks are chosen for B = %d on 256 CUs only" % B)
    xp = ops.pack_nchw(x, 1, C)
    uf, _ = ops.wino_weights(w, C, C, dgrad=False)
    # one extra board past B: the kernel must not touch it
    y = ops.alloc_padded(B + 1, S, ho, C, dev)
    ops.conv_wino(xp, uf, b.contiguous(), y[:B], B, S, C, C, ho, True)
    out = ops.unpack(y[:B], C, ho)
    assert rel_norm(out, ref) < 6e-3
    assert rel_max(out, ref) < 2e-2
    # the output halo and the board past B stay zero
    assert y[B].abs().max().item() == 0
    assert y[:, :ho].abs().max().item() == 0 and y[:, :, -ho:].abs().max().item() == 0
    # and it agrees with the direct implicit-GEMM kernel on the same inputs
    wf, _ = ops.pack_weights(w, C, C)
    yd = ops.alloc_padded(B, S, ho, C, dev)
    ops.conv_igemm(xp, wf, b.contiguous(), yd, B, S, 1, ho, C, C, 3, relu=True)
    assert rel_norm(out, ops.unpack(yd, C, ho)) < 6e-3


@pytest.mark.parametrize("B", [1, 64, 128])
def test_wino_half_board_blocks_match_fp32(ops, B):
    """Small one-wave batches (the self-play plies, the search's partial waves) run half-board
    blocks (two 96-pair blocks per board, all 192 output channels): forward with bias + ReLU
    and dgrad with the ReLU mask against fp32 F.conv2d."""
    dev = torch.device("cuda")
    torch.manual_seed(1)
    S, C = 19, 192
    if ops.conv_wino_mode(B, S, C, C) != 2:
        pytest.skip("half-board blocks are chosen for B <= 128 on 256 CUs only")
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    b = torch.randn(C, device=dev) * 0.1
    xp = ops.pack_nchw(x, 1, C)
    uf, ub = ops.wino_weights(w, C, C)
    y = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_wino(xp, uf, b.contiguous(), y, B, S, C, C, 1, True)
    ref = F.relu(F.conv2d(bf(x), bf(w), b, padding=1))
    out = ops.unpack(y, C, 1)
    assert rel_norm(out, ref) < 6e-3 and rel_max(out, ref) < 2e-2
    g = torch.randn(B, C, S, S, device=dev)
    dx = ops.alloc_padded(B, S, 1, C, dev)
    ops.conv_wino(ops.pack_nchw(g, 1, C), ub, None, dx, B, S, C, C, 1, False, mask=xp)
    xr = bf(x).requires_grad_()
    F.conv2d(xr, bf(w), None, padding=1).backward(bf(g))
    ref_dx = xr.grad * (bf(x) > 0)
    assert rel_norm(ops.unpack(dx, C, 1), ref_dx) < 6e-3
    assert dx[:, :1].abs().max().item() == 0 and dx[:, :, -1:].abs().max().item() == 0


@pytest.mark.parametrize("B,S,ho,C", [(3, 19, 1, 192), (2, 19, 2, 192), (4, 13, 1, 192),
                                      (3, 19, 1, 128), (128, 19, 2, 192)])
def test_wino_dgrad_with_mask_matches_autograd(ops, B, S, ho, C):
    """dgrad form: the Winograd weights of the flipped, transposed kernel (Ub) and the ReLU
    mask of the layer input in the epilogue, output halo 1 or 2 (the SL trunk's layer-1 dgrad
    writes the 5x5 input layer's halo-2 gradient)."""
    dev = torch.device("cuda")
    torch.manual_seed(1)
    x = F.relu(torch.randn(B, C, S, S, device=dev))
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    g = torch.randn(B, C, S, S, device=dev)
    xr = bf(x).requires_grad_()
    (F.conv2d(xr, bf(w), padding=1) * bf(g)).sum().backward()
    ref = xr.grad * (x > 0)
    gp = ops.pack_nchw(g, 1, C)
    xm = ops.pack_nchw(x, ho, C)
    _, ub = ops.wino_weights(w, C, C)
    dx = ops.alloc_padded(B, S, ho, C, dev)
    ops.conv_wino(gp, ub, None, dx, B, S, C, C, ho, False, mask=xm, mask_halo=ho)
    out = ops.unpack(dx, C, ho)
    assert rel_norm(out, ref) < 6e-3
    assert rel_max(out, ref) < 2e-2


def unfrag(u, N, K):
    """Fragment-major [12][K/32][N/16][64 lanes][8] -> [12][N][K] (lane = n%16 + 16 (k%32)/8)."""
    return u.reshape(12, K // 32, N // 16, 4, 16, 8).permute(0, 2, 4, 1, 3, 5).reshape(12, N, K)


def test_wino_pack_layouts(ops):
    """Uf[ky*4+q] = G[q] . w[:, :, ky, :] and Ub the same of w[:, :, 2-ky, ::-1] transposed,
    with zero padding past (cout, cin), both stored fragment-major."""
    dev = torch.device("cuda")
    torch.manual_seed(2)
    cout, cin, coutp, cinp = 150, 100, 192, 128
    w = torch.randn(cout, cin, 3, 3, device=dev)
    uf, ub = ops.wino_weights(w, coutp, cinp)
    uf, ub = unfrag(uf, coutp, cinp), unfrag(ub, cinp, coutp)
    G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], device=dev)
    ref = torch.einsum("qk,ncyk->yqnc", G, w).reshape(12, cout, cin)
    assert torch.equal(uf[:, :cout, :cin].float(), bf(ref))
    assert uf[:, cout:].abs().max().item() == 0 and uf[:, :, cin:].abs().max().item() == 0
    wflip = w.flip(2, 3).transpose(0, 1)  # [cin, cout, ky', kx']
    refb = torch.einsum("qk,cnyk->yqcn", G, wflip).reshape(12, cin, cout)
    assert torch.equal(ub[:, :cin, :cout].float(), bf(refb))


def test_wino_dgrad_carries_deferred_wgrad_reduction_twice(ops):
    """A deferred wgrad reduction rides in the Winograd dgrad launch (every block claims units
    of it after its epilogue; the last block resets the claim counters). Two rounds on the same
    handle: the second launch finds the counters reset and reduces again."""
    dev = torch.device("cuda")
    torch.manual_seed(3)
    B, S, C = 64, 19, 192
    h = ops.PendingReduction()
    ref_dw, ref_db = None, None
    for rnd in range(2):
        x = F.relu(torch.randn(B, C, S, S, device=dev))
        g = torch.randn(B, C, S, S, device=dev)
        xp = ops.pack_nchw(x, 1, C)
        gp = ops.pack_nchw(g, 1, C)
        w = torch.randn(C, C, 3, 3, device=dev) * 0.05
        _, ub = ops.wino_weights(w, C, C)
        # reference: non-deferred wgrad
        ref_dw = torch.zeros(C, C, 3, 3, device=dev)
        ref_db = torch.zeros(C, device=dev)
        ops.conv_wgrad(gp, xp, ref_dw, ref_db, B, S, 1, C, C, C, C, 3, hg=1)
        dw = torch.full((C, C, 3, 3), float("nan"), device=dev)
        db = torch.full((C,), float("nan"), device=dev)
        ops.conv_wgrad(gp, xp, dw, db, B, S, 1, C, C, C, C, 3, hg=1, defer=True, pending=h)
        dx = ops.alloc_padded(B, S, 1, C, dev)
        ops.conv_wino(gp, ub, None, dx, B, S, C, C, 1, False, mask=xp, pending=h)
        torch.cuda.synchronize()
        assert torch.isfinite(dw).all() and torch.isfinite(db).all(), "round %d" % rnd
        assert rel_max(dw, ref_dw) < 1e-5 and rel_max(db, ref_db) < 1e-5


def test_trunk_large_batch_dgrad_on_winograd(ops):
    """HipTrunk runs the dgrad of its Winograd layers on the Winograd kernel at batches of two or
    more block waves (wino_dgrad_min_batch; the deferred wgrad reduction then costs a few us in
    its last wave) with the Winograd dgrad weights packed on first use: its gradients match an
    fp32 CPU train step of the same network and batch (and so does the direct dgrad's)."""
    import numpy as np
    from rocalphago_amd.features.preprocessing import DEFAULT_FEATURES
    from rocalphago_amd.models import kerasish as KZ
    from rocalphago_amd.models.policy import CNNPolicy
    B = 600
    rs = np.random.RandomState(2)
    X = (rs.rand(B, 48, 19, 19) > 0.6).astype(np.uint8)
    Y = np.zeros((B, 361), np.float32)
    Y[np.arange(B), rs.randint(0, 361, B)] = 1
    grads = []
    for min_batch in (512, 10 ** 9):
        pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=4,
                        device="cuda", seed=5)
        trunk = pol.model._plan_for().trunk
        trunk.wino_dgrad_min_batch = min_batch
        pol.model.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
        pol.model.train_on_batch(X, Y)
        torch.cuda.synchronize()
        assert (trunk._ub_version is not None) == (min_batch == 512)
        grads.append(torch.cat([g.detach().reshape(-1).float() for g in pol.model.net._gviews]))
    ref = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=192, layers=4, device="cpu",
                    seed=5)
    ref.model.compile(loss="categorical_crossentropy", optimizer=KZ.SGD(lr=0.0))
    ref.model.train_on_batch(X, Y)
    r = torch.cat([g.detach().reshape(-1).float() for g in ref.model.net._gviews])
    cos = []
    for g in grads:  # Winograd dgrad, direct dgrad
        g = g.cpu()
        cos.append(torch.dot(g, r).item() / (g.norm().item() * r.norm().item()))
        assert abs(g.norm().item() / r.norm().item() - 1) < 2e-2
    # bf16 operands through four layers put either at a cosine of ~0.996 to fp32; the Winograd
    # roundings must not make it measurably worse than the direct kernel's
    assert cos[0] > 0.99 and cos[1] > 0.99, cos
    assert cos[0] >= cos[1] - 1e-3, cos
