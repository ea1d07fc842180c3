"""PixelSNAIL prior on the GPU (vq3d.pixelsnail: causal convs on the libvq3d conv engines,
attention.hip) against the reference's own outputs (tests/golden/psnail_*.npz) and, at the
published mid-level size, against a torch fp32 restatement of the attention.

Tolerances: fp32 path 1e-4 of each tensor's max (summation order only); bf16 path (bf16 conv
operands, fp32 residual streams as under the reference's autocast): logits / loss 3e-2, every
weight-tensor gradient 8e-2 of its max, the whole gradient vector 3e-2 relative L2 with cosine
>= 0.999, the scalar bias / scale gradients as one vector 0.1 relative L2; the attention kernel
in bf16 storage 2e-2.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

G = "tests/golden/"
CL = torch.channels_last_3d


def P_of(d, pre="p/"):
    return {k[len(pre):]: torch.tensor(d[k]) for k in d.files if k.startswith(pre)}


def rel(a, b):
    a = np.asarray(a.detach().float().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def load_params(mod, P, dev):
    sd = {k: v for k, v in P.items()}
    mod.load_state_dict(sd, strict=True)
    return mod.to(dev)


def stack_in(x, dev, dtype=torch.float32):
    """(3, b, c, d, h, w) -> list of 3 channels-last GPU tensors requiring grad"""
    return [torch.tensor(x[i]).to(dev, dtype).contiguous(memory_format=CL).requires_grad_(True) for i in range(3)]


@pytest.mark.parametrize("name,nh", [("psnail_attn_h2", 2), ("psnail_attn_h8", 8)])
def test_attention_golden(gpu, name, nh):
    from vq3d import pixelsnail as PS
    d = np.load(G + name + ".npz")
    att = PS.CausalAttention(dropout_prob=0.0, num_heads=nh).to(gpu)
    keys, queries, values = stack_in(d["q"], gpu), stack_in(d["k"], gpu), stack_in(d["v"], gpu)
    # the golden was made with the reference's binding: its `keys` parameter got d["q"]
    y = att.run(keys, queries, values)
    assert rel(torch.stack(y), d["y"]) < 1e-5
    torch.autograd.backward(y, [torch.tensor(d["gy"][i]).to(gpu).contiguous(memory_format=CL) for i in range(3)])
    assert rel(torch.stack([t.grad for t in keys]), d["gq"]) < 1e-4
    assert rel(torch.stack([t.grad for t in queries]), d["gk"]) < 1e-4
    assert rel(torch.stack([t.grad for t in values]), d["gv"]) < 1e-4


def _attn_ref(q, k, v, nh):
    """torch fp32 restatement (GPU), one stream: q, k (b, ck, n), v (b, cv, n)"""
    b, ck, n = q.shape
    cv = v.shape[1]
    fq = q.reshape(b, nh, ck // nh, n) * (ck // nh) ** -0.5
    fk = k.reshape(b, nh, ck // nh, n)
    fv = v.reshape(b, nh, cv // nh, n)
    logits = torch.matmul(fq.transpose(2, 3), fk)
    mask = torch.tril(torch.ones((n, n), dtype=torch.bool, device=q.device))
    w = torch.softmax(logits.masked_fill(~mask, float("-inf")), -1)
    return torch.matmul(w, fv.transpose(2, 3)).transpose(2, 3).reshape(b, cv, n)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
def test_attention_mid_level_size(gpu, dtype, tol):
    """the published mid level: 32 x 32 x 8 = 8,192 positions, 64 channels = 8 heads x 8"""
    from vq3d import pixelsnail as PS
    g = torch.Generator(device=gpu).manual_seed(0)
    dims, c, nh = (32, 32, 8), 64, 8
    q, k, v = (torch.randn((1, c) + dims, device=gpu, generator=g).to(dtype).contiguous(memory_format=CL)
               .requires_grad_(True) for _ in range(3))
    y = PS.CausalAttentionFn.apply(q, k, v, nh)
    gy = torch.randn(y.shape, device=gpu, generator=g).to(dtype)
    y.backward(gy)
    qf, kf, vf = (t.detach().float().reshape(1, c, -1).requires_grad_(True) for t in (q, k, v))
    yr = _attn_ref(qf, kf, vf, nh)
    yr.backward(gy.float().reshape(1, c, -1))
    assert rel(y.reshape(1, c, -1), yr.detach().cpu().numpy()) < tol
    for t, r in ((q, qf), (k, kf), (v, vf)):
        assert rel(t.grad.reshape(1, c, -1), r.grad.cpu().numpy()) < 2 * tol


@pytest.mark.parametrize("name,mask,k,bias", [("psnail_conv_b3", "B", 3, False), ("psnail_conv_a1", "A", 1, True),
                                              ("psnail_conv_b1", "B", 1, True)])
def test_causal_conv_golden(gpu, name, mask, k, bias):
    from vq3d import pixelsnail as PS
    d = np.load(G + name + ".npz")
    cin, cout = d["x"].shape[2], d["y"].shape[2]
    m = load_params(PS.CausalConv3dAdd(mask=mask, in_channels=cin, out_channels=cout, kernel_size=k, bias=bias),
                    P_of(d), gpu)
    xs = stack_in(d["x"], gpu)
    y = m.run(xs)
    assert rel(torch.stack(y), d["y"]) < 1e-5
    torch.autograd.backward(y, [torch.tensor(d["gy"][i]).to(gpu).contiguous(memory_format=CL) for i in range(3)])
    assert rel(torch.stack([t.grad for t in xs]), d["gx"]) < 1e-4
    for n, p in m.named_parameters():
        assert rel(p.grad, d["g/" + n]) < 1e-4, n


@pytest.mark.parametrize("name,mask,aux", [("psnail_block_a", "A", False), ("psnail_block_b_aux", "B", True)])
def test_causal_block_golden(gpu, name, mask, aux):
    from vq3d import pixelsnail as PS
    d = np.load(G + name + ".npz")
    c = d["x"].shape[2]
    m = load_params(PS.PreActFixupCausalResBlock(c, c, 3, mask=mask, dropout_prob=0.0, bottleneck_divisor=4, aux=aux),
                    P_of(d), gpu)
    xs = stack_in(d["x"], gpu)
    a = stack_in(d["aux"], gpu) if aux else None
    y = m.run(xs, a)
    assert rel(torch.stack(y), d["y"]) < 1e-5
    torch.autograd.backward(y, [torch.tensor(d["gy"][i]).to(gpu).contiguous(memory_format=CL) for i in range(3)])
    assert rel(torch.stack([t.grad for t in xs]), d["gx"]) < 1e-4
    if aux:
        assert rel(torch.stack([t.grad for t in a]), d["gaux"]) < 1e-4
    scale = max(np.abs(d["g/" + n]).max() for n, _ in m.named_parameters())
    for n, p in m.named_parameters():
        err = np.abs(p.grad.detach().cpu().numpy() - d["g/" + n]).max()
        assert err <= max(1e-4 * np.abs(d["g/" + n]).max(), 1e-5 * scale), n


@pytest.mark.parametrize("dtype,tol,gtol", [("fp32", 1e-4, 1e-3), ("bf16", 3e-2, 8e-2)])
def test_pixelsnail_model_golden(gpu, dtype, tol, gtol):
    """whole prior: logits, loss and every parameter gradient of a training step (dropout 0)"""
    from vq3d import pixelsnail as PS
    d = np.load(G + "psnail_model_32.npz")
    ne, md, nl, nb, bd = (int(c) for c in d["cfg"])
    args = PS.default_args(num_embeddings=[ne, 0], model_dim=md, num_layers_per_block=nl, num_blocks=nb,
                           bottleneck_divisor=bd, causal_dropout_prob=0.0, attention_dropout_prob=0.0, lr=1e-3)
    m = load_params(PS.PixelSNAIL(args, compute_dtype=dtype), P_of(d), gpu)
    m.train()
    data = torch.tensor(d["data"]).to(gpu)
    loss, _ = m.cross_entropy([data])
    loss.backward()
    with torch.no_grad():
        onehot = torch.nn.functional.one_hot(data.squeeze(1), ne).permute(0, 4, 1, 2, 3)
        logits = m.logits(onehot)
    print(dtype, "loss", float(loss), float(d["loss"]), "logits rel", rel(logits, d["logits"]))
    assert rel(logits, d["logits"]) < tol
    assert abs(float(loss) - float(d["loss"])) < tol * abs(float(d["loss"]))
    scale = max(np.abs(d["g/" + n]).max() for n, _ in m.named_parameters())
    worst = 0.0
    sc_mine, sc_ref, all_mine, all_ref = [], [], [], []
    for n, p in m.named_parameters():
        ref = d["g/" + n]
        mine = p.grad.detach().cpu().numpy()
        all_mine.append(mine.ravel())
        all_ref.append(ref.ravel())
        if p.numel() == 1 and dtype == "bf16":
            # a lone bias / scale gradient is a sum over every activation of terms that nearly
            # cancel: judged as one vector below (as in test_gpu_bf16_model.py)
            sc_mine.append(mine.ravel())
            sc_ref.append(ref.ravel())
            continue
        err = np.abs(mine - ref).max() / max(np.abs(ref).max(), 1e-3 * scale)
        worst = max(worst, err)
        assert err <= gtol, n
    print(dtype, "worst tensor gradient error (of max(|ref|, 1e-3 scale))", worst)
    a, b = np.concatenate(all_mine).astype(np.float64), np.concatenate(all_ref).astype(np.float64)
    l2 = np.linalg.norm(a - b) / np.linalg.norm(b)
    cos = a @ b / (np.linalg.norm(a) * np.linalg.norm(b))
    print(dtype, "whole gradient rel L2", l2, "cosine", cos)
    assert l2 <= (1e-4 if dtype == "fp32" else 3e-2) and cos >= 0.999
    if sc_mine:
        a, b = np.concatenate(sc_mine).astype(np.float64), np.concatenate(sc_ref).astype(np.float64)
        sl2 = np.linalg.norm(a - b) / np.linalg.norm(b)
        print(dtype, "scalar-parameter gradients as one vector: rel L2", sl2)
        assert sl2 <= 0.1


def test_attention_train_mode_golden(gpu):
    """training mode with dropout 0 (every exact-zero logit -> -1e3, pixel_model/layers.py:633-637)
    against the reference's CausalAttention in train mode on inputs with zeroed key rows"""
    from vq3d import pixelsnail as PS
    d = np.load(G + "psnail_attn_train.npz")
    nh = int(d["nh"])
    att = PS.CausalAttention(dropout_prob=0.0, num_heads=nh).to(gpu)
    att.train()
    keys, queries, values = stack_in(d["keys"], gpu), stack_in(d["queries"], gpu), stack_in(d["values"], gpu)
    y = att.run(keys, queries, values)
    assert rel(torch.stack(y), d["out"]) < 1e-5
    torch.autograd.backward(y, [torch.tensor(d["gy"][i]).to(gpu).contiguous(memory_format=CL) for i in range(3)])
    assert rel(torch.stack([t.grad for t in keys]), d["g_keys"]) < 1e-4
    assert rel(torch.stack([t.grad for t in queries]), d["g_queries"]) < 1e-4
    assert rel(torch.stack([t.grad for t in values]), d["g_values"]) < 1e-4


def _logit_hash(seed, ph, i, j):
    """attention.hip logit_hash restated in numpy (uint32 wrap-around arithmetic)"""
    M = np.uint64(0xFFFFFFFF)
    u = lambda v: np.asarray(v, dtype=np.uint64)  # noqa: E731
    s = u(seed)
    x = (s & M) ^ ((u(int(seed) >> 32) * u(0x9E3779B1)) & M) ^ ((u(ph) * u(0xC2B2AE3D)) & M) \
        ^ ((u(i) * u(0x85EBCA77)) & M) ^ ((u(j) * u(0x27D4EB2F)) & M)
    x = x & M
    x ^= x >> u(16)
    x = (x * u(0x7FEB352D)) & M
    x ^= x >> u(15)
    x = (x * u(0x846CA68B)) & M
    x ^= x >> u(16)
    return x


@pytest.mark.parametrize("p", [0.3, 0.5])
def test_attention_dropout_matches_oracle(gpu, p):
    """attention dropout p > 0 in training: the kernels drop logit (i, j) of (problem, head) when a
    hash of the device seed is below p 2^32 and scale the rest by 1 / (1 - p); the oracle
    (oracle/pixelsnail_cpu.causal_attention, the reference's dropout -> zero -> -1e3 semantics) is
    given that same mask.  Output and input gradients within 1e-4; the kept fraction within 2 % of
    1 - p; another seed draws another mask."""
    from oracle import pixelsnail_cpu as O
    from vq3d import pixelsnail as PS
    g = torch.Generator().manual_seed(3)
    b, c, nh, dims = 2, 16, 2, (4, 8, 8)
    n = dims[0] * dims[1] * dims[2]
    q, k, v = (torch.randn((b, c) + dims, generator=g) for _ in range(3))
    gy = torch.randn((b, c) + dims, generator=g)
    seed = 0x1234_5678_9ABC
    qd, kd, vd = (t.to(gpu).contiguous(memory_format=CL).requires_grad_(True) for t in (q, k, v))
    st = torch.tensor([seed], dtype=torch.int64, device=gpu)
    y = PS.CausalAttentionFn.apply(qd, kd, vd, nh, (p, st))
    y.backward(gy.to(gpu).contiguous(memory_format=CL))
    ii, jj = np.arange(n).reshape(n, 1), np.arange(n).reshape(1, n)
    thr = np.uint64(min(4294967295, int(p * 4294967296.0)))
    dropped = np.stack([np.stack([_logit_hash(seed, bb * nh + h, ii, jj) < thr for h in range(nh)])
                        for bb in range(b)])  # (b, nh, n, n)
    low = np.tril(np.ones((n, n), dtype=bool))
    kept = 1.0 - float((dropped & low).sum()) / float(low.sum() * b * nh)
    assert abs(kept - (1 - p)) < 0.02, kept
    qc, kc, vc = (t.clone().unsqueeze(0).requires_grad_(True) for t in (q, k, v))
    yr = O.causal_attention(kc, qc, vc, nh, train=True, p=p, dropped=torch.from_numpy(dropped).unsqueeze(0))
    yr.backward(gy.unsqueeze(0))
    assert rel(y, yr.detach()[0].numpy()) < 1e-4
    assert rel(qd.grad, qc.grad[0].numpy()) < 1e-4
    assert rel(kd.grad, kc.grad[0].numpy()) < 1e-4
    assert rel(vd.grad, vc.grad[0].numpy()) < 1e-4
    y2 = PS.CausalAttentionFn.apply(qd, kd, vd, nh, (p, st + 1))
    assert rel(y2, y.detach().cpu().numpy()) > 1e-3


def test_published_mid_prior_step(gpu):
    """The published mid-level prior (train_pixelsnail_mid_downscaled.job:76-90: K = 256, model-dim
    256, 8 blocks x 5 layers, causal dropout 0.2, attention dropout 0, mixup 0.2, batch 1) on 32 x 32
    x 8 codes, bf16: two training steps (forward with mixup, backward, Adam) with finite loss and
    gradients, and the first block's attention inside the step equal, on 64 sampled query
    positions, to the CPU oracle's restatement (training-mode logits) of the same q / k / v."""
    from oracle import pixelsnail_cpu as O
    from vq3d import pixelsnail as PS
    from vq3d.flat import FlatParams
    from vq3d.optim import FusedAdam
    torch.manual_seed(0)
    args = PS.default_args(num_embeddings=[256, 0], model_dim=256, num_blocks=8, num_layers_per_block=5,
                           causal_dropout_prob=0.2, attention_dropout_prob=0.0, bottleneck_divisor=4,
                           mixup_alpha=0.2, lr=5e-5)
    m = PS.PixelSNAIL(args, compute_dtype="bf16").to(gpu)
    flat = FlatParams(m.parameters(), gpu)
    opt = FusedAdam(m.parameters(), flat, lr=5e-5, amsgrad=True)
    m.train()
    data = torch.randint(0, 256, (1, 1, 32, 32, 8), generator=torch.Generator().manual_seed(1)).to(gpu)
    seen = []
    orig = PS.CausalAttentionFn.apply

    def spy(q, k, v, nh, train=None):
        out = orig(q, k, v, nh, train)
        if not seen:
            seen.append(tuple(t.detach().float().cpu() for t in (q, k, v, out)) + (nh,))
        return out
    PS.CausalAttentionFn.apply = spy
    try:
        losses = []
        for _ in range(2):
            opt.zero_grad()
            loss = m.training_step([data], 0)
            loss.backward()
            opt.step()
            torch.cuda.synchronize()
            losses.append(float(loss))
            assert all(torch.isfinite(p.grad).all() for p in m.parameters())
    finally:
        PS.CausalAttentionFn.apply = orig
    assert all(np.isfinite(losses)) and 3.0 < losses[0] < 12.0, losses
    q, k, v, out, nh = seen[0]
    n = 32 * 32 * 8
    rows = np.sort(np.random.default_rng(0).choice(n, 64, replace=False))
    rows[0] = 0  # the first position attends to itself only
    ref = O.causal_attention_rows(k.unsqueeze(0), q.unsqueeze(0), v.unsqueeze(0), nh, rows, train=True)[0]
    got = out.reshape(out.shape[0], out.shape[1], -1)[..., torch.as_tensor(rows)]
    print("published prior losses", losses, "attention rel", rel(got, ref.numpy()))
    assert rel(got, ref.numpy()) < 2e-2  # bf16 q / k / v / out storage, fp32 arithmetic


def test_prior_step_with_mixup_captures(gpu):
    """bench.py --prior captures the training step (mixup forward, backward, Adam) as a HIP graph: no
    host-to-device copy may happen inside it; one replay gives the same loss as the eager step."""
    from vq3d import pixelsnail as PS
    from vq3d.flat import FlatParams
    from vq3d.optim import FusedAdam
    torch.manual_seed(0)
    args = PS.default_args(num_embeddings=[16, 0], model_dim=32, num_blocks=2, num_layers_per_block=2,
                           causal_dropout_prob=0.0, attention_dropout_prob=0.0, mixup_alpha=0.2)
    m = PS.PixelSNAIL(args, compute_dtype="bf16").to(gpu)
    flat = FlatParams(m.parameters(), gpu)
    opt = FusedAdam(m.parameters(), flat, lr=0.0, amsgrad=True)  # lr 0: replays see the same weights
    m.train()
    codes = torch.randint(0, 16, (1, 8, 8, 4), generator=torch.Generator().manual_seed(2)).to(gpu)
    onehot = torch.nn.functional.one_hot(codes, 16).permute(0, 4, 1, 2, 3).contiguous()
    mix = (0.3, torch.zeros(1, dtype=torch.int64))

    def step():
        opt.zero_grad()
        loss, _ = m.cross_entropy_onehot(onehot.float(), codes, mix)
        loss.backward()
        opt.step()
        return loss
    eager = float(step().detach())
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static = step()
    graph.replay()
    torch.cuda.synchronize()
    assert np.isfinite(eager) and abs(float(static.detach()) - eager) <= 1e-6 * abs(eager), (eager, float(static))


@pytest.mark.parametrize("dims,p", [((4, 8, 8), 0.3), ((3, 5, 7), 0.0), ((3, 5, 7), None), ((2, 16, 9), 0.5)])
def test_attention_matrix_core_matches_valu(gpu, dims, p):
    """The 16-bit builds' matrix-core attention (head dim 8: forward and both backward kernels)
    against the fp32 VALU kernels (pinned by the oracle above) on the same bf16-representable
    inputs: eval (p None), training without dropout (p 0: the zero-logit replacement) and with
    dropout (the same device-seeded mask), odd position counts (partial 32- and 128-row tiles).
    Output and gradients within 2e-2 / 4e-2 relative (fp16 P / dS operands, bf16 storage)."""
    from vq3d import pixelsnail as PS
    g = torch.Generator().manual_seed(11)
    b, c, nh = 2, 16, 2
    src = [torch.randn((b, c) + dims, generator=g).to(torch.bfloat16).float() for _ in range(4)]
    st = torch.tensor([0x5EED_1234_ABCD], dtype=torch.int64, device=gpu)
    res = []
    for dt in (torch.float32, torch.bfloat16):
        q, k, v = (t.to(gpu).to(dt).contiguous(memory_format=CL).requires_grad_(True) for t in src[:3])
        y = PS.CausalAttentionFn.apply(q, k, v, nh, None if p is None else (p, st))
        y.backward(src[3].to(gpu).to(dt).contiguous(memory_format=CL))
        res.append([t.detach().float().cpu() for t in (y, q.grad, k.grad, v.grad)])
    for i, (a32, a16) in enumerate(zip(*res)):
        assert rel(a16, a32.numpy()) < (2e-2 if i == 0 else 4e-2), (i, rel(a16, a32.numpy()))


@pytest.mark.parametrize("gscale,vscale", [(1e-6, 1.0), (1e-8, 1.0), (1.0, 2e5)])
def test_attention_matrix_core_small_gradients_and_large_values(gpu, gscale, vscale):
    """The bf16 build's matrix-core attention at the magnitudes a real bf16 step has: upstream
    gradients of 1e-6 .. 1e-8 per element (the mean cross-entropy over 8,192 positions x 256
    classes, no loss scaler in bf16 runs) and value rows far beyond fp16's 65504.  The second
    products (P V, dO^T P, K^T dS, Q^T dS) take their operands in the build's own format, so dQ /
    dK / dV keep the same relative accuracy as at O(1) against the fp32 VALU kernels (fp16
    operands flushed dO / dS below 6.1e-5 and overflowed V)."""
    from vq3d import pixelsnail as PS
    g = torch.Generator().manual_seed(13)
    dims, b, c, nh = (4, 8, 8), 1, 16, 2
    src = [torch.randn((b, c) + dims, generator=g) for _ in range(4)]
    src[2] = src[2] * vscale
    src[3] = src[3] * gscale
    src = [t.to(torch.bfloat16).float() for t in src]
    res = []
    for dt in (torch.float32, torch.bfloat16):
        q, k, v = (t.to(gpu).to(dt).contiguous(memory_format=CL).requires_grad_(True) for t in src[:3])
        y = PS.CausalAttentionFn.apply(q, k, v, nh, None)
        y.backward(src[3].to(gpu).to(dt).contiguous(memory_format=CL))
        res.append([t.detach().float().cpu() for t in (y, q.grad, k.grad, v.grad)])
    for i, (a32, a16) in enumerate(zip(*res)):
        assert torch.isfinite(a16).all(), i
        assert rel(a16, a32.numpy()) < (2e-2 if i == 0 else 4e-2), (i, rel(a16, a32.numpy()))


def test_block_glue_kernels_match_torch(gpu):
    """The 16-bit runs' fused block glue (PreActFn: elu(x + a) + b into the conv operand;
    ScaleBiasResFn: o * scale + bias4 + skip) against the torch ops they replace: outputs, input
    gradients and the scalar-parameter gradients (accumulated into the parameters' .grad)."""
    from vq3d import pixelsnail as PS
    g = torch.Generator(device=gpu).manual_seed(5)
    shp = (1, 64, 8, 8, 16)
    x = torch.randn(shp, device=gpu, generator=g).contiguous(memory_format=CL)
    o = torch.randn(shp, device=gpu, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    sk = torch.randn(shp, device=gpu, generator=g).contiguous(memory_format=CL)
    gy = torch.randn(shp, device=gpu, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    gz = torch.randn(shp, device=gpu, generator=g).contiguous(memory_format=CL)
    prev = PS._compute[0]
    PS._compute[0] = torch.bfloat16
    try:
        res = []
        for fused in (True, False):
            a, b, sc, b4 = (torch.nn.Parameter(torch.tensor([v], device=gpu)) for v in (0.3, -0.2, 0.7, 0.1))
            for p in (a, b, sc, b4):
                p.grad = torch.zeros_like(p)
            xa, oa, ska = (t.clone().requires_grad_(True) for t in (x, o, sk))
            if fused:
                y = PS.PreActFn.apply(xa, a, b)
                z = PS.ScaleBiasResFn.apply(oa, sc, b4, ska)
            else:
                y = (torch.nn.functional.elu(xa + a) + b).to(torch.bfloat16)
                z = oa * sc + b4 + ska
            torch.autograd.backward([y, z], [gy, gz])
            res.append([t.detach().float() for t in (y, z, xa.grad, oa.grad, ska.grad, a.grad, b.grad, sc.grad,
                                                        b4.grad)])
    finally:
        PS._compute[0] = prev
    for i, (f, t) in enumerate(zip(*res)):
        tol = 1e-2 if i in (0, 3) else 1e-4  # bf16 outputs: one rounding apart at most
        assert rel(f, t.cpu().numpy()) < tol, (i, rel(f, t.cpu().numpy()))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,cg,cx,ldg,ldx,bias", [(8192, 64, 256, 64, 256, True), (8192, 256, 64, 256, 64, False),
                                                  (8192, 128, 64, 128, 64, True), (1000, 64, 64, 128, 72, True),
                                                  (300, 8, 24, 8, 24, True), (70, 136, 200, 136, 208, True)])
def test_rows_wgrad_matches_fp32(gpu, dt, n, cg, cx, ldg, ldx, bias):
    """vq3d_rows_wgrad (the 16-bit 1x1x1 convs' weight gradient, PointwiseFn.backward) against an
    fp32 torch GEMM of the same 16-bit rows: dw / db ACCUMULATED into preset buffers, ragged row
    counts, channel counts off the 64-tile, row strides wider than the rows (views), and bitwise
    equal on a second run (fixed-order split-K sum).  Tolerance 1e-5 of max |sum| (fp32 order)."""
    import ctypes
    from vq3d import _lib as L
    g0 = torch.Generator(device=gpu).manual_seed(n + cg + cx)
    gb = torch.randn((n, ldg), device=gpu, generator=g0).to(dt)
    xb = torch.randn((n, ldx), device=gpu, generator=g0).to(dt)
    gv, xv = gb[:, :cg], xb[:, :cx]
    want_w = gv.float().t() @ xv.float() + 0.5
    want_b = gv.float().sum(0) - 1.0
    outs = []
    for _ in range(2):
        dw = torch.full((cg, cx), 0.5, device=gpu)
        db = torch.full((cg,), -1.0, device=gpu) if bias else None
        nws = int(L.query("vq3d_rows_wgrad_workspace_bytes", n, cg, cx))
        ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=gpu)
        L.call("vq3d_rows_wgrad", L.dtype_code(gv), n, cg, cx, L.ptr(gv), ldg, L.ptr(xv), ldx, L.ptr(dw), L.ptr(db),
               L.ptr(ws), ctypes.c_size_t(nws), L.stream())
        torch.cuda.synchronize()
        outs.append((dw, db))
    dw, db = outs[0]
    assert rel(dw, want_w.cpu().numpy()) < 1e-5
    if bias:
        assert rel(db, want_b.cpu().numpy()) < 1e-5
    assert torch.equal(outs[0][0], outs[1][0])
    if bias:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,k,co,ldx,ldy,trans,bias", [
    (8192, 256, 64, 256, 64, 0, True),     # branch_conv1 forward (cin 256 -> branch 64)
    (8192, 64, 256, 64, 256, 1, False),    # its backward-data (g 64 -> gx 256)
    (8192, 64, 256, 64, 256, 0, False),    # branch_conv3 forward
    (8192, 520, 128, 520, 128, 0, True),   # key-value projection (515 inputs, padded to 520)
    (8192, 128, 520, 128, 520, 1, False),  # its backward-data
    (1000, 264, 72, 272, 80, 0, True),     # ragged rows, row strides wider than the rows
    (70, 8, 8, 8, 8, 1, False)])
def test_rows_gemm_matches_fp32(gpu, dt, n, k, co, ldx, ldy, trans, bias):
    """vq3d_rows_gemm (the 16-bit 1x1x1 convs' forward and backward-data, PointwiseFn) against an
    fp32 torch GEMM of the same 16-bit operands: y = x w^T (+ b) / gx = g w, rows of the published
    prior's shapes, K past the 64 KB LDS opt-in (520), ragged row counts, strided rows.  Tolerance:
    one rounding of the 16-bit output (2^-8 of max |y|) plus fp32 order."""
    import ctypes
    from vq3d import _lib as L
    g0 = torch.Generator(device=gpu).manual_seed(n + k + co)
    xb = torch.randn((n, ldx), device=gpu, generator=g0).to(dt)
    x = xb[:, :k]
    w = (torch.randn((k, co) if trans else (co, k), device=gpu, generator=g0) * 0.1).to(dt).contiguous()
    b = torch.randn(co, device=gpu, generator=g0) if bias else None
    want = x.float() @ (w.float() if trans else w.float().t())
    if b is not None:
        want = want + b
    yb = torch.full((n, ldy), float("nan"), device=gpu, dtype=dt)
    L.call("vq3d_rows_gemm", L.dtype_code(x), n, k, co, L.ptr(x), ldx, L.ptr(w), w.stride(0), trans, L.ptr(b),
           L.ptr(yb), ldy, L.stream())
    torch.cuda.synchronize()
    y = yb[:, :co].float()
    assert torch.isfinite(y).all()
    assert rel(y, want.cpu().numpy()) < 8e-3, rel(y, want.cpu().numpy())
    if ldy > co:
        assert torch.isnan(yb[:, co:].float()).all()  # nothing written past the rows


def test_rows_wgrad_rejects_unaligned(gpu):
    """channel counts / strides off a multiple of 8 fail loudly (PointwiseFn keeps those on the
    fp32 batched GEMM)"""
    import ctypes
    from vq3d import _lib as L
    gv = torch.zeros((64, 12), device=gpu, dtype=torch.bfloat16)
    xv = torch.zeros((64, 16), device=gpu, dtype=torch.bfloat16)
    dw = torch.zeros((12, 16), device=gpu)
    ws = torch.empty(1 << 16, dtype=torch.uint8, device=gpu)
    with pytest.raises(L.Vq3dError):
        L.call("vq3d_rows_wgrad", L.dtype_code(gv), 64, 12, 16, L.ptr(gv), 12, L.ptr(xv), 16, L.ptr(dw), None,
               L.ptr(ws), ctypes.c_size_t(1 << 16), L.stream())


def test_flat_weight_shadow_bitwise(gpu):
    """PixelSNAIL.logits on FlatParams reads its GEMM weights from one 16-bit cast of the flat
    buffer (FlatParams.refresh_shadow) instead of per-call casts: loss and every gradient equal to
    the per-call-cast run bit for bit, and again after the parameters change (the shadow follows)."""
    from vq3d import pixelsnail as PS
    from vq3d.flat import FlatParams
    kw = dict(num_embeddings=[64, 0], model_dim=64, num_blocks=1, num_layers_per_block=2, causal_dropout_prob=0.0,
              attention_dropout_prob=0.0)
    codes = torch.randint(0, 64, (1, 8, 8, 4), generator=torch.Generator().manual_seed(3)).to(gpu)
    onehot = torch.nn.functional.one_hot(codes, 64).permute(0, 4, 1, 2, 3).float().contiguous()
    res = []
    for flat in (False, True):
        torch.manual_seed(0)
        m = PS.PixelSNAIL(PS.default_args(**kw), compute_dtype="bf16").to(gpu)
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.01 * torch.randn_like(p))
        fl = FlatParams(m.parameters(), gpu) if flat else None
        out = []
        for it in range(2):
            for p in m.parameters():
                p.grad = None if fl is None else p.grad
            if fl is not None:
                fl.zero_grad()
            loss, _ = m.cross_entropy_onehot(onehot, codes)
            loss.backward()
            out.append([float(loss)] + [p.grad.detach().clone() for p in m.parameters()])
            with torch.no_grad():
                for p in m.parameters():
                    p.mul_(1.01)
        res.append(out)
    for a, b in zip(res[0], res[1]):
        assert a[0] == b[0]
        assert all(torch.equal(x, y) for x, y in zip(a[1:], b[1:]))


@pytest.mark.parametrize("stream", [0, 1, 2])
@pytest.mark.parametrize("shape", [(1, 64, 8, 32, 32), (1, 64, 5, 6, 7), (2, 32, 4, 8, 16)])
def test_tap_mask_conv_matches_dense(gpu, stream, shape):
    """The causal convs' tap mask (vq3d_conv_desc.tap_mask: the lines engines run their k-steps and
    weight-gradient tiles over the live taps only) against the dense conv of the same embedded
    kernel: forward, input gradient, prologue / bias sums and the live taps' weight gradient within
    fp32 summation order (1e-5 of max; 1e-2 for the bf16 outputs), dead taps' gradient unwritten."""
    from vq3d import ops, pixelsnail as PS
    from vq3d.ops import ConvGeom
    torch.manual_seed(stream)
    b, c = shape[:2]
    x = torch.randn(shape, device=gpu).to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(shape, device=gpu).to(torch.bfloat16).contiguous(memory_format=CL)
    mask = PS._tap_mask(stream, 3, 2)
    live = torch.tensor([(mask >> t) & 1 for t in range(27)], device=gpu, dtype=torch.bool).view(3, 3, 3)
    w = torch.randn((c, c, 3, 3, 3), device=gpu) * 0.05 * live
    cb = torch.randn(c, device=gpu)
    pa, pb = torch.tensor([0.1], device=gpu), torch.tensor([-0.2], device=gpu)
    geom = ConvGeom(3, 1, 1, False)
    res = []
    for taps in (0, mask):
        y = ops.conv_fwd(x, w, geom, pro=(pa, pb), cbias=cb, taps=taps)
        dw = torch.zeros_like(w)
        dcb, da, db = torch.zeros_like(cb), torch.zeros(1, device=gpu), torch.zeros(1, device=gpu)
        gx, _ = ops.conv_bwd(g, x, w, geom, pro=(pa, pb), aux=x, dw=dw, dcbias=dcb, dpro_pre=db, dpro_post=da,
                             taps=taps)
        ops.join_side()
        torch.cuda.synchronize()
        res.append((y.float(), gx.float(), dw, dcb, da, db))
    (y0, gx0, dw0, cb0, da0, db0), (y1, gx1, dw1, cb1, da1, db1) = res
    assert rel(y1, y0.cpu().numpy()) < 1e-2
    assert rel(gx1, gx0.cpu().numpy()) < 1e-2
    assert rel(dw1[..., live], dw0[..., live].cpu().numpy()) < 1e-5
    assert not dw1[..., ~live].any()
    for a1, a0 in ((cb1, cb0), (da1, da0), (db1, db0)):
        assert rel(a1, a0.cpu().numpy()) < 1e-4


def _lanes_model(gpu, **over):
    from vq3d import pixelsnail as PS
    from vq3d.flat import FlatParams
    kw = dict(num_embeddings=[64, 0], model_dim=64, num_blocks=2, num_layers_per_block=2, causal_dropout_prob=0.0,
              attention_dropout_prob=0.0)
    kw.update(over)
    torch.manual_seed(0)
    m = PS.PixelSNAIL(PS.default_args(**kw), compute_dtype="bf16").to(gpu)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.01 * torch.randn_like(p))
    fl = FlatParams(m.parameters(), gpu)
    return m, fl


def _captured_grads(gpu, m, fl, onehot, codes, lanes, replays):
    """eager warm-up on a side stream, one capture with PS.set_lanes(lanes), `replays` replays: the
    loss and every parameter's gradient after each replay"""
    from vq3d import pixelsnail as PS

    def step():
        fl.zero_grad()
        loss, _ = m.cross_entropy_onehot(onehot, codes)
        loss.backward()
        return loss
    prev = PS.lanes_mode()
    try:
        PS.set_lanes(lanes)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static = step()
        out = []
        for _ in range(replays):
            graph.replay()
            torch.cuda.synchronize()
            out.append([float(static)] + [p.grad.detach().clone() for p in m.parameters()])
        del graph
    finally:
        PS.set_lanes(prev)
    return out


def _replay_diffs(names, runs):
    """(replay index, [(parameter, relative L2 difference)]) for every replay that differs from the first"""
    bad = []
    for r, run in enumerate(runs[1:], 1):
        d = [(n, rel(y, x.cpu().numpy())) for n, x, y in zip(names, runs[0][1:], run[1:]) if not torch.equal(x, y)]
        if d or run[0] != runs[0][0]:
            bad.append((r, d[:12]))
    return bad


def test_lanes_match_single_stream_and_repeat_bitwise(gpu):
    """16-bit PixelSNAIL with the three stack streams on their own HIP streams (pixelsnail lanes, the
    default inside HIP-graph captures): a captured step's loss equals the eager single-stream step's
    and every gradient matches it within one bf16 rounding of the activation gradients summed in
    another order (2e-2 of each gradient's max), and four replays are bitwise equal (cross-lane
    gradients through _Fork: one lane per autograd accumulation, held until the backward ends;
    shared one-element parameters through per-lane rows; per-stream ticket regions)."""
    from vq3d import pixelsnail as PS
    m, fl = _lanes_model(gpu)
    codes = torch.randint(0, 64, (1, 8, 8, 4), generator=torch.Generator().manual_seed(4)).to(gpu)
    onehot = torch.nn.functional.one_hot(codes, 64).permute(0, 4, 1, 2, 3).float().contiguous()
    names = [n for n, _ in m.named_parameters()]
    prev = PS.lanes_mode()
    try:
        PS.set_lanes(False)
        fl.zero_grad()
        loss, _ = m.cross_entropy_onehot(onehot, codes)
        loss.backward()
        torch.cuda.synchronize()
        single = [float(loss)] + [p.grad.detach().clone() for p in m.parameters()]
        del loss  # (its graph would keep autograd nodes made on this stream alive into the capture)
    finally:
        PS.set_lanes(prev)
    runs = _captured_grads(gpu, m, fl, onehot, codes, "graph", 4)
    bad = _replay_diffs(names, runs)
    assert not bad, bad
    assert abs(single[0] - runs[0][0]) <= 1e-6 * abs(single[0])
    for n, x, y in zip(names, single[1:], runs[0][1:]):
        assert rel(y, x.cpu().numpy()) < 2e-2, n


def test_single_stream_replays_bitwise(gpu):
    """The same captured step without lanes: four replays bitwise equal (the deterministic
    single-stream baseline the lanes test is held to)."""
    m, fl = _lanes_model(gpu)
    codes = torch.randint(0, 64, (1, 8, 8, 4), generator=torch.Generator().manual_seed(4)).to(gpu)
    onehot = torch.nn.functional.one_hot(codes, 64).permute(0, 4, 1, 2, 3).float().contiguous()
    names = [n for n, _ in m.named_parameters()]
    bad = _replay_diffs(names, _captured_grads(gpu, m, fl, onehot, codes, False, 4))
    assert not bad, bad