"""ORACLE (test infrastructure only): functional CPU restatement of the reference's PixelSNAIL
prior (pixel_model/pixelsnail.py, pixel_model/layers.py), fp32 plain PyTorch CPU ops.

Only tests/ (and bench.py's cpu_baseline leg) may import this module; the product package
never does.  Everything operates on a reference-layout parameter dict (the keys of the
reference's `PixelSNAIL.state_dict()`), so the golden fixtures and the HIP framework plug in.
Parity pinned against tests/golden/psnail_*.npz (tools/make_goldens_pixelsnail.py, generated
by importing the reference); gradients come from torch autograd over these same CPU ops.

A "stack" is the reference's (3, b, c, d, h, w) tensor: the depth-, height- and width-wise
causal streams (pixel_model/layers.py:103-110).
"""
import math

import torch
import torch.nn.functional as F


# ---------------------------------------------------------------- shifts (layers.py:13-100)
def shift_back(t):
    """front-pad d by one, drop the last d slice (shift_backwards_3d, layers.py:13-29)"""
    return F.pad(t, (0, 0, 0, 0, 1, 0))[:, :, :-1]


def shift_down(t):
    """front-pad h by one (shift_down_3d, layers.py:51-66)"""
    return F.pad(t, (0, 0, 1, 0, 0, 0))[:, :, :, :-1]


def shift_right(t):
    """front-pad w by one (shift_right_3d, layers.py:85-100)"""
    return F.pad(t, (1, 0, 0, 0, 0, 0))[..., :-1]


# ---------------------------------------------------------------- CausalConv3dAdd (layers.py:122-222)
def causal_conv(stack, P, pre, mask, k, bias):
    """depth conv (k-1, k, k) / height conv (1, k-1, k) / width conv (1, 1, k//2 + [mask B]),
    zero padding on the causal side only (layers.py:188-222)."""
    d, h, w = stack[0], stack[1], stack[2]
    if mask == "A":
        d, h, w = shift_back(d), shift_down(h), shift_right(w)
    dsz = max(k - 1, 1)
    wsz = max(k // 2 + (1 if mask == "B" else 0), 1)
    hk = k // 2
    b = (lambda n: P[pre + n + ".bias"]) if bias else (lambda n: None)
    d = F.conv3d(F.pad(d, (hk, hk, hk, hk, dsz - 1, 0)), P[pre + "depth_conv.weight"], b("depth_conv"))
    h = F.conv3d(F.pad(h, (hk, hk, dsz - 1, 0, 0, 0)), P[pre + "height_conv.weight"], b("height_conv"))
    w = F.conv3d(F.pad(w, (wsz - 1, 0, 0, 0, 0, 0)), P[pre + "width_conv.weight"], b("width_conv"))
    return torch.stack([d, h, w])


def expand_rf(stack, P, pre):
    """ExpandRFConv (layers.py:225-248): the depth stream feeds height and width, height feeds width."""
    d, h, w = stack[0], stack[1], stack[2]
    dch, dcw = torch.chunk(F.conv3d(d, P[pre + "depth_conv.weight"], P[pre + "depth_conv.bias"]), 2, dim=1)
    w = w + F.conv3d(h, P[pre + "height_conv.weight"], P[pre + "height_conv.bias"]) + dcw
    h = h + dch
    return torch.stack([d, h, w])


# ---------------------------------------------------------------- PreActFixupCausalResBlock (layers.py:338-467)
def preact_causal_block(stack, P, pre, mask, k=3, aux=None):
    s = lambda n: P[pre + n]  # noqa: E731
    out = F.elu(stack + s("bias1a"))
    out = causal_conv(out + s("bias1b"), P, pre + "branch_conv1.", mask, 1, False)
    out = expand_rf(out, P, pre + "expand_rf.")
    if aux is not None:
        out = out + causal_conv(F.elu(aux), P, pre + "aux.", "B", 1, True)
    out = F.elu(out + s("bias2a"))
    out = causal_conv(out + s("bias2b"), P, pre + "branch_conv2.", "B", k, False)
    out = F.elu(out + s("bias3a"))
    out = causal_conv(out + s("bias3b"), P, pre + "branch_conv3.", "B", 1, False)
    out = out * s("scale") + s("bias4")
    skip = pre + "skip_conv.depth_conv.weight"
    return out + (causal_conv(stack, P, pre + "skip_conv.", mask, 1, True) if skip in P else stack)


# ---------------------------------------------------------------- CausalAttention (layers.py:613-647)
def causal_attention(keys, queries, values, nh, train=False, p=0.0, dropped=None):
    """The reference's parameter binding: `keys` / `queries` as CausalAttention.forward names
    them.  CausalAttentionPixelBlock passes (queries, keys, values) positionally
    (layers.py:694), so the projected queries land in `keys` and vice versa.
    train (the module's dropout in training mode, layers.py:633-637): logits through dropout --
    `dropped` (bool, broadcastable to (sd, b, nh, n, n)) zeroed, the rest scaled by 1 / (1 - p);
    the reference draws it from torch's RNG, a test passes the mask it wants -- then every logit
    == 0 replaced by -1e3 (masked_fill: no gradient through the replaced entries)."""
    sd, b, ck = keys.shape[:3]
    dims = keys.shape[3:]
    n = math.prod(dims)
    cv = values.shape[2]
    fq = queries.reshape(sd, b, nh, ck // nh, n) * (ck // nh) ** -0.5
    fk = keys.reshape(sd, b, nh, ck // nh, n)
    fv = values.reshape(sd, b, nh, cv // nh, n)
    logits = torch.matmul(fq.transpose(3, 4), fk)
    if train:
        if p > 0:
            logits = torch.where(dropped, torch.zeros_like(logits), logits / (1.0 - p))
        logits = logits.masked_fill(logits == 0, -1e3)
    mask = torch.tril(torch.ones((n, n), dtype=torch.bool))
    logits = logits.masked_fill(~mask, float("-inf"))
    wts = F.softmax(logits, -1)
    out = torch.matmul(wts, fv.transpose(3, 4)).transpose(3, 4)
    return out.reshape(sd, b, -1, *dims)


def causal_attention_rows(keys, queries, values, nh, rows, train=False):
    """causal_attention's output at the query positions `rows` only (flattened d, h, w order):
    the same arithmetic restricted to those rows of the logits, so a sampled slice of an
    8,192-position attention is checkable on the CPU.  Returns (sd, b, cv, len(rows))."""
    sd, b, ck = keys.shape[:3]
    n = math.prod(keys.shape[3:])
    cv = values.shape[2]
    rows = torch.as_tensor(rows)
    fq = queries.reshape(sd, b, nh, ck // nh, n)[..., rows] * (ck // nh) ** -0.5
    fk = keys.reshape(sd, b, nh, ck // nh, n)
    fv = values.reshape(sd, b, nh, cv // nh, n)
    logits = torch.matmul(fq.transpose(3, 4), fk)  # (sd, b, nh, len(rows), n)
    if train:
        logits = logits.masked_fill(logits == 0, -1e3)
    mask = torch.arange(n).view(1, n) <= rows.view(-1, 1)
    wts = F.softmax(logits.masked_fill(~mask, float("-inf")), -1)
    out = torch.matmul(wts, fv.transpose(3, 4)).transpose(3, 4)  # (sd, b, nh, cv // nh, len(rows))
    return out.reshape(sd, b, cv, len(rows))


def background(b, dims):
    """_generate_background (pixelsnail.py:283-293): linspace(-1, 1) over d, h, w, per stack."""
    d, h, w = dims
    return torch.cat([
        torch.linspace(-1, 1, d).view(1, 1, 1, -1, 1, 1).expand(3, b, 1, d, h, w),
        torch.linspace(-1, 1, h).view(1, 1, 1, 1, -1, 1).expand(3, b, 1, d, h, w),
        torch.linspace(-1, 1, w).view(1, 1, 1, 1, 1, -1).expand(3, b, 1, d, h, w),
    ], dim=2)


def attention_block(stack, bg, P, pre, nlayers, nh=8):
    """CausalAttentionPixelBlock.forward (layers.py:683-703)."""
    out = stack
    for i in range(nlayers):
        out = preact_causal_block(out, P, f"{pre}causal_layers.{i}.", "B")
    kv = causal_conv(torch.cat([stack, out, bg], dim=2), P, pre + "key_value_proj.", "B", 1, True)
    keys, values = torch.chunk(kv, 2, dim=2)
    queries = causal_conv(torch.cat([out, bg], dim=2), P, pre + "query_proj.", "B", 1, True)
    att = causal_attention(queries, keys, values, nh)
    return preact_causal_block(out, P, pre + "out_proj.", "B", aux=att)


# ---------------------------------------------------------------- PixelSNAIL (pixelsnail.py:101-161, 301-320)
def forward(P, onehot, nblocks, nlayers):
    b = onehot.shape[0]
    dims = tuple(onehot.shape[2:])
    x = F.conv3d(onehot, P["parse_input.weight"], P["parse_input.bias"])
    stack = x.unsqueeze(0).expand(3, *x.shape)
    stack = preact_causal_block(stack, P, "to_causal.", "A")
    bg = background(b, dims)
    for i in range(nblocks):
        stack = attention_block(stack, bg, P, f"layers.{i}.", nlayers)
    return F.conv3d(stack.sum(0), P["parse_output.weight"], P["parse_output.bias"])


def loss(P, data, num_embeddings, nblocks, nlayers):
    """cross_entropy (pixelsnail.py:112-161) without mixup / conditioning: mean CE of the logits
    over every code position."""
    codes = data.squeeze(1)
    onehot = F.one_hot(codes, num_embeddings).permute(0, 4, 1, 2, 3).float()
    logits = forward(P, onehot, nblocks, nlayers)
    return F.cross_entropy(logits, codes, reduction="none").mean(), logits
