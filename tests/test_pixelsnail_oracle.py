"""CPU oracle of the PixelSNAIL prior (oracle/pixelsnail_cpu.py) against the reference's own
outputs (tests/golden/psnail_*.npz, tools/make_goldens_pixelsnail.py): causal 3-stack convs
(mask A / B, kernel 1 / 3), PreActFixupCausalResBlock (mask A, mask B with the attention aux
input), CausalAttention (2 and 8 heads, the reference's swapped keys / queries binding), and a
whole PixelSNAIL training loss with every parameter gradient."""
import numpy as np
import pytest
import torch

from oracle import pixelsnail_cpu as O

G = "tests/golden/"


def P_of(d, pre="p/"):
    return {k[len(pre):]: torch.tensor(d[k]) for k in d.files if k.startswith(pre)}


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


@pytest.mark.parametrize("name,mask,k,bias", [("psnail_conv_b3", "B", 3, False), ("psnail_conv_a1", "A", 1, True),
                                              ("psnail_conv_b1", "B", 1, True)])
def test_causal_conv(name, mask, k, bias):
    d = np.load(G + name + ".npz")
    P = {n: t.requires_grad_(True) for n, t in P_of(d).items()}
    x = torch.tensor(d["x"], requires_grad=True)
    y = O.causal_conv(x, P, "", mask, k, bias)
    assert rel(y.detach(), d["y"]) < 1e-6
    y.backward(torch.tensor(d["gy"]))
    assert rel(x.grad, d["gx"]) < 1e-5
    for n in P:
        assert rel(P[n].grad, d["g/" + n]) < 1e-5, n


@pytest.mark.parametrize("name,mask,aux", [("psnail_block_a", "A", False), ("psnail_block_b_aux", "B", True)])
def test_causal_block(name, mask, aux):
    d = np.load(G + name + ".npz")
    P = {n: t.requires_grad_(True) for n, t in P_of(d).items()}
    x = torch.tensor(d["x"], requires_grad=True)
    a = torch.tensor(d["aux"], requires_grad=True) if aux else None
    y = O.preact_causal_block(x, P, "", mask, aux=a)
    assert rel(y.detach(), d["y"]) < 1e-6
    y.backward(torch.tensor(d["gy"]))
    assert rel(x.grad, d["gx"]) < 1e-5
    if aux:
        assert rel(a.grad, d["gaux"]) < 1e-5
    for n in P:
        assert rel(P[n].grad, d["g/" + n]) < 1e-5, n


@pytest.mark.parametrize("name,nh", [("psnail_attn_h2", 2), ("psnail_attn_h8", 8)])
def test_causal_attention(name, nh):
    d = np.load(G + name + ".npz")
    q, k, v = (torch.tensor(d[n], requires_grad=True) for n in ("q", "k", "v"))
    y = O.causal_attention(q, k, v, nh)
    assert rel(y.detach(), d["y"]) < 1e-6
    y.backward(torch.tensor(d["gy"]))
    for t, n in ((q, "gq"), (k, "gk"), (v, "gv")):
        assert rel(t.grad, d[n]) < 1e-5, n


def test_pixelsnail_loss_and_grads():
    d = np.load(G + "psnail_model_32.npz")
    P = {n: t.requires_grad_(True) for n, t in P_of(d).items()}
    ne, _, nl, nb, _ = (int(c) for c in d["cfg"])
    loss, logits = O.loss(P, torch.tensor(d["data"]), ne, nb, nl)
    assert rel(logits.detach(), d["logits"]) < 1e-6
    assert abs(float(loss) - float(d["loss"])) < 1e-6 * abs(float(d["loss"]))
    loss.backward()
    scale = max(np.abs(d["g/" + n]).max() for n in P)
    for n in P:  # the key-role projection biases have exactly-zero true gradients (softmax shift)
        err = np.abs(P[n].grad.numpy() - d["g/" + n]).max()
        assert err <= max(1e-4 * np.abs(d["g/" + n]).max(), 1e-6 * scale), n


def test_product_module_tree_and_seeded_init():
    """vq3d.pixelsnail.PixelSNAIL builds the reference's module tree (state_dict keys / shapes)
    and, seeded, bit-identical initial parameters (construction order + initialize_weights)."""
    from vq3d import pixelsnail as PS
    d = np.load(G + "psnail_init_64.npz")
    torch.manual_seed(3)
    m = PS.PixelSNAIL(PS.default_args(model_dim=64, num_blocks=2, num_layers_per_block=2, num_embeddings=[16, 0],
                                      causal_dropout_prob=0.0, attention_dropout_prob=0.0), compute_dtype="fp32")
    ref = {k[2:]: d[k] for k in d.files}
    mine = dict(m.named_parameters())
    assert sorted(mine) == sorted(ref)
    for n, p in mine.items():
        assert tuple(p.shape) == ref[n].shape, n
        assert np.array_equal(p.detach().numpy(), ref[n]), n


def test_attention_train_mode_golden():
    """training-mode logits (dropout p = 0: exact-zero logits -> -1e3, layers.py:633-637) against
    the reference's CausalAttention in train mode on inputs with zeroed key rows"""
    d = np.load(G + "psnail_attn_train.npz")
    k, q, v = (torch.tensor(d[n], requires_grad=True) for n in ("keys", "queries", "values"))
    y = O.causal_attention(k, q, v, int(d["nh"]), train=True)
    assert rel(y.detach(), d["out"]) < 1e-5
    y.backward(torch.tensor(d["gy"]))
    for t, n in ((k, "g_keys"), (q, "g_queries"), (v, "g_values")):
        assert rel(t.grad, d[n]) < 1e-4, n
    # eval mode differs on these inputs: the replacement is exercised
    ye = O.causal_attention(k, q, v, int(d["nh"]), train=False)
    assert rel(ye.detach(), d["out"]) > 1e-3


def test_mixup_draws_match_reference():
    """vq3d.pixelsnail.mixup_draw: lam ~ Beta(alpha, alpha) from numpy's global generator and the
    Sattolo cycle from Python's random, in the reference's order (train_helpers.py:20-51): the same
    lam and index under the same seeds, and the same blend lam x + (1 - lam) x[index]"""
    import random

    from vq3d import pixelsnail as PS
    d = np.load(G + "psnail_mixup.npz")
    for i in range(len(d["seed"])):
        random.seed(int(d["seed"][i]))
        np.random.seed(int(d["seed"][i]))
        b = int(d["batch"][i])
        lam, index = PS.mixup_draw(b, float(d["alpha"][i]))
        assert np.float32(lam) == np.float32(d["lam"][i])  # the reference keeps lam in x.dtype (fp32)
        assert index.tolist() == d["index"][i][:b].tolist()
        x = torch.arange(b, dtype=torch.float32)
        lt = torch.as_tensor(lam, dtype=torch.float32)
        assert torch.equal(lt * x + (1 - lt) * x[index], torch.tensor(d["mixed"][i][:b]))
