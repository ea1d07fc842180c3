"""Captured PixelSNAIL step (the lanes test's small model), replayed 4 times, single stream and with
lanes: per replay the loss and the relative distance of a few gradients from the eager single-stream
step's, so a replay that differs from the others shows which one is off.

usage: python tools/dbg/replay_check.py"""
import sys

import torch

sys.path.insert(0, "3d-vq-vae-2_amd")
sys.path.insert(0, "tests")
from vq3d import pixelsnail as PS  # noqa: E402
from test_gpu_pixelsnail import _lanes_model  # noqa: E402

gpu = torch.device("cuda:0")
m, fl = _lanes_model(gpu)
codes = torch.randint(0, 64, (1, 8, 8, 4), generator=torch.Generator().manual_seed(4)).to(gpu)
onehot = torch.nn.functional.one_hot(codes, 64).permute(0, 4, 1, 2, 3).float().contiguous()
names = [n for n, _ in m.named_parameters()]
watch = [i for i, n in enumerate(names) if n in ("parse_input.weight", "to_causal.bias1b", "parse_output.weight",
                                                  "layers.0.causal_layers.0.branch_conv2.depth_conv.weight")]


def step():
    fl.zero_grad()
    loss, _ = m.cross_entropy_onehot(onehot, codes)
    loss.backward()
    return loss


def grads():
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in m.parameters()]


PS.set_lanes(False)
for _ in range(2):
    loss = step()
ref = grads()
print("eager single-stream loss", float(loss), flush=True)
del loss
for mode in (False, "graph"):
    PS.set_lanes(mode)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static = step()
    for r in range(4):
        g.replay()
        gr = grads()
        d = {names[i]: float((gr[i] - ref[i]).abs().max() / ref[i].abs().max().clamp_min(1e-30)) for i in watch}
        worst = max(range(len(names)), key=lambda i: float((gr[i] - ref[i]).abs().max() /
                                                            ref[i].abs().max().clamp_min(1e-30)))
        print(f"lanes={mode} replay {r}: loss {float(static)!r}; rel vs eager {d}; worst {names[worst]}", flush=True)
    del g, static
