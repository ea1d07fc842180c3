"""PixelSNAIL lanes replay check at the published mid-prior size (model-dim 256, 8 x 5 layers,
32 x 32 x 8 codes, dropout 0 so two replays must agree bit for bit): for each of `ncap` independent
captures (lanes on, and once lanes off as the baseline), `nrep` replays of forward + backward,
every parameter gradient compared with the first replay's; prints the differing parameters in
BACKWARD order (the first one listed is where a race would start) and the replay time.

usage: python tools/dbg/lanes_race.py [ncap] [nrep]"""
import sys
import time

import torch

sys.path.insert(0, "3d-vq-vae-2_amd")
from vq3d import pixelsnail as PS  # noqa: E402
from vq3d.flat import FlatParams  # noqa: E402

ncap = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nrep = int(sys.argv[2]) if len(sys.argv) > 2 else 4
gpu = torch.device("cuda:0")
torch.manual_seed(0)
args = PS.default_args(num_embeddings=[256, 0], model_dim=256, num_blocks=8, num_layers_per_block=5,
                       causal_dropout_prob=0.0, attention_dropout_prob=0.0, bottleneck_divisor=4, mixup_alpha=0.2,
                       lr=5e-5)
m = PS.PixelSNAIL(args, compute_dtype="bf16").to(gpu)
fl = FlatParams(m.parameters(), gpu)
m.train()
data = torch.randint(0, 256, (1, 1, 32, 32, 8), generator=torch.Generator().manual_seed(1)).to(gpu)
codes = data.squeeze(1)
onehot = torch.nn.functional.one_hot(codes, 256).permute(0, 4, 1, 2, 3).contiguous().float()
names = [n for n, _ in m.named_parameters()]
mix = (0.37, torch.arange(1))


def step():
    fl.zero_grad()
    loss, _ = m.cross_entropy_onehot(onehot, codes, mix)
    loss.backward()
    return loss


def run(lanes):
    PS.set_lanes(lanes)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static = step()
    torch.cuda.synchronize()
    runs, ts = [], []
    for _ in range(nrep):
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
        runs.append([float(static)] + [p.grad.detach().clone() for p in m.parameters()])
    del graph
    bad = 0
    for r, run_ in enumerate(runs[1:], 1):
        d = [n for n, x, y in zip(names, runs[0][1:], run_[1:]) if not torch.equal(x, y)]
        if d or run_[0] != runs[0][0]:
            bad += 1
            print(f"  replay {r}: loss {run_[0]!r} vs {runs[0][0]!r}, {len(d)} of {len(names)} gradients differ; "
                  f"backward order: {list(reversed(d))[:10]}", flush=True)
    return bad, min(ts), runs[0]


tot = 0
base_bad, base_ms, base = run(False)
print(f"single stream: {base_bad} differing replays, {base_ms:.2f} ms per fwd+bwd replay", flush=True)
for c in range(ncap):
    bad, ms, first = run("graph")
    worst = max(float((x - y).abs().max() / max(float(y.abs().max()), 1e-30))
                for x, y in zip(first[1:], base[1:]))
    print(f"lanes capture {c}: {bad} differing replays, {ms:.2f} ms per replay, loss {first[0]!r} "
          f"(single {base[0]!r}), worst gradient vs single-stream {worst:.3g} of max", flush=True)
    tot += bad
print("RESULT", "race-free" if tot == 0 and base_bad == 0 else f"{tot} differing lanes replays", flush=True)
sys.exit(0 if tot == 0 and base_bad == 0 else 1)
