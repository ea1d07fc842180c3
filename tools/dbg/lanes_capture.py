"""PixelSNAIL lanes + HIP-graph capture, small model: eager warm-up on a side stream, then one
capture of the step (mode "fwd": forward only; "bwd": forward + backward), one replay.  Run under
AMD_LOG_LEVEL=3 to see the stream / event API calls of the capture (tools/dbg/lanes.sh).

usage: python tools/dbg/lanes_capture.py fwd|bwd [num_blocks] [layers]"""
import faulthandler
import sys

import torch

faulthandler.enable()
sys.path.insert(0, "3d-vq-vae-2_amd")
from vq3d import pixelsnail as PS  # noqa: E402
from vq3d.flat import FlatParams  # noqa: E402

mode = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 1
gpu = torch.device("cuda:0")
torch.manual_seed(0)
args = PS.default_args(num_embeddings=[16, 0], model_dim=32, num_blocks=nb, num_layers_per_block=nl,
                       causal_dropout_prob=0.0, attention_dropout_prob=0.0)
m = PS.PixelSNAIL(args, compute_dtype="bf16").to(gpu)
fl = FlatParams(m.parameters(), gpu)
codes = torch.randint(0, 16, (1, 8, 8, 4), generator=torch.Generator().manual_seed(2)).to(gpu)
onehot = torch.nn.functional.one_hot(codes, 16).permute(0, 4, 1, 2, 3).contiguous().float()
lanes = [None]


def step():
    fl.zero_grad()
    loss, _ = m.cross_entropy_onehot(onehot, codes)
    if mode != "fwd":
        loss.backward()
    return loss


PS.set_lanes("graph")
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("eager ok", mode, "capture stream / lanes:", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    print("  capture stream", hex(torch.cuda.current_stream().cuda_stream),
          "lane1", hex(PS.ops.aux_stream(gpu, "psnail_lane1").cuda_stream),
          "lane2", hex(PS.ops.aux_stream(gpu, "psnail_lane2").cuda_stream), flush=True)
    step()
    print("  step issued, ending capture", flush=True)
print("captured", mode, flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed", mode, flush=True)
