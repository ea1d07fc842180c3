"""bisect the lanes + graph-capture crash: forward only / forward+backward / full step"""
import faulthandler
import sys
import torch
faulthandler.enable()
sys.path.insert(0, "3d-vq-vae-2_amd")
from vq3d import pixelsnail as PS
from vq3d.flat import FlatParams
from vq3d.optim import FusedAdam

mode = sys.argv[1]
if mode == "bwd_noflush":
    PS._lane_ctx = lambda: None
if mode == "bwd_emptyflush":
    def _nop(self):
        self.queued = False
    PS._LaneGrads.flush = _nop
PS.set_lanes(mode != "bwd_nolanes")
gpu = torch.device("cuda:0")
torch.manual_seed(0)
args = PS.default_args(num_embeddings=[16, 0], model_dim=32, num_blocks=1, num_layers_per_block=1,
                       causal_dropout_prob=0.0, attention_dropout_prob=0.0)
m = PS.PixelSNAIL(args, compute_dtype="bf16").to(gpu)
flat = FlatParams(m.parameters(), gpu)
opt = FusedAdam(m.parameters(), flat, lr=0.0, amsgrad=True)
codes = torch.randint(0, 16, (1, 8, 8, 4), generator=torch.Generator().manual_seed(2)).to(gpu)
onehot = torch.nn.functional.one_hot(codes, 16).permute(0, 4, 1, 2, 3).contiguous().float()


def step():
    opt.zero_grad()
    loss, _ = m.cross_entropy_onehot(onehot, codes)
    if mode != "fwd":
        print("backward", flush=True)
        loss.backward()
        print("backward done", flush=True)
        if mode != "bwd_nolanes":
            torch.cuda.current_stream().wait_stream(PS.ops.aux_stream(gpu, "psnail_lane1"))
            torch.cuda.current_stream().wait_stream(PS.ops.aux_stream(gpu, "psnail_lane2"))
    if mode == "full":
        opt.step()
    return loss


step()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("eager ok", mode, flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
print("captured", mode, flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed", mode, flush=True)
