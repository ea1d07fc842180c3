"""Single-stream captured PixelSNAIL step (the lanes test's small model): does replay 1 reproduce
replay 0?  Each variant monkeypatches one suspect and reports the first differing gradients.

usage: python tools/dbg/replay_bisect.py"""
import sys

import torch

sys.path.insert(0, "3d-vq-vae-2_amd")
sys.path.insert(0, "tests")
if len(sys.argv) > 1 and sys.argv[1] == "r05":  # the round-5 Python layer (tools/dbg/r05/) on this library
    import importlib.util
    import vq3d
    for mod, path in (("vq3d.flat", "tools/dbg/r05/flat_r05.py"), ("vq3d.pixelsnail", "tools/dbg/r05/pixelsnail_r05.py")):
        spec = importlib.util.spec_from_file_location(mod, path)
        m_ = importlib.util.module_from_spec(spec)
        sys.modules[mod] = m_
        spec.loader.exec_module(m_)
        setattr(vq3d, mod.split(".")[1], m_)
from vq3d import pixelsnail as PS  # noqa: E402
from vq3d import flat as FL  # noqa: E402
from test_gpu_pixelsnail import _lanes_model  # noqa: E402

gpu = torch.device("cuda:0")
codes = torch.randint(0, 64, (1, 8, 8, 4), generator=torch.Generator().manual_seed(4)).to(gpu)
onehot = torch.nn.functional.one_hot(codes, 64).permute(0, 4, 1, 2, 3).float().contiguous()


def shadow_inplace(self, dtype):
    sh = self._shadow.get(dtype)
    if sh is None:
        sh = self._shadow[dtype] = torch.empty(self.numel, dtype=dtype, device=self.device)
    sh.copy_(self.data)
    return sh


def run(name):
    m, fl = _lanes_model(gpu)
    names = [n for n, _ in m.named_parameters()]

    def step():
        fl.zero_grad()
        loss, _ = m.cross_entropy_onehot(onehot, codes)
        loss.backward()
        return loss
    PS.set_lanes(False)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static = step()
    out = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        out.append([p.grad.detach().clone() for p in m.parameters()])
    bad = [n for n, a, b in zip(names, out[0], out[1]) if not torch.equal(a, b)]
    gsum = [float(sum(t.double().abs().sum() for t in o)) for o in out]
    print(f"{name}: {len(bad)} of {len(names)} gradients differ replay 1 vs 0; |grad| sums {gsum}; "
          f"first in backward order {list(reversed(bad))[:5]}", flush=True)
    del g, static


cur_run_one = PS.CausalConv3dAdd.run_one
run("base")
if len(sys.argv) > 1 and sys.argv[1] == "r05":
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "zero":
    # every vq3d zero-fill as torch's fill kernel instead of hipMemsetAsync (a graph memset node)
    from vq3d import ops as OPS
    z0 = OPS.zero_
    OPS.zero_ = lambda t: t.zero_()
    for r in range(3):
        run(f"torch zero fills, try {r}")
    OPS.zero_ = z0
    for r in range(2):
        run(f"memset zero fills again, try {r}")
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "swap":
    # one round-5 class at a time in the current module (tools/dbg/r05/pixelsnail_r05.py)
    import importlib.util
    spec = importlib.util.spec_from_file_location("vq3d.pixelsnail_r05", "tools/dbg/r05/pixelsnail_r05.py")
    R5 = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(R5)
    for g_ in ("_compute", "_shadow", "_LANES", "_LSTATE", "_CUR", "_lanes_on"):  # shared module state
        setattr(R5, g_, getattr(PS, g_))
    cur = {n: getattr(PS, n) for n in ("CausalConvFn", "PointwiseFn", "pointwise", "PreActFn", "ScaleBiasResFn",
                                       "CausalConv3dAdd")}
    for name, names in (("r05 causal conv (Fn + run_one)", ("CausalConvFn", "CausalConv3dAdd")),
                        ("r05 pointwise", ("PointwiseFn", "pointwise")),
                        ("r05 glue", ("PreActFn", "ScaleBiasResFn"))):
        for n in names:
            if n == "CausalConv3dAdd":
                PS.CausalConv3dAdd.run_one = R5.CausalConv3dAdd.run_one
            else:
                setattr(PS, n, getattr(R5, n))
        run(name)
        for n in names:
            if n == "CausalConv3dAdd":
                PS.CausalConv3dAdd.run_one = cur_run_one
            else:
                setattr(PS, n, cur[n])
    sys.exit(0)
orig = FL.FlatParams.refresh_shadow
FL.FlatParams.refresh_shadow = shadow_inplace
run("shadow refreshed in place")
FL.FlatParams.refresh_shadow = orig
d0 = PS._direct
PS._direct = lambda p: False
run("no direct gradient adds")
PS._direct = d0
