"""torch.optim.Adam(amsgrad=True) (reference vqvae/model.py:91-93) as one fused kernel over
the flat parameter buffer.  state_dict() uses torch Adam's per-parameter layout
(exp_avg / exp_avg_sq / max_exp_avg_sq / step) so checkpoints interchange."""
import torch

from . import _lib as L
from . import ops


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=True):
        if weight_decay != 0 or not amsgrad:
            raise NotImplementedError("FusedAdam implements the reference's Adam(amsgrad=True, weight_decay=0)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=True))
        self.flat = flat
        for g in self.param_groups:
            for p in g["params"]:
                if not flat.owns(p):
                    raise ValueError("FusedAdam: every parameter must live in the model's flat buffer")
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.vmax = torch.zeros_like(flat.data)
        # completed steps, on the device: the kernel derives the bias corrections from it and
        # increments it, so a captured HIP graph of the whole step replays correctly
        self.step_t = torch.zeros((), dtype=torch.int64, device=flat.data.device)

    @property
    def step_count(self):
        return int(self.step_t.item())

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        ops.join_side()  # weight gradients issued on the side stream are complete
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        f = self.flat
        L.call("vq3d_adam_amsgrad_dev", L.ptr(f.data), L.ptr(f.grad), L.ptr(self.m), L.ptr(self.v),
               L.ptr(self.vmax), f.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]), L.ptr(self.step_t),
               L.stream())
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict(self):
        sd = super().state_dict()
        st = {}
        step_count = self.step_count
        offs = {id(q): off for q, off in zip(self.flat.params, self.flat.offsets)}
        idx = 0
        for g in self.param_groups:
            for p in g["params"]:
                off = offs[id(p)]
                n = p.numel()
                if step_count:
                    st[idx] = dict(step=torch.tensor(float(step_count)),
                                   exp_avg=self.m[off:off + n].view(p.shape).clone(),
                                   exp_avg_sq=self.v[off:off + n].view(p.shape).clone(),
                                   max_exp_avg_sq=self.vmax[off:off + n].view(p.shape).clone())
                idx += 1
        sd["state"] = st
        return sd

    def load_state_dict(self, state_dict):
        st = state_dict["state"]
        offs = {id(q): off for q, off in zip(self.flat.params, self.flat.offsets)}
        idx = 0
        steps = set()
        for g in self.param_groups:
            for p in g["params"]:
                off = offs[id(p)]
                n = p.numel()
                s = st.get(idx)
                if s is not None:
                    self.m[off:off + n].copy_(s["exp_avg"].reshape(-1))
                    self.v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
                    self.vmax[off:off + n].copy_(s["max_exp_avg_sq"].reshape(-1))
                    steps.add(int(float(s["step"])))
                idx += 1
        self.step_t.fill_(steps.pop() if steps else 0)
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            g["lr"] = sg["lr"]
