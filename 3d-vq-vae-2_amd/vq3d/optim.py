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
    def step(self, closure=None, skip=None):
        """skip: optional device flag (GradScaler.found_inf): when non-zero the update and the step
        count are skipped on the device."""
        loss = closure() if closure is not None else None
        ops.join_side()  # weight gradients issued on the side stream are complete
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        f = self.flat
        L.call("vq3d_adam_amsgrad_dev", L.ptr(f.data), L.ptr(f.grad), L.ptr(self.m), L.ptr(self.v),
               L.ptr(self.vmax), f.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]), L.ptr(self.step_t),
               L.ptr(skip) if skip is not None else None, L.stream())
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


class GradScaler:
    """Dynamic loss scaling for the fp16 path: torch.cuda.amp.GradScaler as PL 1.2.10's native AMP
    plugin uses it for the reference's precision=16 (vqvae/train.py:32; init_scale 2**16, growth
    x2 after 2000 clean steps, backoff x0.5), over the model's flat fp32 gradient with every piece
    of state on the device, so a captured step graph replays it:

        scaler.scale(loss).backward(); allreduce(); scaler.step(opt); scaler.update()

    step() unscales the flat gradient in place and flags a non-finite value (vq3d_grad_unscale);
    FusedAdam then skips the update and its step count on a flagged step; update() backs the
    scale off or grows it (vq3d_loss_scale_update).  enabled=False (bf16 / fp32): pass-through."""

    def __init__(self, device, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        self.enabled = enabled
        self.growth_factor, self.backoff_factor, self.growth_interval = growth_factor, backoff_factor, growth_interval
        self.scale_t = torch.full((), float(init_scale), dtype=torch.float32, device=device)
        self.tracker = torch.zeros((), dtype=torch.int32, device=device)
        self.found_inf = torch.zeros((), dtype=torch.float32, device=device)
        self._unscaled = False

    def scale(self, loss):
        return loss * self.scale_t if self.enabled else loss

    def unscale_(self, opt):
        """The flat gradient divided by the scale in place (+ the non-finite flag), as
        torch.cuda.amp.GradScaler.unscale_; step() then does not unscale again."""
        if not self.enabled or self._unscaled:
            return
        ops.join_side()
        f = opt.flat
        L.call("vq3d_grad_unscale", L.ptr(f.grad), f.numel, L.ptr(self.scale_t), L.ptr(self.found_inf), L.stream())
        self._unscaled = True

    def step(self, opt):
        if not self.enabled:
            return opt.step()
        self.unscale_(opt)
        self._unscaled = False
        return opt.step(skip=self.found_inf)

    def update(self):
        if self.enabled:
            L.call("vq3d_loss_scale_update", L.ptr(self.scale_t), L.ptr(self.tracker), L.ptr(self.found_inf),
                   float(self.growth_factor), float(self.backoff_factor), int(self.growth_interval), L.stream())

    def get_scale(self):
        return float(self.scale_t) if self.enabled else 1.0

    def state_dict(self):
        """torch GradScaler.state_dict()'s keys (PL stores it as 'native_amp_scaling_state')."""
        if not self.enabled:
            return {}
        return {"scale": float(self.scale_t), "growth_factor": self.growth_factor,
                "backoff_factor": self.backoff_factor, "growth_interval": self.growth_interval,
                "_growth_tracker": int(self.tracker)}

    def load_state_dict(self, sd):
        if not sd:
            return
        self.scale_t.fill_(float(sd["scale"]))
        self.tracker.fill_(int(sd["_growth_tracker"]))
        self.growth_factor, self.backoff_factor = float(sd["growth_factor"]), float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
