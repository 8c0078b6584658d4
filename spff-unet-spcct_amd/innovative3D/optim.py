"""Fused Adam / AdamW on the HIP engine.

``SPFFAdam`` is a drop-in for ``torch.optim.Adam`` / ``AdamW`` (the optimizers
of BaseLitModel.configure_optimizers, models.py:591-594, and
apply_unified_optimizer, unified_optimizer.py:5-60): same hyper-parameters, the
same state-dict layout ({"step", "exp_avg", "exp_avg_sq"} per parameter) and
torch's fp32 arithmetic, but each group's update is ONE HBM pass per
contiguous run of (param, grad, state) memory -- the engine keeps parameters
and gradients in flat buffers (models.py here), and the state is allocated
flat in parameter order, so a step is typically one kernel launch
(include/spff.h spff_adam_step).  Parameters created after the optimizer (the
lazily materialised FourierGate mask) are not in its groups, as
in the reference."""
from __future__ import annotations

from typing import List, Tuple

import torch

from . import _engine as E


class SPFFAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 decoupled_weight_decay=False, amsgrad=False, maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("SPFFAdam: amsgrad / maximize are not used by the reference")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("invalid lr / eps / weight_decay")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        decoupled_weight_decay=bool(decoupled_weight_decay))
        super().__init__(params, defaults)
        self._flat_state = {}

    def _state_for(self, group_idx: int, ps: List[torch.Tensor]):
        """exp_avg / exp_avg_sq views into one flat buffer per group (parameter order)."""
        key = (group_idx, tuple(p.data_ptr() for p in ps))
        if key not in self._flat_state:
            n = sum(p.numel() for p in ps)
            dev = ps[0].device
            m = torch.zeros(n, dtype=torch.float32, device=dev)
            v = torch.zeros(n, dtype=torch.float32, device=dev)
            o = 0
            for p in ps:
                st = self.state[p]
                k = p.numel()
                if "exp_avg" in st:  # loaded from a state dict: keep its values
                    m[o:o + k].copy_(st["exp_avg"].reshape(-1))
                    v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
                st["exp_avg"] = m[o:o + k].view_as(p)
                st["exp_avg_sq"] = v[o:o + k].view_as(p)
                st.setdefault("step", torch.tensor(0.0))
                o += k
            self._flat_state[key] = (m, v)
        return self._flat_state[key]

    @staticmethod
    def _runs(items: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]]):
        """Merge consecutive (p, g, m, v) whose four memories are all contiguous."""
        runs = []
        for p, g, m, v in items:
            if runs:
                P, G, M, V, n = runs[-1]
                if (p.data_ptr() == P + 4 * n and g.data_ptr() == G + 4 * n and
                        m.data_ptr() == M + 4 * n and v.data_ptr() == V + 4 * n):
                    runs[-1][4] += p.numel()
                    continue
            runs.append([p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel()])
        return runs

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = E.lib()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                E.require_device(p, "SPFFAdam")
                if p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise E.SpffError("SPFFAdam: contiguous fp32 parameters and gradients only")
            self._state_for(gi, ps)
            # one step counter per group (every parameter with a gradient steps together)
            steps = []
            for p in ps:
                st = self.state[p]
                st["step"] += 1
                steps.append(int(st["step"].item()))
            b1, b2 = group["betas"]
            items = [(p, p.grad, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]) for p in ps]
            stream = E._stream(ps[0].device)
            if len(set(steps)) == 1:
                for P, G, M, V, n in self._runs(items):
                    E.check(L.spff_adam_step(P, G, M, V, n, group["lr"], b1, b2, group["eps"],
                                             group["weight_decay"],
                                             int(group["decoupled_weight_decay"]), steps[0],
                                             stream), "spff_adam_step")
            else:  # parameters joined at different times: per-parameter launches
                for (p, g, m, v), t in zip(items, steps):
                    E.check(L.spff_adam_step(p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                             v.data_ptr(), p.numel(), group["lr"], b1, b2,
                                             group["eps"], group["weight_decay"],
                                             int(group["decoupled_weight_decay"]), t, stream),
                            "spff_adam_step")
        return loss


def SPFFAdamW(params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, **kw):
    """torch.optim.AdamW semantics (decoupled weight decay)."""
    return SPFFAdam(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                    decoupled_weight_decay=True, **kw)
