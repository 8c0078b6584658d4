"""Knife-edge resolution for gradient comparisons (test infrastructure).

A LeakyReLU input within fp32 rounding of 0 (or a MaxPool window whose two
largest entries are within rounding of each other) may take either branch,
depending on the summation order of the conv that produced it.  The
reference's fixtures were written by oneDNN on one CPU; the oracle on another
CPU (or the engine on the GPU) can land on the other side of such a knife
edge, which moves whole gradient tensors by up to a few per cent while every
forward value still agrees to 1e-6.

``resolve_kinks`` finds the knife-edge candidates of an fp64 oracle run
(LeakyReLU inputs nearest 0 in units of the channel's normalised std, MaxPool
windows with the narrowest top-2 gap) and greedily flips the fewest of them
under which the fp64 oracle reproduces the fixture's gradients.  The test
asserts how many flips that took (a real formula error is not fixable by a
handful of single-voxel branch flips).
"""
import itertools

import numpy as np
import torch
import torch.nn.functional as F

from oracle import spff_oracle as O


class _Hooks:
    """Route conv_in_lrelu / maxpool of the oracle through recorded or forced branches."""

    def __init__(self):
        self.record = {}
        self.force = {}           # (layer, flat index) -> flipped
        self.pool_force = {}      # (pool k, flat index) -> argmax slot
        self.npool = 0

    def conv_in_lrelu(self, P, pre, inp, ksd):
        y = F.conv3d(inp, P[pre + ".0.weight"], None, padding=(ksd // 2, 1, 1))
        r = F.instance_norm(y, weight=P[pre + ".1.weight"], bias=P[pre + ".1.bias"], eps=1e-5)
        pos = r.detach() > 0
        # margin in units of the channel's normalised std: |r| / |gamma_c|
        g = P[pre + ".1.weight"].detach().abs().clamp_min(1e-30).reshape(1, -1, 1, 1, 1)
        self.record[pre] = (r.detach() / g).clone()
        flips = [i for (l, i) in self.force if l == pre]
        if flips:
            pos = pos.clone().reshape(-1)
            for i in flips:
                pos[i] = ~pos[i]
            pos = pos.reshape(r.shape)
        return torch.where(pos, r, 0.01 * r)

    def maxpool(self, t):
        k = self.npool % 3
        self.npool += 1
        B_, C_, D_, H_, W_ = t.shape
        v = t[..., :H_ // 2 * 2, :W_ // 2 * 2].reshape(B_, C_, D_, H_ // 2, 2, W_ // 2, 2)
        v = v.permute(0, 1, 2, 3, 5, 4, 6)
        v = v.reshape(B_, C_, D_, H_ // 2, W_ // 2, 4)
        self.record[f"pool{k + 1}"] = v.detach().clone()
        idx = v.detach().argmax(-1)
        forced = [(i, s) for (kk, i), s in self.pool_force.items() if kk == k]
        if forced:
            idx = idx.clone().reshape(-1)
            for i, s in forced:
                idx[i] = s
            idx = idx.reshape(v.shape[:-1])
        return v.gather(-1, idx.unsqueeze(-1)).squeeze(-1)


def _run(st, x, labels, cfg, hooks, dtype=torch.float64):
    orig = O.conv_in_lrelu, O.maxpool
    O.conv_in_lrelu, O.maxpool = hooks.conv_in_lrelu, hooks.maxpool
    try:
        hooks.npool = 0
        P = O.params_from_state(st, dtype=dtype)
        O.fwd_bwd(P, x.to(dtype), labels, cfg)
    finally:
        O.conv_in_lrelu, O.maxpool = orig
    return {k: (v.grad.double().numpy() if v.grad is not None else np.zeros(tuple(v.shape)))
            for k, v in P.items()}


def candidates(hooks, n):
    """The n knife-edge candidates of a recorded run, most marginal first:
    ("act", layer, flat index) by |r| / |gamma_c| (the IN output in units of
    the channel's normalised std, where a conv's rounding error lands), and
    ("pool", k, flat index, runner-up slot) by the top-2 gap / max|window|."""
    acts, pools = [], []
    for name, r in hooks.record.items():
        if name.startswith("pool"):
            v = r.reshape(-1, 4)
            top2 = torch.topk(v, 2, dim=-1)
            gap = (top2.values[:, 0] - top2.values[:, 1]) / max(float(v.abs().max()), 1e-30)
            gap = torch.where(gap > 0, gap, torch.full_like(gap, float("inf")))  # exact ties: first max
            m = min(n, gap.numel())
            g, i = torch.topk(gap, m, largest=False)
            for gg, ii in zip(g.tolist(), i.tolist()):
                pools.append((gg, ("pool", int(name[4:]) - 1, ii, int(top2.indices[ii, 1]))))
        else:
            a = r.abs().reshape(-1)
            m = min(n, a.numel())
            g, i = torch.topk(a, m, largest=False)
            for gg, ii in zip(g.tolist(), i.tolist()):
                acts.append((gg, ("act", name, ii)))
    # the two margins are not on one scale: interleave the two rankings
    acts.sort(key=lambda t: t[0])
    pools.sort(key=lambda t: t[0])
    out = []
    for a, p in itertools.zip_longest(acts, pools):
        out += [t[1] for t in (a, p) if t is not None]
    return out[:n]


def _apply(hooks, flips):
    hooks.force, hooks.pool_force = {}, {}
    for f in flips:
        if f[0] == "act":
            hooks.force[(f[1], f[2])] = True
        else:
            hooks.pool_force[(f[1], f[2])] = f[3]


def resolve_kinks(st, x, labels, cfg, err, tol, n_cand=16, max_flips=3):
    """Greedy search for the knife-edge flips under which the fp64 oracle's
    gradients reproduce the fixture: ``err(grads) -> float`` is the worst
    relative gradient error, ``tol`` the bar.  Each round tries flipping each
    of the n_cand most marginal candidates (on top of the flips already
    taken), stops at the first set that passes and otherwise keeps the best
    single improvement.  Returns (grads, flips, error); error > tol if no set
    of <= max_flips flips passes."""
    hooks = _Hooks()
    g = _run(st, x, labels, cfg, hooks)
    best_e, best_g, taken = err(g), g, []
    if best_e <= tol:
        return g, taken, best_e
    cand = candidates(hooks, n_cand)
    for _ in range(max_flips):
        step = None
        for c in cand:
            if c in taken:
                continue
            _apply(hooks, taken + [c])
            g = _run(st, x, labels, cfg, hooks)
            e = err(g)
            if e <= tol:
                return g, taken + [c], e
            if e < best_e and (step is None or e < step[0]):
                step = (e, c, g)
        if step is None:
            break
        best_e, best_g = step[0], step[2]
        taken = taken + [step[1]]
    return best_g, taken, best_e


class forced_branches:
    """Context manager: the oracle's LeakyReLUs and MaxPools take the given
    branch decisions (``masks`` as tests/test_gpu_parity.engine_branch_masks
    returns them: a bool sign mask per "<block>.<conv>" and an argmax-slot
    tensor per "pool1..3"), in whatever dtype the oracle runs."""

    def __init__(self, masks):
        self.masks = masks
        self.npool = 0
        self._dev = {}

    def _m(self, key, like):
        """The mask on the device the oracle runs on (moved once)."""
        m = self.masks[key]
        if m.device != like.device:
            if key not in self._dev:
                self._dev[key] = m.to(like.device)
            m = self._dev[key]
        return m

    def _lrelu(self, P, pre, inp, ksd):
        y = F.conv3d(inp, P[pre + ".0.weight"], None, padding=(ksd // 2, 1, 1))
        r = F.instance_norm(y, weight=P[pre + ".1.weight"], bias=P[pre + ".1.bias"], eps=1e-5)
        return torch.where(self._m(pre, r), r, 0.01 * r)

    def _pool(self, t):
        k = self.npool % 3
        self.npool += 1
        B_, C_, D_, H_, W_ = t.shape
        v = t[..., :H_ // 2 * 2, :W_ // 2 * 2].reshape(B_, C_, D_, H_ // 2, 2, W_ // 2, 2)
        v = v.permute(0, 1, 2, 3, 5, 4, 6)
        v = v.reshape(B_, C_, D_, H_ // 2, W_ // 2, 4)
        return v.gather(-1, self._m(f"pool{k + 1}", v).unsqueeze(-1)).squeeze(-1)

    def __enter__(self):
        self._orig = O.conv_in_lrelu, O.maxpool
        O.conv_in_lrelu, O.maxpool = self._lrelu, self._pool
        return self

    def __exit__(self, *exc):
        O.conv_in_lrelu, O.maxpool = self._orig
        return False
