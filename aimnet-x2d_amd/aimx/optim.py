"""Fused gradient clipping + Adam on the device (aimx_fused_adam, include/aimx.h).

Drop-in for the reference trainer's step (src/training/trainer.py:163-164, 221-223):

    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    optimizer.step()                      # optimizer = torch.optim.Adam(params, lr=...)

becomes

    optimizer = FusedAdam(params, lr=..., max_grad_norm=1.0)
    optimizer.step()

Same update as torch.optim.Adam (amsgrad=False, maximize=False), with the same param_groups /
state layout ('step', 'exp_avg', 'exp_avg_sq' per parameter), and the same in-place gradient
scaling clip_grad_norm_ performs. The whole step is three kernel launches independent of the
number of parameters, and it is graph-capturable: the step counter and the per-group learning
rates are device tensors. A scheduler that changes group['lr'] takes effect at the next eager
step; a captured graph reads the device copy, so call sync_lr() (outside the capture) after
changing lr when replaying a graph.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import AdamHyper, AdamTensor, AimxError, check, stream_ptr


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("FusedAdam: invalid hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = max_grad_norm
        self._step_t = None
        self._lr_t = None
        self._lr_host = None
        self._norm = None
        self._ws = None
        self._table_key = None
        self._arr = None

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._table_key = None  # state tensors replaced: rebuild the table on the next step

    def _build_table(self):
        """AdamTensor table of the parameters that have a gradient (torch.optim.Adam skips the
        others), with their state tensors and per-parameter step slots."""
        rows = []
        dev = None
        slot = -1
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                slot += 1
                if p.grad is None:
                    continue
                g = p.grad
                if not p.is_cuda or p.dtype != torch.float32 or g.dtype != torch.float32:
                    raise AimxError("FusedAdam: fp32 parameters on the HIP device only (no CPU path)")
                if not (p.is_contiguous() and g.is_contiguous()):
                    raise AimxError("FusedAdam: parameters and gradients must be contiguous")
                st = self.state[p]
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                dev = p.device
                rows.append((p, g, st["exp_avg"], st["exp_avg_sq"], gi, slot))
        self._rows, self._dev = rows, dev
        if not rows:
            self._arr = None
            return
        self._device_state(dev)
        for p, *_, k in rows:
            st, view = self.state[p], self._step_t[k]  # 0-dim view of this parameter's device counter
            old = st.get("step")
            if old is not None and (not torch.is_tensor(old) or old.data_ptr() != view.data_ptr()):
                view.fill_(float(old))  # a step count from load_state_dict
            st["step"] = view
        arr = (AdamTensor * len(rows))()
        for i, (p, g, m, v, gi, k) in enumerate(rows):
            arr[i].param, arr[i].grad = p.data_ptr(), g.data_ptr()
            arr[i].exp_avg, arr[i].exp_avg_sq = m.data_ptr(), v.data_ptr()
            arr[i].numel, arr[i].group, arr[i].step_slot = p.numel(), gi, k
        self._arr = arr
        self._wsb = _lib.load().aimx_fused_adam_workspace_bytes(arr, len(rows))

    def _shared_hyper(self):
        g0 = self.param_groups[0]
        for g in self.param_groups[1:]:
            if g["betas"] != g0["betas"] or g["eps"] != g0["eps"] or g["weight_decay"] != g0["weight_decay"]:
                raise AimxError("FusedAdam: parameter groups may differ in lr only")
        return g0

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._table_key = None  # new slots: the device arrays grow and the table is rebuilt

    def _device_state(self, dev):
        n = max(sum(len(g["params"]) for g in self.param_groups), 1)
        if self._step_t is None:
            # one step counter per parameter (torch.optim.Adam's state['step']), advanced on the
            # device only for parameters that have a gradient in that step
            self._step_t = torch.zeros(n, dtype=torch.float32, device=dev)
            self._norm = torch.zeros(1, dtype=torch.float32, device=dev)
            self._lr_t = torch.zeros(len(self.param_groups), dtype=torch.float32, device=dev)
        elif self._step_t.numel() < n or self._lr_t.numel() != len(self.param_groups):
            # add_param_group after the first step: slots are numbered over the groups in order, so
            # the new parameters' slots come after the existing ones, whose counters are kept
            step = torch.zeros(n, dtype=torch.float32, device=dev)
            step[: self._step_t.numel()].copy_(self._step_t)
            self._step_t = step
            k = 0
            for group in self.param_groups:  # re-point the 0-dim views (they index the old array)
                for p in group["params"]:
                    if p in self.state and "step" in self.state[p]:
                        self.state[p]["step"] = step[k]
                    k += 1
            self._lr_t = torch.zeros(len(self.param_groups), dtype=torch.float32, device=dev)
            self._lr_host = None
        lrs = [float(g["lr"]) for g in self.param_groups]
        if lrs != self._lr_host and not torch.cuda.is_current_stream_capturing():
            self._lr_t.copy_(torch.tensor(lrs, dtype=torch.float32))
            self._lr_host = lrs

    def sync_lr(self):
        """Push group['lr'] values to the device copy (call outside graph capture)."""
        if self._lr_t is not None:
            self._lr_host = None
            self._device_state(self._lr_t.device)

    @property
    def last_grad_norm(self):
        """Device tensor holding the total gradient norm of the last step (clip_grad_norm_'s value)."""
        return self._norm

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        hyper_g = self._shared_hyper()
        # the tensor table is rebuilt only when the set of stepped parameters changed (or a
        # parameter moved); a gradient that merely lives at a new address (eager steps with
        # zero_grad(set_to_none=True)) is patched into its row
        key = tuple((p.data_ptr(), p.grad is not None) for group in self.param_groups for p in group["params"])
        if key != self._table_key:
            self._build_table()
            self._table_key = key
        elif self._arr is not None:
            arr = self._arr
            for i, row in enumerate(self._rows):
                g = row[0].grad
                gp = g.data_ptr()
                if gp != arr[i].grad:
                    if g.dtype != torch.float32 or not g.is_contiguous() or not g.is_cuda:
                        raise AimxError("FusedAdam: gradients must be contiguous fp32 device tensors")
                    arr[i].grad = gp
                    self._rows[i] = (row[0], g) + tuple(row[2:])
        if self._arr is None:
            return loss
        rows, arr, dev = self._rows, self._arr, self._dev
        self._device_state(dev)  # group lr changes (schedulers)
        lib = _lib.load()
        wsb = self._wsb
        if self._ws is None or self._ws.numel() * 8 < wsb:
            # zero-filled once: holds aimx_fused_adam's self-resetting arrival counter
            self._ws = torch.zeros((wsb + 7) // 8, dtype=torch.float64, device=dev)
        h = AdamHyper()
        h.beta1, h.beta2 = hyper_g["betas"]
        h.one_minus_beta1, h.one_minus_beta2 = 1.0 - hyper_g["betas"][0], 1.0 - hyper_g["betas"][1]
        h.eps, h.weight_decay = hyper_g["eps"], hyper_g["weight_decay"]
        h.max_grad_norm = float(self.max_grad_norm) if self.max_grad_norm else 0.0
        check(lib.aimx_fused_adam(arr, len(rows), ctypes.byref(h), self._step_t.data_ptr(), self._lr_t.data_ptr(),
                                  self._norm.data_ptr(), self._ws.data_ptr(), self._ws.numel() * 8,
                                  stream_ptr(dev)), "fused_adam")
        return loss
