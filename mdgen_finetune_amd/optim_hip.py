"""The graphed training step's optimizer update on library kernels (csrc/optim.hip,
mdg_adam_step): global-norm gradient clipping + Adam / AdamW in two passes over HBM.

Reference semantics: the Lightning loop's gradient clipping (``gradient_clip_val``, train.py:52,
i.e. ``torch.nn.utils.clip_grad_norm_``) followed by the optimizer of
``configure_optimizers`` (wrapper.py:167-173, torch.optim.Adam or AdamW).  The update works on
the torch optimizer's own state tensors (``exp_avg``, ``exp_avg_sq``, ``step``), so checkpoints
(``optimizer.state_dict()``) and the eager path see the same state.  The gradients are read,
not clipped in place.
"""
import ctypes

import torch

from . import _lib


class FusedClipAdam:
    """clip_grad_norm_(params, max_norm) + optimizer.step() as three launches (mdg_adam_step).

    ``step(capturing=True)`` records the launches inside a stream capture; the device table of
    tensor addresses it reads is written by ``finish_capture()`` after the capture ends (the
    gradients' addresses are the capture's own allocations).  The table, workspace and norm
    buffers of a captured step come from ``reserve()``, called BEFORE the capture: memory the
    capture itself allocated may be reused by the graph's earlier kernels on every replay (the
    private pool recycles blocks freed within the capture), which would overwrite a table
    written once from the host."""

    def __init__(self, optimizer, params, max_norm):
        if not self.supported(optimizer):
            raise ValueError("FusedClipAdam: one Adam / AdamW parameter group without amsgrad / maximize")
        self.opt = optimizer
        self.params = list(params)
        self.max_norm = float(max_norm or 0.0)
        self._pending = []
        self._reserved = None
        self._keep = []  # tables / workspaces of every recorded step, referenced while graphs may replay

    def _sizes(self, ps):
        lib = _lib.load()
        tab = (_lib.MdgAdamTensor * len(ps))()
        for i, p in enumerate(ps):
            tab[i] = _lib.MdgAdamTensor(1, 1, 1, 1, 1, p.numel())
        nc = lib.mdg_adam_chunks(len(ps), tab)
        if nc <= 0:
            raise ValueError("FusedClipAdam: empty parameter")
        return lib.mdg_adam_table_bytes(len(ps), tab), lib.mdg_adam_workspace_bytes(nc)

    def _buffers(self, ps):
        tb, wsb = self._sizes(ps)
        dev = ps[0].device
        return (torch.empty(tb, dtype=torch.uint8, device=dev), torch.empty(wsb, dtype=torch.uint8, device=dev),
                torch.empty((), dtype=torch.float32, device=dev))

    def reserve(self):
        """Buffers for the next step(capturing=True), sized for every parameter (outside a capture)."""
        self._reserved = self._buffers([p for p in self.params if p.requires_grad])

    @staticmethod
    def supported(optimizer):
        if not isinstance(optimizer, (torch.optim.Adam, torch.optim.AdamW)) or len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        return not g.get("amsgrad", False) and not g.get("maximize", False) and not g.get("differentiable", False)

    def _state(self, p):
        st = self.opt.state[p]
        if "exp_avg" not in st:  # torch's lazy init (capturable form: the step on the device)
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        step = st["step"]
        if not (torch.is_tensor(step) and step.is_cuda and step.dtype == torch.float32):
            raise ValueError("FusedClipAdam: the optimizer's step counts must be fp32 device tensors (capturable)")
        return st["exp_avg"], st["exp_avg_sq"], step

    def step(self, capturing=False):
        """Returns the total gradient norm (a 0-d device tensor)."""
        lib = _lib.load()
        ps = [p for p in self.params if p.grad is not None]
        if not ps:
            raise ValueError("FusedClipAdam: no parameter has a gradient")
        tab = (_lib.MdgAdamTensor * len(ps))()
        for i, p in enumerate(ps):
            m, v, st = self._state(p)
            g = p.grad
            for t in (p, g, m, v):
                if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p.numel() or not t.is_cuda:
                    raise ValueError("FusedClipAdam: parameters, gradients and state must be contiguous fp32 "
                                     "device tensors of one shape")
            tab[i] = _lib.MdgAdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), st.data_ptr(),
                                        p.numel())
        n = len(ps)
        nc = lib.mdg_adam_chunks(n, tab)
        nbytes = lib.mdg_adam_table_bytes(n, tab)
        if nc <= 0 or nbytes == 0:
            raise ValueError("FusedClipAdam: empty parameter")
        host = (ctypes.c_uint8 * nbytes)()
        _lib.check(lib.mdg_adam_table_build(n, tab, host, nbytes), "mdg_adam_table_build")
        host_t = torch.frombuffer(bytearray(host), dtype=torch.uint8)
        if capturing:
            if self._reserved is None:
                raise RuntimeError("FusedClipAdam: reserve() the buffers before the capture")
            table, ws, gnorm = self._reserved
            self._reserved = None
        else:
            table, ws, gnorm = self._buffers(ps)
        wsb = lib.mdg_adam_workspace_bytes(nc)
        if table.numel() < nbytes or ws.numel() < wsb:
            raise RuntimeError("FusedClipAdam: reserved buffers too small")
        if not capturing:
            table[:nbytes].copy_(host_t)
        g = self.opt.param_groups[0]
        b1, b2 = g["betas"]
        decoupled = isinstance(self.opt, torch.optim.AdamW) or bool(g.get("decoupled_weight_decay", False))
        _lib.check(lib.mdg_adam_step(n, nc, table.data_ptr(), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                     float(g["weight_decay"]), int(decoupled), self.max_norm, gnorm.data_ptr(),
                                     ws.data_ptr(), wsb, _lib.stream_handle()), "mdg_adam_step")
        if capturing:  # a graph replays these buffers: keep them for the optimizer's lifetime
            self._pending.append((table, host_t))
            self._keep.append((table, ws, gnorm, host_t))
        # eager: the caching allocator recycles table / ws only after this stream's launch
        return gnorm

    def finish_capture(self):
        """Write the device tables of the launches recorded by step(capturing=True)."""
        for table, host_t in self._pending:
            table[:host_t.numel()].copy_(host_t)
        self._pending = []
        torch.cuda.synchronize()
