"""Device aggregation engine behind Strategy.server_ensemble.

`Aggregator.ensemble(agg_weight_lst, w_local_lst, key_lst)` is the MI355X replacement for
flearn/common/strategy/strategy.py:102-130: plan the buckets (bucket.py), copy the uploads into
HBM, run ONE fused reduce launch per bucket kind on torch's current stream, and hand back a
fresh dict with the reference's value types.

`ServerOptimizer` keeps the previous global model and the optimizer state v_t resident in HBM
and fuses the FedAVGM / FedOPT update (avgm.py:19-36, opt.py:23-65 — in the reference these run
in client_receive with w_local = the client's weights; here w_local = the previous global model)
into the same launch, so the server step reads every client byte once and touches the O(P)
state once.

Device-level entry points (`reduce_stack`, `apply_update`, `fill_uniform`) operate on torch CUDA
tensors directly and are what bench.py and the multi-GPU path use.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as na
from .bucket import BucketPlan, Packer, RowTable, make_plan
from .semantics import KIND_F32, KIND_F64, KIND_I64, Numerics

_F64 = np.dtype(np.float64)
_ONE_W32 = Numerics(KIND_F32, na.MODE_W32_DIV64, np.ones(1, np.float32), 1.0, np.dtype(np.float32), _F64)  # fl32(1.0)


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _check_cuda(t: torch.Tensor, name: str, dtype: torch.dtype, ndim: int | None = None):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")


def _epilogue(op: int, prev, v, beta=0.9, eta=1e-1, tau=1e-9, beta2=0.99, h=None, alpha=0.0, n_dyn=0, v_out=None):
    return na.Epilogue(op, 0, _ptr(prev), _ptr(v), beta, eta, tau, beta2, _ptr(h), alpha, float(n_dyn), _ptr(v_out))


def _byte_range(t: torch.Tensor, ncols: int):
    return t.data_ptr(), t.data_ptr() + ncols * t.element_size()


def _check_v_out(v_out, v, ncols, others=()):
    """v_out (the updated v / theta) must not share a byte with v, nor with the other operands
    the epilogue reads (prev, h): the kernel's stores would race its loads."""
    if v_out is None:
        return
    _check_cuda(v_out, "v_out", v.dtype)
    if v_out.numel() < ncols or not v_out.is_contiguous():
        raise ValueError("v_out too small or not contiguous")
    if v_out.data_ptr() == v.data_ptr():
        raise ValueError("v_out must be None (in place) or another buffer")
    o0, o1 = _byte_range(v_out, ncols)
    for name, t in (("v", v),) + tuple(others):
        if t is None or ncols == 0:
            continue
        a0, a1 = _byte_range(t, ncols)
        if o0 < a1 and a0 < o1:
            raise ValueError(f"v_out overlaps {name}")


# ---------------------------------------------------------------------------------------------
# device-level entry points
# ---------------------------------------------------------------------------------------------


def reduce_stack(
    stack: torch.Tensor,
    weights: torch.Tensor,
    mode: int,
    denom: float,
    *,
    col_begin: int = 0,
    n_cols: int | None = None,
    n_clients: int | None = None,
    out32: torch.Tensor | None = None,
    out64: torch.Tensor | None = None,
    op: int = na.OP_MEAN,
    prev: torch.Tensor | None = None,
    v: torch.Tensor | None = None,
    beta: float = 0.9,
    eta: float = 1e-1,
    tau: float = 1e-9,
    beta2: float = 0.99,
    h: torch.Tensor | None = None,
    alpha: float = 0.01,
    reorder: bool = False,
    v_out: torch.Tensor | None = None,
) -> None:
    """Weighted mean of the fp32 client stack [N, stride] over columns [col_begin, +n_cols)
    (+ fused update), queued on torch's current stream.  out32/out64/prev/v/h are indexed from
    col_begin.  weights: fp32 for MODE_W32_*, f64 for MODE_W64 (device tensors).
    op=OP_DYN: FedDyn with h (fp32, in place) and v = theta; prev unused.
    v_out: where the updated v / theta goes (None: back into v).  The fast form of a fused step
    is double-buffered — out32 not prev, v_out not v, the caller swapping the pairs — because
    stores onto the lines the epilogue has just loaded cost 1-3% (DESIGN.md §4 finding 20).
    reorder=True: allow fa_reduce_f32_splitn (client splits + a fixed tree: deterministic, within
    1e-6 normwise of the reference, not bit-exact) where it is faster — narrow windows, many
    clients; stack input only."""
    L = na.lib()
    rows = isinstance(stack, RowTable)  # device uploads read in place (fa_reduce_f32_rows)
    if rows:
        if stack.elem_size != 4 or not stack.aligned:
            raise ValueError("row table is not an aligned fp32 bucket")
        if col_begin != 0 or (n_cols is not None and n_cols != stack.shape[1]):
            raise ValueError("a row table is reduced over its whole bucket")
        if n_clients is not None and n_clients != stack.shape[0]:
            raise ValueError("a row table is reduced over all of its clients")
    else:
        _check_cuda(stack, "stack", torch.float32, 2)
        if stack.stride(1) != 1:
            raise ValueError("stack rows must be contiguous")
    n = stack.shape[0] if n_clients is None else n_clients
    if not 1 <= n <= stack.shape[0]:
        raise ValueError("n_clients out of range")
    ncols = stack.shape[1] - col_begin if n_cols is None else n_cols
    if col_begin < 0 or ncols < 0 or col_begin + ncols > stack.shape[1]:
        raise ValueError("column window out of range")
    wdt = torch.float64 if mode == na.MODE_W64 else torch.float32
    _check_cuda(weights, "weights", wdt)
    if weights.numel() < n:
        raise ValueError("fewer weights than clients")
    for name, t, dt in (("out32", out32, torch.float32), ("out64", out64, torch.float64)):
        if t is not None:
            _check_cuda(t, name, dt)
            if t.numel() < ncols or not t.is_contiguous():
                raise ValueError(f"{name} too small or not contiguous")
    epi = None
    if op == na.OP_DYN:
        vdt = torch.float32 if mode == na.MODE_W32_DIV32 else torch.float64
        _check_cuda(h, "h", torch.float32)
        _check_cuda(v, "theta", vdt)
        if h.numel() < ncols or v.numel() < ncols:
            raise ValueError("h / theta too small")
        _check_v_out(v_out, v, ncols, (("h", h),))
        epi = _epilogue(op, None, v, h=h, alpha=alpha, n_dyn=n, v_out=v_out)
    elif op != na.OP_MEAN:
        vdt = torch.float32 if mode == na.MODE_W32_DIV32 else torch.float64
        _check_cuda(prev, "prev", torch.float32)
        _check_cuda(v, "v", vdt)
        if prev.numel() < ncols or v.numel() < ncols:
            raise ValueError("prev / v too small")
        _check_v_out(v_out, v, ncols, (("prev", prev),))
        epi = _epilogue(op, prev, v, beta, eta, tau, beta2, v_out=v_out)
    if rows:
        pieces, npieces, grid = stack.piece_table(op)
        rc = L.fa_reduce_f32_rows(
            stack.ptrs.data_ptr(), n, mode, weights.data_ptr(), float(denom), pieces.data_ptr(), npieces, grid,
            stack.work.data_ptr(),
            ctypes.byref(epi) if epi is not None else None, _ptr(out32), _ptr(out64),
            na.stream_handle(stack.device),
        )
        na.check(rc, "fa_reduce_f32_rows")
        stack.release()
        return
    fn = L.fa_reduce_f32_splitn if reorder else L.fa_reduce_f32
    rc = fn(
        stack.data_ptr(), stack.stride(0), n, mode, weights.data_ptr(), float(denom), col_begin, ncols,
        ctypes.byref(epi) if epi is not None else None, _ptr(out32), _ptr(out64),
        na.stream_handle(stack.device),
    )
    na.check(rc, "fa_reduce_f32_splitn" if reorder else "fa_reduce_f32")


def reduce_stack_f64(stack, weights, denom, out64, n_clients=None):
    L = na.lib()
    _check_cuda(stack, "stack", torch.float64, 2)
    _check_cuda(weights, "weights", torch.float64)
    _check_cuda(out64, "out64", torch.float64)
    n = stack.shape[0] if n_clients is None else n_clients
    rc = L.fa_reduce_f64(stack.data_ptr(), stack.stride(0), n, weights.data_ptr(), float(denom), 0,
                         stack.shape[1], out64.data_ptr(), na.stream_handle(stack.device))
    na.check(rc, "fa_reduce_f64")


def reduce_stack_i64(stack, weights, denom, out64, n_clients=None):
    L = na.lib()
    _check_cuda(stack, "stack", torch.int64, 2)
    _check_cuda(weights, "weights", torch.int64)
    _check_cuda(out64, "out64", torch.float64)
    n = stack.shape[0] if n_clients is None else n_clients
    rc = L.fa_reduce_i64(stack.data_ptr(), stack.stride(0), n, weights.data_ptr(), float(denom), 0,
                         stack.shape[1], out64.data_ptr(), na.stream_handle(stack.device))
    na.check(rc, "fa_reduce_i64")


def apply_update(op: int, local32, glob, v, *, out32=None, out64=None, beta=0.9, eta=1e-1, tau=1e-9,
                 beta2=0.99) -> None:
    """Standalone AVGM/OPT update (client_receive form): w = update(glob, local32, v)."""
    L = na.lib()
    prec = na.PREC_F64 if glob.dtype == torch.float64 else na.PREC_F32
    _check_cuda(local32, "local", torch.float32)
    _check_cuda(glob, "glob", torch.float64 if prec == na.PREC_F64 else torch.float32)
    _check_cuda(v, "v", glob.dtype)
    n = local32.numel()
    if glob.numel() != n or v.numel() != n:
        raise ValueError("local / glob / v sizes differ")
    epi = _epilogue(op, local32, v, beta, eta, tau, beta2)
    rc = L.fa_opt_apply(prec, ctypes.byref(epi), local32.data_ptr(), glob.data_ptr(), n, _ptr(out32),
                        _ptr(out64), na.stream_handle(local32.device))
    na.check(rc, "fa_opt_apply")


def apply_dyn(glob, h, theta, n_clients: int, alpha: float = 0.01, *, out32=None, out64=None) -> None:
    """Standalone FedDyn step on a computed mean (dyn.py:17-36): h and theta in place,
    w -> out32/out64 (which may alias glob / theta)."""
    L = na.lib()
    prec = na.PREC_F64 if glob.dtype == torch.float64 else na.PREC_F32
    _check_cuda(glob, "glob", torch.float64 if prec == na.PREC_F64 else torch.float32)
    _check_cuda(h, "h", torch.float32)
    _check_cuda(theta, "theta", glob.dtype)
    n = glob.numel()
    if h.numel() != n or theta.numel() != n:
        raise ValueError("glob / h / theta sizes differ")
    epi = _epilogue(na.OP_DYN, None, theta, h=h, alpha=alpha, n_dyn=n_clients)
    rc = L.fa_opt_apply(prec, ctypes.byref(epi), None, glob.data_ptr(), n, _ptr(out32), _ptr(out64),
                        na.stream_handle(glob.device))
    na.check(rc, "fa_opt_apply")


def set_reduce_grid(grid: int) -> int:
    """Blocks of the fp32 stack reduce, process-wide (fa_set_reduce_grid): 0 = the library's
    choice; fewer leave CUs to kernels running beside the reduce (RCCL's gather in the multi-GPU
    pipeline).  Returns the previous setting.  Results never depend on it."""
    L = na.load()
    rc = L.fa_set_reduce_grid(int(grid))
    if rc < 0:
        na.check(rc, "fa_set_reduce_grid")
    return rc


def fill_uniform(dst: torch.Tensor, seed: int, row_begin: int = 0, col_begin: int = 0,
                 n_cols: int | None = None) -> None:
    """Synthetic client data on device: dst[r, c] = U(-1,1) hash of (seed, row_begin+r,
    col_begin+c) for c < n_cols (default: all columns)."""
    L = na.lib()
    _check_cuda(dst, "dst", torch.float32)
    d2 = dst if dst.dim() == 2 else dst.view(1, -1)
    ncols = d2.shape[1] if n_cols is None else n_cols
    for r0 in range(0, d2.shape[0], 65535):
        rows = min(65535, d2.shape[0] - r0)
        rc = L.fa_fill_uniform_f32(d2[r0].data_ptr(), d2.stride(0), rows, ncols, seed & (2**64 - 1),
                                   row_begin + r0, col_begin, na.stream_handle(dst.device))
        na.check(rc, "fa_fill_uniform_f32")


def mean_tables(tables, device=None):
    """FedDistill's logits mean (distill.py:42-46) on the device: user_logits = 0, += each table
    in list order, / len(tables), in the tables' dtype (fp32 or f64), bit-identical to torch /
    numpy on the host.  One reduce launch over a [N+1, C*C] stack whose row 0 is zeros with
    weight 1 (so the sum starts from +0.0 exactly as `0 + t0` does) and weights 1 elsewhere.
    Returns the container type of tables[0] (torch tensor on its device, or ndarray)."""
    if len(tables) == 0:
        raise ZeroDivisionError("division by zero")  # 0 / len([])  distill.py:46
    first = tables[0]
    as_torch = isinstance(first, torch.Tensor)
    host = [t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t) for t in tables]
    dt, shape = host[0].dtype, host[0].shape
    for a in host[1:]:
        if a.dtype != dt or a.shape != shape:
            raise ValueError(f"logits tables differ: {a.dtype}{a.shape} vs {dt}{shape}")
    if dt not in (np.float32, np.float64):
        raise NotImplementedError(f"logits dtype {dt}: the device mean handles float32 / float64 tables")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    n, m = len(host), int(np.prod(shape, dtype=np.int64))
    stride = max(64, -(-m // 64) * 64)
    stack = np.zeros((n + 1, stride), dtype=dt)
    for i, a in enumerate(host):
        stack[i + 1, :m] = a.reshape(-1)
    tdt = torch.float32 if dt == np.float32 else torch.float64
    with torch.cuda.device(dev):
        sd = torch.from_numpy(stack).to(dev)
        w = torch.ones(n + 1, dtype=tdt, device=dev)
        out = torch.empty(stride, dtype=tdt, device=dev)
        if tdt == torch.float32:
            reduce_stack(sd, w, na.MODE_W32_DIV32, float(n), out32=out)  # fp32 sum, fp32 / fl32(N)
        else:
            reduce_stack_f64(sd, w, float(n), out)
        res = out[:m].view(shape)
        if as_torch:
            return res.to(first.device).clone() if first.device != dev else res.clone()
        return res.cpu().numpy()


# ---------------------------------------------------------------------------------------------
# server-side optimizer state
# ---------------------------------------------------------------------------------------------


class ServerOptimizer:
    """FedAVGM / FedOPT state for the fused server step.

    op     : "avgm" | "adagrad" | "yogi" | "adam"
    state  : per column shard (one per device), prev (fp32 previous global, flattened like the
             f32 bucket) and v_t (f64, or fp32 when the weights make the reference's w_glob
             float32), resident in HBM and never communicated.
    First round without `init_global`: the update is skipped (the mean is returned), prev is set
    to the fp32 mean and v_t to zeros — the reference has no previous global model either.
    """

    def __init__(self, op: str, beta=0.9, eta=1e-1, tau=1e-9, beta2=0.99):
        if op not in ("avgm", "adagrad", "yogi", "adam"):
            raise ValueError(f"unknown server optimizer {op!r}")
        self.op = na.OP_BY_NAME[op]
        self.name = op
        self.beta, self.eta, self.tau, self.beta2 = beta, eta, tau, beta2
        self.state = {}  # shard index -> (prev, v): the current previous global model and v_t
        self.spare = {}  # shard index -> (prev, v) buffers the next fused step writes into
        self._sig = None
        self._pending_init = None
        self._pending_v = None
        self._plan = None  # the bucket plan the state is bound to (the last round's)
        self.group = None  # (process group, world) when bound to a column-sharded Aggregator

    def init_global(self, glob: dict):
        """Set the previous global model (dict of arrays/tensors); v_t is reset to zeros."""
        self._pending_init = {k: _host_array(v) for k, v in glob.items()}
        self._pending_v = None
        self.state, self._sig = {}, None

    def set_v_t(self, v_t: dict):
        """Restore v_t — the dict `v_t()` returns (keyed like w_glob, f64, or fp32 when the
        weights make w_glob float32) — for the next fused round.  Follows `init_global` (or
        `load_state`): the state a restarted server needs is the previous global model AND v_t
        (avgm.py:28-32 / opt.py:45-60 keep v_t across rounds).  Applied when the next round binds
        the state to its bucket; a key of the model that v_t lacks, or a shape that differs,
        raises there (KeyError / ValueError)."""
        if self._pending_init is None:
            raise RuntimeError("set_v_t restores v_t next to a previous global model: call init_global(w_glob) "
                               "first (or load_state)")
        self._pending_v = {k: _host_array(v) for k, v in v_t.items()}

    def load_state(self, state: dict):
        """Restore what `state_dict()` returned ({"w_glob": previous global, "v_t": v_t}; without
        "v_t" it is zeros, as after init_global)."""
        self.init_global(state["w_glob"])
        if state.get("v_t") is not None:
            self.set_v_t(state["v_t"])

    def state_dict(self, plan: BucketPlan | None = None) -> dict:
        """{"w_glob": the fp32 previous global model the next fused round starts from, "v_t":
        v_t()} as host arrays keyed like w_glob (plan: the last round's by default): what
        `load_state` restores on a fresh optimizer.  With a column-sharded process group this is a
        collective (two all-gathers)."""
        return {"w_glob": self._host_dict(plan, 0), "v_t": self._host_dict(plan, 1)}

    @staticmethod
    def _signature(plan: BucketPlan, shards):
        g = plan.f32
        return (tuple((s.key, s.shape) for s in g.segments), g.numerics.out_dtype.str,
                tuple((sh.device, sh.c0, sh.c1) for sh in shards))

    @staticmethod
    def _vdtype(plan):
        return torch.float32 if plan.f32.numerics.out_dtype == np.float32 else torch.float64

    def prepare(self, plan: BucketPlan, shards) -> bool:
        """Bind the state to this plan's f32 bucket.  Returns False when there is no previous
        model yet (first round): the caller then runs a plain mean and calls `adopt`."""
        g = plan.f32
        sig = self._signature(plan, shards)
        if self._pending_init is not None:
            prev = np.zeros(g.stride, dtype=np.float32)
            vdt = np.float32 if self._vdtype(plan) == torch.float32 else np.float64
            vflat = np.zeros(g.stride, dtype=vdt)
            for s in g.segments:
                prev[s.offset : s.offset + s.numel] = np.asarray(self._pending_init[s.key], np.float32).reshape(-1)
                if self._pending_v is not None:
                    if s.key not in self._pending_v:
                        raise KeyError(s.key)
                    v = np.asarray(self._pending_v[s.key])
                    if tuple(v.shape) != tuple(s.shape):
                        raise ValueError(f"v_t[{s.key!r}] shape {v.shape} != model shape {tuple(s.shape)}")
                    vflat[s.offset : s.offset + s.numel] = v.astype(vdt, copy=False).reshape(-1)
            self.state = {
                sh.index: (torch.from_numpy(prev[sh.c0 : sh.c1].copy()).to(sh.device),
                           torch.from_numpy(vflat[sh.c0 : sh.c1].copy()).to(sh.device))
                for sh in shards
            }
            self._sig, self._plan = sig, plan
            self._pending_init = self._pending_v = None
            return True
        if self._sig is None:
            return False
        if sig != self._sig:
            raise ValueError("model layout changed between rounds; call init_global() again")
        self._plan = plan
        return True

    def adopt(self, plan: BucketPlan, shards, means: dict):
        """First round: the fp32 mean becomes prev, v_t = 0.  means: shard index -> fp32 tensor."""
        self.state = {sh.index: (means[sh.index][: sh.width].clone(),
                                 torch.zeros(sh.width, dtype=self._vdtype(plan), device=sh.device))
                      for sh in shards}
        self._sig, self._plan = self._signature(plan, shards), plan

    def swap_buffers(self, sh):
        """(prev, v, prev_out, v_out) of a fused step on shard sh, and the state advanced to the
        output pair: the step reads the current pair and writes the other one (double-buffered,
        DESIGN.md §4 finding 20); the pair it read becomes the next step's output."""
        prev, v = self.state[sh.index]
        spare = self.spare.get(sh.index)
        if spare is None or spare[0].shape != prev.shape or spare[1].dtype != v.dtype or spare[0].device != prev.device:
            spare = (torch.empty_like(prev), torch.empty_like(v))
        self.state[sh.index], self.spare[sh.index] = spare, (prev, v)
        return prev, v, spare[0], spare[1]

    def unswap(self, sh):
        """Undo swap_buffers(sh) when the fused step it was for did not run (the state keeps the
        pair it had: the spare buffers hold nothing yet)."""
        self.state[sh.index], self.spare[sh.index] = self.spare[sh.index], self.state[sh.index]

    def v_t(self, plan: BucketPlan | None = None) -> dict:
        """The state as the reference exposes it (self.v_t dict of arrays; plan: the last round's by
        default).  With a column-sharded
        process group (Aggregator(group=...)) every rank holds only its columns: this is then a
        collective (an all-gather) that every rank must call."""
        return self._host_dict(plan, 1)

    def _host_dict(self, plan: BucketPlan, i: int) -> dict:
        """State i (0: prev, 1: v_t) over the whole bucket, keyed like w_glob."""
        plan = plan if plan is not None else self._plan
        if not self.state or plan is None:
            raise RuntimeError("no server optimizer state yet (no fused round has run)")
        if self.group is not None:
            from .bucket import rank_width
            from .dist import gather_columns

            (loc,) = [self.state[j][i] for j in sorted(self.state)]
            group, world = self.group
            stride = plan.f32.stride
            host = gather_columns(loc, rank_width(stride, world), stride, group).cpu().numpy()
        else:
            host = np.concatenate([self.state[j][i].cpu().numpy() for j in sorted(self.state)])
        return {s.key: host[s.offset : s.offset + s.numel].reshape(s.shape).copy() for s in plan.f32.segments}


def _host_array(v):
    return np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v)


def _as_host(v):
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v


class DynState:
    """FedDyn server state (flearn/common/strategy/dyn.py:10-36), resident in HBM.

    h      : the caller's dict (a model state_dict).  fp32 entries for fp32 model keys live on the
             device as one flat fp32 array per column shard, laid out like the f32 bucket, and are
             updated in place by the fused epilogue; `sync_h()` copies them back into the
             caller's arrays (the reference mutates them in place, dyn.py:26).  Integer entries
             (BN counters) are the keys whose in-place float update numpy refuses: the reference
             skips them (dyn.py:24-31) and so do we — w_glob keeps the plain mean there.
    theta  : per shard, in the precision numpy gives w_glob (f64 for Python-float weights, fp32
             for np.float32 weights); starts as a copy of h (dyn.py:14) and becomes w_glob each
             round (dyn.py:34).
    One launch per round: mean, delta_theta, h, w and theta for every fp32 column.  When h does
    not cover every fp32 key, the mean is computed first and the update is applied to the
    covered column runs only.
    """

    op = na.OP_DYN
    name = "dyn"

    def __init__(self, h, alpha: float = 0.01):
        self.alpha = alpha
        self.h_host = h
        self._theta_init = None if h is None else {k: np.array(_as_host(v), copy=True) for k, v in h.items()}
        self.state = {}  # shard index -> (h fp32, theta)
        self._spare = {}  # shard index -> the theta buffer the next fused round writes into
        self._sig = None
        self._tdt = None
        self._dirty = False
        self._covered = True
        self.dev_keys = ()
        self.skipped = ()
        self.group = None  # (process group, world) when bound to a column-sharded Aggregator

    # -- state management -------------------------------------------------------------------
    def set_h(self, h):
        """Replace h (uploaded at the next round); theta is kept."""
        self.sync_h()
        if self.state:
            self._theta_init = self.theta_host()
        self.h_host, self.state, self._sig = h, {}, None

    def set_theta(self, theta):
        self.sync_h()
        self._theta_init = {k: np.array(_as_host(v), copy=True) for k, v in theta.items()}
        self.state, self._sig = {}, None

    def classify(self, plan: BucketPlan):
        """(device keys, skipped keys) of h for this plan; raises like the reference would."""
        if self.h_host is None:
            raise AttributeError("FedDyn h is None (dyn.py:20 iterates self.h.keys())")
        dev, skip = [], []
        for k, hv in self.h_host.items():
            if k not in plan.key_group:
                raise KeyError(k)  # dyn.py:21: w_glob[k]
            a = _as_host(hv)
            if not isinstance(a, np.ndarray):
                raise NotImplementedError(f"FedDyn h[{k!r}] is a {type(a).__name__}, expected an array")
            if np.issubdtype(a.dtype, np.integer) or a.dtype == np.bool_:
                skip.append(k)  # h[k] -= float array raises in numpy: skipped  dyn.py:24-29
                continue
            seg = plan.key_segment[k]
            if plan.key_group[k] != KIND_F32 or a.dtype != np.float32:
                raise NotImplementedError(
                    f"FedDyn h[{k!r}] ({a.dtype}) on a {plan.key_group[k]} key: only fp32 h on fp32 keys runs on the device")
            if tuple(a.shape) != tuple(seg.shape):
                raise ValueError(f"FedDyn h[{k!r}] shape {a.shape} != model shape {seg.shape}")
            dev.append(k)
        return dev, skip

    def prepare(self, plan: BucketPlan, shards) -> bool:
        g = plan.f32
        dev, skip = self.classify(plan)
        tdt = torch.float32 if g.numerics.out_dtype == np.float32 else torch.float64
        sig = (tuple((s.key, s.shape) for s in g.segments), tuple(dev),
               tuple((sh.device, sh.c0, sh.c1) for sh in shards))
        if not self.state:
            hflat = np.zeros(g.stride, dtype=np.float32)
            tflat = np.zeros(g.stride, dtype=np.float64)
            for k in dev:
                s = plan.key_segment[k]
                hflat[s.offset : s.offset + s.numel] = np.asarray(_as_host(self.h_host[k])).reshape(-1)
                t0 = np.asarray(self._theta_init[k], dtype=np.float64).reshape(-1)
                tflat[s.offset : s.offset + s.numel] = t0
            self.state = {
                sh.index: (torch.from_numpy(hflat[sh.c0 : sh.c1].copy()).to(sh.device),
                           torch.from_numpy(tflat[sh.c0 : sh.c1].copy()).to(sh.device, tdt))
                for sh in shards
            }
            self._sig, self._tdt = sig, tdt
        elif sig != self._sig:
            raise ValueError("model layout changed between FedDyn rounds; set h again")
        elif tdt != self._tdt:
            raise TypeError("FedDyn: the weights' type changed between rounds (theta precision)")
        self.dev_keys, self.skipped = tuple(dev), tuple(skip)
        self._covered = len(dev) == len(g.segments)
        self._plan_f32 = g
        return True

    def step(self, agg: "Aggregator", sh, stack, w, nm: Numerics, want64: bool):
        """The fused round for one shard: returns the output tensor (theta itself for f64)."""
        hs, th = self.state[sh.index]
        f64 = th.dtype == torch.float64
        self._dirty = True
        if self._covered:
            out32 = None if want64 else agg.packer.device_bucket(("out32", KIND_F32, sh.index), (sh.width,),
                                                                   torch.float32, sh.device)
            # theta double-buffered (read one, write the other, swap; DESIGN.md §4 finding 20); h, the
            # caller-visible state synced back by sync_h, stays in place
            th_o = self._spare.get(sh.index)
            if th_o is None or th_o.shape != th.shape or th_o.dtype != th.dtype or th_o.device != th.device:
                th_o = torch.empty_like(th)
            reduce_stack(stack, w, nm.mode, nm.denom, out32=out32, out64=th_o if want64 else None,
                         op=na.OP_DYN, v=th, v_out=th_o, h=hs, alpha=self.alpha)
            self.state[sh.index], self._spare[sh.index] = (hs, th_o), th
            return th_o if want64 else out32
        # partial coverage: mean in theta's precision, then the update on the covered runs
        gbuf = agg.packer.device_bucket(("dyn_g", KIND_F32, sh.index), (sh.width,), th.dtype, sh.device)
        reduce_stack(stack, w, nm.mode, nm.denom, out32=None if f64 else gbuf, out64=gbuf if f64 else None)
        for a, b in self._runs(sh):
            gs = gbuf[a:b]
            apply_dyn(gs, hs[a:b], th[a:b], stack.shape[0], self.alpha,
                      out64=gs if f64 else None, out32=None if f64 else gs)
        if want64 or not f64:
            return gbuf
        return gbuf.to(torch.float32)

    def _runs(self, sh):
        """Maximal column runs [a, b) of device keys within the shard, shard-relative."""
        segs = sorted((s.offset, s.offset + s.numel) for s in self._plan_f32.segments if s.key in set(self.dev_keys))
        runs = []
        for lo, hi in segs:
            lo, hi = max(lo, sh.c0), min(hi, sh.c1)
            if lo >= hi:
                continue
            if runs and runs[-1][1] == lo - sh.c0:
                runs[-1][1] = hi - sh.c0
            else:
                runs.append([lo - sh.c0, hi - sh.c0])
        return runs

    # -- host views ---------------------------------------------------------------------------
    def _host_flat(self, i):
        """State i (0: h, 1: theta) over the whole bucket.  With a column-sharded process group
        every rank holds only its columns: this is then a collective (an all-gather) that every
        rank must call — reading `Dyn.h`, `set_h`, `set_theta` included."""
        if self.group is not None:
            from .bucket import rank_width
            from .dist import gather_columns

            (loc,) = [self.state[j][i] for j in sorted(self.state)]
            group, world = self.group
            stride = self._plan_f32.stride
            return gather_columns(loc, rank_width(stride, world), stride, group).cpu().numpy()
        return np.concatenate([self.state[j][i].cpu().numpy() for j in sorted(self.state)])

    def sync_h(self):
        """Copy the device h into the caller's arrays (in place) and return the dict."""
        if self._dirty and self.state:
            flat = self._host_flat(0)
            for k in self.dev_keys:
                s = self._plan_f32_segment(k)
                val = flat[s.offset : s.offset + s.numel].reshape(s.shape)
                dst = self.h_host[k]
                if isinstance(dst, torch.Tensor):
                    dst.copy_(torch.from_numpy(val))
                else:
                    np.copyto(dst, val)
            self._dirty = False
        return self.h_host

    def theta_host(self) -> dict:
        flat = self._host_flat(1)
        out = dict(self._theta_init)
        for k in self.dev_keys:
            s = self._plan_f32_segment(k)
            out[k] = flat[s.offset : s.offset + s.numel].reshape(s.shape).copy()
        return out

    def _plan_f32_segment(self, k):
        for s in self._plan_f32.segments:
            if s.key == k:
                return s
        raise KeyError(k)


# ---------------------------------------------------------------------------------------------
# the engine behind Strategy.server_ensemble
# ---------------------------------------------------------------------------------------------

OUTPUTS = ("reference", "float32", "device")


class Aggregator:
    """output: "reference" — values with the reference's types and dtypes (float64 ndarrays, numpy
    scalars for 0-d buffers, torch CPU tensors when the uploads were tensors);
    "float32" — fp32 ndarrays for fp32 keys (the values load_state_dict ends up with);
    "device" — fresh torch CUDA tensors on the first device, fp32 for fp32 keys (no D2H).

    devices: the HIP devices the f32 bucket is split over (column shards); each ingests its
    columns through its own PCIe link.  Default: torch's current device only."""

    #: small host rounds (_small_round): the reduce kernel reads the uploads straight from the
    #: pinned staging and writes the result into pinned host memory (zero-copy over PCIe) instead
    #: of an H2D copy, the launch and a D2H copy: C1 server call 141 -> 123 us on one box, same
    #: process, bit-equal (tools/prof_host_c1.py --ab, profiles/r03/c1_zc/); False = copy engines
    small_zero_copy = True
    #: the zero-copy fp32 bucket of a small round may be summed in this many chained launches
    #: (client parts, each launched as soon as native threads have packed it: bucket.AsyncPack);
    #: 1 = one native pack on the calling thread, one launch.  At flearn's config 1 every extra
    #: launch costs more than the overlap saves: 1 / 2 / 3 / 4 launches 113.5 / 120.3 / 127.4 /
    #: 135.7 us per server call, numpy 142 us (tools/prof_host_c1.py --parts, profiles/r04/c1_parts/)
    small_parts = 1

    def __init__(self, device=None, output: str = "reference", workers: int = 8, devices=None, group=None,
                 reorder: bool = False):
        na.lib()  # fail loudly right away if the HIP path is unavailable
        if output not in OUTPUTS:
            raise ValueError(f"output must be one of {OUTPUTS}")
        if group is not None and devices is not None and len(devices) > 1:
            raise ValueError("group (one GPU per process) and devices (several GPUs in this process) exclude each other")
        if devices is None:
            devices = [torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())]
        self.devices = [torch.device(d) for d in devices]
        self.device = self.devices[0]
        self.output = output
        self.reorder = reorder  # allow the split-N kernel (not bit-exact; <= 1e-6 normwise)
        self.packer = Packer(self.devices, workers)
        # group: this process is one rank of a column-sharded aggregation (flearn_amd.dist): it
        # packs and reduces only its columns of the fp32 bucket and an RCCL all-gather over xGMI
        # reassembles the global model on every rank.  True = the default process group.
        self.group = None
        if group is not None:
            import torch.distributed as dist

            self.group = None if group is True else group
            if not dist.is_initialized():
                raise RuntimeError("group= needs torch.distributed initialised (one process per GPU)")
            self.packer.rank_cols = (dist.get_rank(self.group), dist.get_world_size(self.group))
            self._dist = True
        else:
            self._dist = False
        self.last_plan: BucketPlan | None = None
        self._wcache = {}  # (device, dtype, bytes) -> device weights: a pageable H2D per round saved

    def _weights(self, nm: Numerics, device) -> torch.Tensor:
        key = (str(device), nm.weights.dtype.str, nm.weights.tobytes())
        t = self._wcache.get(key)
        if t is None:
            if len(self._wcache) >= 64:
                self._wcache.clear()
            t = self._wcache[key] = torch.from_numpy(np.ascontiguousarray(nm.weights)).to(device)
        return t

    def ensemble(self, agg_weight_lst, w_local_lst, key_lst=None, server_opt: ServerOptimizer | None = None):
        plan = make_plan(agg_weight_lst, w_local_lst, key_lst)
        self.last_plan = plan
        if server_opt is None and not self._dist and len(self.devices) == 1 and self.output != "device":
            glob = self._small_round(plan, w_local_lst)
            if glob is not None:
                return glob
        stacks = self.packer.pack(plan, w_local_lst)
        fused = False
        self._post_denom = None
        if server_opt is not None and KIND_F32 in plan.groups:
            if self._dist:
                server_opt.group = (self.group, self.packer.rank_cols[1])
            fused = server_opt.prepare(plan, [sh for sh, _ in stacks[KIND_F32]])
        results = {}
        first_means = {}
        for kind, parts in stacks.items():
            g = plan.groups[kind]
            nm = g.numerics
            res = []
            for sh, stack in parts:
                with torch.cuda.device(sh.device):
                    w = self._weights(nm, sh.device)
                    if kind == KIND_F32:
                        out = self._reduce_f32(g, sh, stack, w, server_opt, fused, first_means)
                    else:
                        out = self.packer.device_bucket(("out64", kind, sh.index), (sh.width,), torch.float64, sh.device)
                        (reduce_stack_f64 if kind == KIND_F64 else reduce_stack_i64)(stack, w, nm.denom, out)
                res.append((sh, out))
            results[kind] = res
            if self.packer.last_row_tables.get(kind) == "slab":  # the caller's memory, read in place:
                self.packer.hold([st for _, st in parts], parts[0][0].device)  # alive until read
        if server_opt is not None and first_means:
            server_opt.adopt(plan, [sh for sh, _ in stacks[KIND_F32]], first_means)
        if self._dist and KIND_F32 in results:
            results[KIND_F32] = self._gather_columns(plan, results[KIND_F32])
        return self._finish(plan, results)

    # -- small host rounds ---------------------------------------------------------------------
    def _small_record(self, plan: BucketPlan, w_local_lst):
        """The prebuilt round of a small host-upload plan (every bucket together < SMALL_BYTES:
        LeNet-sized models, flearn's config 1), cached on the plan: per bucket kind its own
        pinned staging, device stack, device weights and result buffers, the native pack table
        and the ctypes arguments of its reduce launch, and the (key, offset, size, shape) list
        of the result.  None (cached as False) when the plan does not qualify."""
        zc = bool(self.small_zero_copy)
        key = ("small_round", id(self.packer), str(self.device), self.output, zc, int(self.small_parts))
        rec = plan.memo.get(key)
        if rec is not None:
            return rec or None
        from .bucket import _FMT, SMALL_BYTES, AsyncPack, Packer, Shard, _NativeRows, _STORE, _TORCH

        n = plan.n_clients
        total = sum(n * g.stride * np.dtype(_STORE[k]).itemsize for k, g in plan.groups.items())
        if plan.input_kind != "numpy" or total >= SMALL_BYTES or not plan.groups:
            plan.memo[key] = False
            return None
        L, dev = na.lib(), self.device
        kinds = []
        for kind, g in plan.groups.items():
            tdt = _TORCH[_STORE[kind]]
            pieces = Packer._pieces(g, [Shard(0, dev, 0, g.stride)])
            # spare rows: the chained zero-copy round's partial sums (below)
            parts = max(1, min(int(self.small_parts), n // 2))
            host = torch.zeros((n + parts - 1, g.stride), dtype=tdt, pin_memory=True)
            if not _NativeRows.usable(pieces, [host]):
                plan.memo[key] = False
                return None
            nat = _NativeRows(pieces, [host], w_local_lst, [None] * n)
            nm = g.numerics
            w = self._weights(nm, dev)
            f64 = kind != KIND_F32 or (self.output == "reference" and nm.out_dtype == _F64)
            odt = torch.float64 if f64 else torch.float32
            hout = torch.empty(g.stride, dtype=odt, pin_memory=True)
            if zc:  # the kernel reads the pinned staging and writes the pinned result over PCIe
                stack, dout = host, hout
            else:
                stack = torch.empty((n, g.stride), dtype=tdt, device=dev)
                dout = torch.empty(g.stride, dtype=odt, device=dev)
            split = None
            if kind == KIND_F32:
                fn = L.fa_reduce_f32
                args = (stack.data_ptr(), g.stride, n, nm.mode, w.data_ptr(), float(nm.denom), 0, g.stride, None,
                        None if f64 else dout.data_ptr(), dout.data_ptr() if f64 else None)
                if zc and parts >= 2 and nm.mode in (na.MODE_W32_DIV64, na.MODE_W32_DIV32):
                    split = self._small_chain(g, pieces, host, w, nm, dout, f64, n, parts, dev, AsyncPack, _FMT)
            else:
                fn = L.fa_reduce_f64 if kind == KIND_F64 else L.fa_reduce_i64
                args = (stack.data_ptr(), g.stride, n, w.data_ptr(), float(nm.denom), 0, g.stride, dout.data_ptr())
            out = [(s.key, s.offset, s.numel, s.shape) for s in g.segments]
            kinds.append((nat, host, stack, w, dout, hout, hout.numpy(), fn, args, out, split))
        g32 = plan.groups.get(KIND_F32)
        wsig = (tuple((s.key, s.shape, s.offset) for s in g32.segments) + (g32.stride,)) if g32 is not None else None
        rec = plan.memo[key] = (tuple(kinds), na.load_pyhost().fa_py_pack_rows, wsig)
        return rec

    @staticmethod
    def _small_chain(g, pieces, host, w, nm, dout, f64, n, parts, dev, AsyncPack, fmt_of):
        """The fp32 bucket of a small zero-copy round as `parts` chained launches.  Clients are cut
        into parts b_0 = 0 < b_1 < ... < b_K = n (the first smallest, so the GPU starts early);
        client i of part k sits in staging row i + k.  Launch 0 sums rows [0, b_1) in fp32 (mode
        W32_DIV32 with W = 1: the epilogue returns the sum itself) into row b_1; launch k sums
        rows [b_k + k - 1, b_{k+1} + k) — the previous partial with weight fl32(1.0), then part
        k's clients — into row b_{k+1} + k, the last one with the real denominator and output.
        fl32(1 * acc) = acc, so the chain of adds is the single launch's, bit for bit, and no
        launch writes a row it reads.  The parts are packed by native threads
        (AsyncPack chunk k = part k) and each launch waits only for its own part.
        Returns ("chain", AsyncPack, [launch args], [weight tensors kept alive])."""
        base, rem = divmod(n, parts)
        sizes = [base] * parts
        for j in range(rem):  # the remainder goes to the last parts
            sizes[parts - 1 - j] += 1
        bounds = [0]
        for s_ in sizes:
            bounds.append(bounds[-1] + s_)
        row = g.stride * 4
        hp = host.data_ptr()
        rows = []
        for k in range(parts):
            for i in range(bounds[k], bounds[k + 1]):
                for s, a, b, _sh, d in pieces:
                    it = s.src_dtype.itemsize
                    rows.append((i, s.numel * it, fmt_of[s.src_dtype], hp + (i + k) * row + d * it, k, a * it,
                                 (b - a) * it))
        keys = tuple(s.key for s, *_ in pieces) * n
        ap = AsyncPack(keys, np.array(rows, dtype=np.int64).reshape(-1, 7), parts)
        one = torch.ones(1, dtype=torch.float32, device=dev)
        args, ws = [], []
        for k in range(parts):
            lo, hi = bounds[k], bounds[k + 1]
            if k == 0:
                first, cnt, wk = hp, hi, w[:hi]
            else:
                first, cnt = hp + (lo + k - 1) * row, hi - lo + 1
                wk = torch.cat([one, w[lo:hi]])
            ws.append(wk)
            if k < parts - 1:  # an fp32 partial into row hi + k
                args.append((first, g.stride, cnt, na.MODE_W32_DIV32, wk.data_ptr(), 1.0, 0, g.stride, None,
                             hp + (hi + k) * row, None))
            else:
                args.append((first, g.stride, cnt, nm.mode, wk.data_ptr(), float(nm.denom), 0, g.stride, None,
                             None if f64 else dout.data_ptr(), dout.data_ptr() if f64 else None))
        return ("chain", ap, args, ws)

    def _small_round(self, plan: BucketPlan, w_local_lst):
        """One small host round with no per-key Python: the uploads are packed natively into the
        record's pinned staging (every value checked against the plan: C-contiguous, dtype, byte
        size), each bucket is one reduce launch reading that staging and writing a pinned result
        over PCIe (zero-copy; with small_zero_copy False: one H2D, the launch and one D2H) on
        torch's current stream, one synchronisation, and the result is handed out as views of one fresh array per bucket
        (numpy scalars for 0-d keys) — what Packer.unpack returns.  Returns None (nothing queued)
        when a value does not fit the record; the caller then takes the general path."""
        rec = self._small_record(plan, w_local_lst)
        if rec is None:
            return None
        kinds, pack, wsig = rec
        lst = w_local_lst if type(w_local_lst) is list else list(w_local_lst)
        if wsig is not None:
            from .wire import wire_row

            if wire_row(lst[0], wsig) is not None:  # decoded by the wire codec into pinned rows of
                return None                          # this layout: the general path DMAs them as is
        n = len(lst)
        for nat, *rest in kinds:  # every bucket packed here, except a chained one (native threads)
            if rest[-1] is None and pack(lst, nat.keys, len(nat.keys), nat.ptr, 0, n) != 0:
                return None
        handles = {}
        try:
            for i, (nat, *rest) in enumerate(kinds):
                if rest[-1] is not None:
                    h = rest[-1][1].start(lst)
                    if h is None:  # a value off the plan: nothing was copied, nothing launched
                        return None
                    handles[i] = h
            dev = self.device
            if dev.index is not None and dev.index != torch.cuda.current_device():
                with torch.cuda.device(dev):  # launches go to dev's stream from dev's context
                    parts = self._small_launch(kinds, handles, dev)
            else:
                parts = self._small_launch(kinds, handles, dev)
        finally:
            for i, h in handles.items():  # every copy done (and the values released)
                kinds[i][-1][1].end(h)
        return {k: parts[k] for k in plan.keys}

    def _small_launch(self, kinds, handles, dev):
        """The queued part of _small_round: launches (and copies) on dev's current stream — a
        chained bucket's launches each right after its part's copies are in — one
        synchronisation, the results as {key: value}."""
        stream = torch.cuda.current_stream(dev)
        sh = stream.cuda_stream
        try:
            self._small_enqueue(kinds, handles, stream, sh)
        finally:
            stream.synchronize()  # also: the staging may be rewritten by the next call
        parts = {}
        for nat, host, stack, w, dout, hout, hnp, fn, args, out, split in kinds:
            fresh = hnp.copy()
            for k, off, m, shape in out:
                a = fresh[off : off + m].reshape(shape)
                parts[k] = a.dtype.type(a[()]) if shape == () else a
        return parts

    def _small_enqueue(self, kinds, handles, stream, sh):
        for i, (nat, host, stack, w, dout, hout, hnp, fn, args, out, split) in enumerate(kinds):
            if split is not None:  # chained zero-copy launches, each after its part is packed
                _, ap, chain, _ws = split
                for k, a in enumerate(chain):
                    ap.wait(handles[i], k)
                    na.check(fn(*a, sh), fn.__name__)
                continue
            if stack is host:  # zero-copy record
                na.check(fn(*args, sh), fn.__name__)
                continue
            stack.copy_(host[: stack.shape[0]], non_blocking=True)
            na.check(fn(*args, sh), fn.__name__)
            hout.copy_(dout, non_blocking=True)

    def _gather_columns(self, plan: BucketPlan, parts):
        """Column-sharded group: every rank's reduced columns -> the whole f32 bucket on every
        rank, one all_gather_into_tensor (RCCL over xGMI; equal padded widths).

        Plain mean in FA_MODE_W32_DIV64 with the reference's float64 output: the ranks reduced
        with W = 1, i.e. they hold the exact fp32 sums acc (fl32(fl64(acc)/1) = acc), so the
        gather moves P*4 bytes instead of P*8, and one 1-client reduce of the gathered sums
        (weight fl32(1.0), W = np.sum(weights)) then computes fl64(acc)/W — the value the
        unsharded kernel's epilogue computes, bit for bit."""
        from .bucket import Shard, rank_width
        from .dist import gather_columns

        (sh, out), = parts
        stride = plan.groups[KIND_F32].stride
        full = gather_columns(out[: sh.width], rank_width(stride, self.packer.rank_cols[1]), stride, self.group)
        if self._post_denom is not None:
            out64 = self.packer.device_bucket(("out64_full", KIND_F32), (stride,), torch.float64, self.device)
            one = self._weights(_ONE_W32, self.device)
            reduce_stack(full.view(1, stride), one, na.MODE_W32_DIV64, self._post_denom, out64=out64)
            full = out64
        return [(Shard(0, self.device, 0, stride), full)]

    def _reduce_f32(self, g, sh, stack, w, server_opt, fused, first_means):
        nm = g.numerics
        want64 = self.output == "reference" and nm.out_dtype == _F64
        # column-sharded plain mean with float64 output: gather fp32 sums, divide after
        sums = self._dist and want64 and server_opt is None and nm.mode == na.MODE_W32_DIV64
        if sums:
            self._post_denom = float(nm.denom)
        if sh.width == 0:  # a rank whose column range is empty (tiny model, many ranks)
            if isinstance(server_opt, ServerOptimizer) and not fused:
                first_means[sh.index] = torch.empty(0, dtype=torch.float32, device=sh.device)
            gathers64 = want64 and not sums
            return torch.empty(0, dtype=torch.float64 if gathers64 else torch.float32, device=sh.device)
        if sums:
            out32 = self.packer.device_bucket(("sum32", KIND_F32, sh.index), (sh.width,), torch.float32, sh.device)
            reduce_stack(stack, w, nm.mode, 1.0, out32=out32, reorder=self.reorder and not isinstance(stack, RowTable))
            return out32
        out64 = (self.packer.device_bucket(("out64", KIND_F32, sh.index), (sh.width,), torch.float64, sh.device)
                 if want64 else None)
        if isinstance(server_opt, DynState):
            return server_opt.step(self, sh, stack, w, nm, want64)
        if server_opt is not None and fused:
            # fused: fl32(w) becomes the next round's prev (the model clients load), v_t advances;
            # both into the spare pair, which then becomes the state (double-buffered)
            prev, v, prev_o, v_o = server_opt.swap_buffers(sh)
            try:
                reduce_stack(stack, w, nm.mode, nm.denom, out32=prev_o, out64=out64, op=server_opt.op, prev=prev,
                             v=v, v_out=v_o, beta=server_opt.beta, eta=server_opt.eta, tau=server_opt.tau,
                             beta2=server_opt.beta2, reorder=self.reorder and not isinstance(stack, RowTable))
            except BaseException:
                server_opt.unswap(sh)  # a refused launch must not leave the state on the empty spare pair
                raise
            return out64 if want64 else prev_o
        out32 = None
        if not want64 or server_opt is not None:
            out32 = self.packer.device_bucket(("out32", KIND_F32, sh.index), (sh.width,), torch.float32, sh.device)
        reduce_stack(stack, w, nm.mode, nm.denom, out32=out32, out64=out64,
                     reorder=self.reorder and not isinstance(stack, RowTable))
        if server_opt is not None:
            first_means[sh.index] = out32
        return out64 if want64 else out32

    def _finish(self, plan: BucketPlan, results: dict):
        if self.output == "device":
            return assemble_on_device(plan, results, self.device)
        return self.packer.unpack(plan, results, as_torch=plan.input_kind == "torch")


def assemble_on_device(plan: BucketPlan, results: dict, device) -> dict:
    """output="device": the global model as fresh tensors on `device`.  Per bucket kind ONE fresh
    buffer of the bucket's stride is filled with one copy per column shard (a peer copy over
    xGMI for shards on other GPUs; a plain device copy for the local one), and every key is a
    view of it — not one slice copy per (key, shard).  results: kind -> [(shard, tensor)]."""
    device = torch.device(device)
    full = {}
    for kind, parts in results.items():
        dt = parts[0][1].dtype
        buf = torch.empty(plan.groups[kind].stride, dtype=dt, device=device)
        for sh, t in parts:
            buf[sh.c0 : sh.c1].copy_(t[: sh.width], non_blocking=True)
        full[kind] = buf
    glob = {}
    for k in plan.keys:
        s = plan.key_segment[k]
        glob[k] = full[plan.key_group[k]][s.offset : s.offset + s.numel].view(s.shape)
    return glob
