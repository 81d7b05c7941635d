"""Tensor-level wrappers around the C ABI.  All tensors are CUDA (HIP) fp32, contiguous.
Activations are NDHWC tensors of shape [N, D, H, W, C].  Every call runs on the current
torch stream; no call allocates inside the library (workspaces come from `Workspace`)."""
from __future__ import annotations

import ctypes as _ct
import os
from typing import Optional, Sequence

import torch

from ._lib import call, query

ACT = {None: 0, "none": 0, "relu": 1, "lrelu": 2, "tanh": 3, "sigmoid": 4}


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _check_weights(wp: Optional[torch.Tensor], wsplit: Optional[torch.Tensor], n: int, what: str):
    """The packed weight (n fp32 elements) and / or its pre-split copy (n·4 bytes).  wp may be None
    when wsplit is given (ABI 19): the caller's fp32 pack is stale (only the pre-split copy is
    refreshed for a ResnetBlock conv in the one-plane modes), and the library then refuses any
    kernel that would read the fp32 pack instead of reading stale weights."""
    if wp is None and wsplit is None:
        raise ValueError(f"{what}: neither the packed weight nor its pre-split copy given")
    if wp is not None and wp.numel() != n:
        raise ValueError(f"{what}: packed weight has {wp.numel()} elements, expected {n}")
    if wsplit is not None and wsplit.numel() * wsplit.element_size() != n * 4:
        raise ValueError(f"{what}: wsplit size does not match the packed weight")


def _check(t: torch.Tensor, name: str, ndim: int = 5):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor (HIP); got {t.device}")
    if t.dtype != torch.float32:
        raise ValueError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    if ndim and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-d NDHWC tensor, got shape {tuple(t.shape)}")


_LANE = [0]


class lane:
    """`with ops.lane(i):` — calls inside use lane i's workspace.  Work issued concurrently on
    two streams must use two lanes (the model's G_A / G_B chains); the lane index, not the
    stream, keys the buffer, so an eager step and its graph capture use the same buffers."""

    def __init__(self, i: int):
        self.i = i

    def __enter__(self):
        self.prev = _LANE[0]
        _LANE[0] = self.i
        return self

    def __exit__(self, *exc):
        _LANE[0] = self.prev
        return False


class Workspace:
    """Grow-only scratch buffer per (device, lane) (sized by the first step; reused afterwards)."""

    def __init__(self):
        self._buf = {}
        self._retired = []      # outgrown buffers stay allocated: a captured HIP graph may hold them

    def get(self, nbytes: int) -> torch.Tensor:
        dev = (torch.cuda.current_device(), _LANE[0])
        b = self._buf.get(dev)
        if b is None or b.numel() < nbytes:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("workspace growth during HIP graph capture (run the step eagerly first)")
            if b is not None:
                self._retired.append(b)
            b = torch.empty(max(int(nbytes * 1.25), 1 << 20), dtype=torch.uint8, device=f"cuda:{dev[0]}")
            self._buf[dev] = b
        return b


WS = Workspace()


# A/B switch: MRAGAN_EAGER_CLASS_TIMING=1 times the launch classes by eager re-issue (rounds 1-6)
_EAGER_CLASS_TIMING = os.environ.get("MRAGAN_EAGER_CLASS_TIMING") is not None


class KernelTimer:
    """Per-launch-class timing of the instrumented C-ABI calls (bench.py's dominant-kernel
    roofline).  While `match` is set, each instrumented wrapper hands its call to `run(info, fn)`:
    the call is issued as usual and recorded — launch class `cls`, algorithmic `flops`
    (MFMA-bound) or `bytes` (HBM-bound), the kernels it launched (library launch log) and the
    call itself.  `classes(reps)` then re-issues ONE recorded call of each class `reps` times back
    to back on the current stream between two HIP events (one warm launch first), so a class's
    mean is the kernels' own duration and no spin kernel appears in a profile of the run.  Since
    round 6 the `reps` re-issues are captured once as a HIP graph and the graph is replayed between
    the events: eagerly, a host slower than ~25 µs per ctypes call (a busy box) left submission gaps
    inside the interval and inflated the short classes by up to 25 % (r06ac); a class whose call
    cannot be captured falls back to the eager re-issue (`timing` then says so)."""

    def __init__(self):
        self.match = None       # callable(info: dict) -> bool
        self.calls = []         # (info, kernel names, fn)

    def run(self, info, fn):
        if self.match is None or not self.match(info) or torch.cuda.is_current_stream_capturing():
            fn()
            return
        from ._lib import lib
        lib().mragan_launch_log(1)
        fn()
        self.calls.append((info, lib().mragan_launch_log(1).decode(), fn))

    def reset(self):
        self.calls = []

    def classes(self, reps: int = 10):
        """{cls: dict(n, total_ms, mean_ms, flops|bytes per launch, kernels)} for the recorded
        calls (n = launches recorded, total_ms = n × mean_ms), largest total time first."""
        out = {}
        for info, names, fn in self.calls:
            c = out.setdefault(info["cls"], dict(n=0, flops=info.get("flops"), bytes=info.get("bytes"), kernels=names,
                                                 info=info, fn=fn))
            c["n"] += 1
        for c in out.values():
            fn = c.pop("fn")
            fn()                                    # warm: first-touch of the operands, code load
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            graph = None
            if not _EAGER_CLASS_TIMING:
                try:
                    torch.cuda.synchronize()
                    graph = torch.cuda.CUDAGraph()
                    side = torch.cuda.Stream()
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
                        for _ in range(reps):
                            fn()
                    torch.cuda.current_stream().wait_stream(side)
                    graph.replay()                  # warm replay
                except Exception:                   # not capturable: the eager re-issue below
                    graph = None
                    torch.cuda.synchronize()
            s.record()
            if graph is not None:
                graph.replay()
            else:
                for _ in range(reps):
                    fn()
            e.record()
            e.synchronize()
            c["mean_ms"] = s.elapsed_time(e) / reps
            c["total_ms"] = c["mean_ms"] * c["n"]
            c["reps"] = reps
            c["graphed"] = graph is not None
            del graph
        self.calls = []
        return dict(sorted(out.items(), key=lambda kv: -kv[1]["total_ms"]))


TIMER = KernelTimer()


def _timed(info_fn, fn):
    """Issue fn(); when the timer records, under the launch class info_fn() describes."""
    if TIMER.match is None:
        fn()
    else:
        TIMER.run(info_fn(), fn)


PRECISION = {"f32": 0, "bf16x3": 1, "bf16": 2, "fp16": 3}


def set_conv_precision(mode: str) -> None:
    """Contraction precision of the MFMA convolutions: 'f32' exact, 'bf16x3' split (fp32-grade),
    'bf16' or 'fp16' (one MFMA per product, fp32 accumulation); see include/mragan_hip.h.
    Process-wide."""
    if mode not in PRECISION:
        raise ValueError(f"conv precision must be one of {sorted(PRECISION)}, got {mode!r}")
    call("mragan_set_conv_precision", PRECISION[mode])


def get_conv_precision() -> str:
    from ._lib import lib
    code = lib().mragan_get_conv_precision()
    return {v: k for k, v in PRECISION.items()}[code]


def set_loss_scale(scale: float) -> None:
    """Static loss scale applied to the gradients the loss kernels emit (fp16 mode); the
    optimizer's grad_scale must divide it out.  Process-wide."""
    call("mragan_set_loss_scale", float(scale))


def get_loss_scale() -> float:
    from ._lib import lib
    return float(lib().mragan_get_loss_scale())


def conv_out_size(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


def convT_out_size(n: int, k: int, s: int, p: int, op: int = 0) -> int:
    return (n - 1) * s - 2 * p + k + op


def conv3d(x: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int, out_spatial: Sequence[int],
           bias: Optional[torch.Tensor] = None, act=None, transposed: bool = False,
           out: Optional[torch.Tensor] = None, wsplit: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Forward-form (transposed=False) or transposed-form convolution; see include/mragan_hip.h.
    `wsplit`: the same packed weight pre-split by a tr 2/3 pack (mragan_conv3d_presplit)."""
    _check(x, "conv3d.x")
    N, Di, Hi, Wi, cin = x.shape
    Do, Ho, Wo = out_spatial
    _check_weights(wp, wsplit, k ** 3 * cin * cout, "conv3d")
    if out is None:
        out = torch.empty((N, Do, Ho, Wo, cout), device=x.device, dtype=torch.float32)
    elif tuple(out.shape) != (N, Do, Ho, Wo, cout):
        raise ValueError(f"conv3d: out shape {tuple(out.shape)} != {(N, Do, Ho, Wo, cout)}")
    name = "mragan_conv3d_transposed" if transposed else "mragan_conv3d_fwd"
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    if wsplit is not None:
        fn = lambda: call("mragan_conv3d_presplit", _ptr(x), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), _ptr(bias),
                          cout, k, s, p, ACT[act], _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _stream())
    else:
        fn = lambda: call(name, _ptr(x), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(bias), cout, k, s, p, ACT[act], _ptr(out),
                          Do, Ho, Wo, _ptr(ws), nbytes, _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out


def _conv_info(cin, cout, k, s, p, transposed, N, in_sp, out_sp):
    vox = in_sp[0] * in_sp[1] * in_sp[2] if transposed else out_sp[0] * out_sp[1] * out_sp[2]   # every tap of every voxel
    Di, Hi, Wi = in_sp
    return dict(op="conv", cin=cin, cout=cout, k=k, s=s, p=p, transposed=transposed, N=N, in_spatial=in_sp,
                out_spatial=out_sp, cls=f"{'convT' if transposed else 'conv'} {cin}->{cout} k{k} s{s} [{N}x{Di}x{Hi}x{Wi}]",
                flops=2.0 * N * vox * cin * cout * k ** 3)


# ---- ABI 15: in-launch InstanceNorm finalize ---------------------------------------------------
# One zeroed pool of uint32 ticket counters per device; each call takes the next N·cout/32 slots
# round-robin (the launch leaves them zero).  A graph capture holds ≪ 2^16 slots' worth of calls,
# so no two kernels that can run at the same time share a slot.  MRAGAN_NO_IN_TICKETS: off (A/B).
_TICKET_SLOTS = 1 << 16
_tickets = {}
_ticket_next = [0]
_NO_IN_TICKETS = __import__("os").environ.get("MRAGAN_NO_IN_TICKETS") is not None


def in_tickets_enabled() -> bool:
    return not _NO_IN_TICKETS


def ensure_ticket_pool(device) -> torch.Tensor:
    """The device's zeroed ticket pool, created on the device's default stream and synchronized
    before it is returned: every lane's first kernel that draws a ticket runs after the fill,
    whichever stream it is on (call before forking lanes; _ticket_ptr falls back to it)."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    pool = _tickets.get(dev)
    if pool is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("in-launch InstanceNorm finalize: the ticket pool must be allocated before a graph "
                               "capture (run one eager step first)")
        with torch.cuda.stream(torch.cuda.default_stream(dev)):
            pool = torch.zeros(_TICKET_SLOTS, device=dev, dtype=torch.int32)
        torch.cuda.synchronize(dev)
        _tickets[dev] = pool
    return pool


def _ticket_ptr(n: int, device) -> int:
    pool = ensure_ticket_pool(device)
    if n > _TICKET_SLOTS:
        raise ValueError(f"in-launch finalize: {n} ticket slots > the pool's {_TICKET_SLOTS}")
    if _ticket_next[0] + n > _TICKET_SLOTS:
        _ticket_next[0] = 0
    off = _ticket_next[0]
    _ticket_next[0] += n
    return pool.data_ptr() + 4 * off


def in_partials_buffer(N: int, out_spatial: Sequence[int], cout: int, device) -> torch.Tensor:
    """fp64 buffer for conv3d_in_stats' InstanceNorm statistics partials (the header's bound)."""
    Do, Ho, Wo = out_spatial
    return torch.empty(N * Do * (-(-Ho // 4)) * (-(-Wo // 6)) * cout * 2, device=device, dtype=torch.float64)



def conv3d_in_stats(x: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int, out_spatial: Sequence[int],
                    wsplit: Optional[torch.Tensor], part: torch.Tensor, transposed: bool = False):
    """conv3d (presplit weights if any, no bias / act) that also leaves the following
    InstanceNorm's statistics partials in `part` when the kernel that runs it produces them (the
    brick, ABI 9; the 16-bit implicit GEMM without a K split, ABI 11).  Returns (out, chunks);
    chunks = 0: no partials, run instnorm_fwd as usual."""
    _check(x, "conv3d.x")
    N, Di, Hi, Wi, cin = x.shape
    Do, Ho, Wo = out_spatial
    _check_weights(wp, wsplit, k ** 3 * cin * cout, "conv3d_in_stats")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("conv3d_in_stats: part must be a float64 device tensor")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_presplit_in_stats", _ptr(x), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), None,
                      cout, k, s, p, ACT[None], _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _ptr(part),
                      part.numel() * 8, _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out, chunks.value


def conv3d_wgrad(dense: torch.Tensor, gathered: torch.Tensor, k: int, s: int, p: int, dw: torch.Tensor,
                 accumulate: bool) -> torch.Tensor:
    _check(dense, "wgrad.dense")
    _check(gathered, "wgrad.gathered")
    N, Dd, Hd, Wd, Cd = dense.shape
    Ng, Dg, Hg, Wg, Cg = gathered.shape
    if Ng != N:
        raise ValueError("wgrad: batch mismatch")
    if dw.numel() != Cd * Cg * k ** 3 or not dw.is_contiguous():
        raise ValueError(f"wgrad: dw has {dw.numel()} elements, expected {Cd}x{Cg}x{k}^3 (contiguous)")
    nbytes = query("mragan_conv3d_wgrad_workspace", N, Dd, Hd, Wd, Cd, Cg, k, s)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_conv3d_wgrad", _ptr(dense), N, Dd, Hd, Wd, Cd, _ptr(gathered), Dg, Hg, Wg, Cg, k, s, p,
                      _ptr(dw), int(accumulate), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="wgrad", cls=f"wgrad {Cd}x{Cg} k{k} s{s} [{N}x{Dd}x{Hd}x{Wd}]",
                        flops=2.0 * N * Dd * Hd * Wd * Cd * Cg * k ** 3), fn)
    return dw


def pack_weight(src: torch.Tensor, A: int, B: int, T: int, transpose_ab: bool, out: torch.Tensor) -> torch.Tensor:
    call("mragan_pack_weight", _ptr(src), A, B, T, int(transpose_ab), _ptr(out), _stream())
    return out


class PackTable:
    """Device table of weight packs (src, dst, A, B, T, transpose) run by ONE launch
    (mragan_pack_weights).  Built once from stable pointers; `run` falls back to one launch per
    pack when the table is stale inside a graph capture (no host→device copy allowed there)."""

    def __init__(self):
        self.key = None
        self.dev = None
        self.n = 0
        self.max_elems = 0

    def run(self, packs):
        """packs: list of (src, A, B, T, transpose_ab, dst) tensors / ints."""
        import ctypes as C

        class _E(C.Structure):
            _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("A", C.c_int32), ("B", C.c_int32),
                        ("T", C.c_int32), ("tr", C.c_int32)]
        key = tuple((src.data_ptr(), dst.data_ptr(), A, B, T, int(tr)) for src, A, B, T, tr, dst in packs)
        if key != self.key:
            if torch.cuda.is_current_stream_capturing():
                for src, A, B, T, tr, dst in packs:
                    pack_weight(src, A, B, T, tr, dst)
                return
            if query("mragan_pack_entry_size") != C.sizeof(_E):
                raise RuntimeError("mragan_pack_entry_size mismatch")
            arr = (_E * len(packs))()
            for e, (sp, dp, A, B, T, tr) in zip(arr, key):
                e.src, e.dst, e.A, e.B, e.T, e.tr = sp, dp, A, B, T, tr
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self.dev = host.to(packs[0][0].device)
            self.key, self.n = key, len(packs)
            self.max_elems = max(A * B * T for _, _, A, B, T, _ in key)
        call("mragan_pack_weights", _ptr(self.dev), self.n, self.max_elems, _stream())


def instnorm_fwd(x: torch.Tensor, act=None, ypad: int = 0, resid: Optional[torch.Tensor] = None, rpad: int = 0,
                 out: Optional[torch.Tensor] = None, mean: Optional[torch.Tensor] = None,
                 rstd: Optional[torch.Tensor] = None, part: Optional[torch.Tensor] = None, chunks: int = 0):
    """InstanceNorm forward (+act, residual, replication pad of the output).  With `part` /
    `chunks` from conv3d_in_stats the statistics pass is skipped (ABI 9)."""
    _check(x, "instnorm.x")
    N, D, H, W, C = x.shape
    shp = (N, D + 2 * ypad, H + 2 * ypad, W + 2 * ypad, C)
    if out is None:
        out = torch.empty(shp, device=x.device, dtype=torch.float32)
    if mean is None:
        mean = torch.empty((N, C), device=x.device, dtype=torch.float32)
    if rstd is None:
        rstd = torch.empty((N, C), device=x.device, dtype=torch.float32)
    if resid is not None:
        _check(resid, "instnorm.resid")
        if tuple(resid.shape) != (N, D + 2 * rpad, H + 2 * rpad, W + 2 * rpad, C):
            raise ValueError("instnorm: residual shape mismatch")
    nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
    ws = WS.get(nbytes)
    if part is not None and chunks > 0:
        fn = lambda: call("mragan_instnorm_fwd_partials", _ptr(x), N, D, H, W, C, _ptr(out), ypad, ACT[act],
                          _ptr(resid), rpad, _ptr(mean), _ptr(rstd), _ptr(part), chunks, _stream())
    else:
        fn = lambda: call("mragan_instnorm_fwd", _ptr(x), N, D, H, W, C, _ptr(out), ypad, ACT[act], _ptr(resid), rpad,
                          _ptr(mean), _ptr(rstd), _ptr(ws), ws.numel(), _stream())
    # essential HBM bytes: read x (+ the residual), write y (padded)
    _timed(lambda: dict(op="in_fwd", cls=f"instnorm_fwd C{C} [{N}x{D}x{H}x{W}] pad{ypad}",
                        bytes=4.0 * (x.numel() * (2 if resid is not None else 1) + out.numel())), fn)
    return out, mean, rstd


def instnorm_bwd(x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, dy: torch.Tensor, dypad: int = 0,
                 dy_add: Optional[torch.Tensor] = None, act=None, out: Optional[torch.Tensor] = None,
                 g_out: Optional[torch.Tensor] = None):
    """dx of InstanceNorm(+act) from dy (replication-padded by dypad: folded) + dy_add.  With
    g_out, the folded gradient before act' is written there in the same pass (ABI 8)."""
    _check(x, "instnorm_bwd.x")
    N, D, H, W, C = x.shape
    if tuple(dy.shape) != (N, D + 2 * dypad, H + 2 * dypad, W + 2 * dypad, C):
        raise ValueError(f"instnorm_bwd: dy shape {tuple(dy.shape)} does not match pad {dypad}")
    if out is None:
        out = torch.empty_like(x)
    nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
    ws = WS.get(nbytes)
    if g_out is None:
        fn = lambda: call("mragan_instnorm_bwd", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy), dypad,
                          _ptr(dy_add), ACT[act], _ptr(out), _ptr(ws), ws.numel(), _stream())
    else:
        _check(g_out, "instnorm_bwd.g_out")
        if tuple(g_out.shape) != tuple(x.shape):
            raise ValueError("instnorm_bwd: g_out shape mismatch")
        fn = lambda: call("mragan_instnorm_bwd_g", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy), dypad,
                          _ptr(dy_add), ACT[act], _ptr(out), _ptr(g_out), _ptr(ws), ws.numel(), _stream())
    # essential HBM bytes: read x, dy (padded) (+ dy_add), write dx
    _timed(lambda: dict(op="in_bwd", cls=f"instnorm_bwd C{C} [{N}x{D}x{H}x{W}] pad{dypad}",
                        bytes=4.0 * (2 * x.numel() + dy.numel() + (x.numel() if dy_add is not None else 0)
                                     + (x.numel() if g_out is not None else 0))), fn)
    return out


# ---- 16-bit operand planes (bf16 / fp16 modes, ABI 11) ----------------------------------------
# The plane of an fp32 tensor holds the bf16 (fp16) words every MFMA convolution of the mode rounds
# it to, as a torch.bfloat16 (float16) tensor of the same shape; see include/mragan_hip.h.

def op16_dtype() -> Optional[torch.dtype]:
    """dtype of the operand planes in the current precision mode (None in the fp32-grade modes)."""
    return {"bf16": torch.bfloat16, "fp16": torch.float16}.get(get_conv_precision())


def _check16(t: torch.Tensor, name: str):
    dt = op16_dtype()
    if dt is None:
        raise ValueError(f"{name}: 16-bit operand planes need the bf16 or fp16 precision mode")
    if not t.is_cuda or t.dtype != dt or not t.is_contiguous() or t.dim() != 5:
        raise ValueError(f"{name}: expected a contiguous 5-d {dt} device tensor, got {t.dtype} {tuple(t.shape)}")


def instnorm_fwd_op16(x: torch.Tensor, act=None, ypad: int = 0, resid: Optional[torch.Tensor] = None, rpad: int = 0,
                      part: Optional[torch.Tensor] = None, chunks: int = 0, want_f32: bool = False, stats=None):
    """instnorm_fwd writing the output's operand plane (and the fp32 output too when want_f32).
    stats = (mean, rstd) finalized by the producing conv (ABI 15): the apply pass alone.
    Returns (out or None, out16, mean, rstd)."""
    if stats is not None:
        return _instnorm_apply_op16(x, act, ypad, resid, rpad, want_f32, stats)
    _check(x, "instnorm.x")
    dt = op16_dtype()
    if dt is None:
        raise ValueError("instnorm_fwd_op16: 16-bit operand planes need the bf16 or fp16 precision mode")
    N, D, H, W, C = x.shape
    shp = (N, D + 2 * ypad, H + 2 * ypad, W + 2 * ypad, C)
    out = torch.empty(shp, device=x.device, dtype=torch.float32) if want_f32 else None
    out16 = torch.empty(shp, device=x.device, dtype=dt)
    mean = torch.empty((N, C), device=x.device, dtype=torch.float32)
    rstd = torch.empty((N, C), device=x.device, dtype=torch.float32)
    if resid is not None:
        _check(resid, "instnorm.resid")
        if tuple(resid.shape) != (N, D + 2 * rpad, H + 2 * rpad, W + 2 * rpad, C):
            raise ValueError("instnorm: residual shape mismatch")
    if part is not None and chunks > 0:
        fn = lambda: call("mragan_instnorm_fwd_partials_op16", _ptr(x), N, D, H, W, C, _ptr(out), _ptr(out16), ypad,
                          ACT[act], _ptr(resid), rpad, _ptr(mean), _ptr(rstd), _ptr(part), chunks, _stream())
    else:
        nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
        ws = WS.get(nbytes)
        fn = lambda: call("mragan_instnorm_fwd_op16", _ptr(x), N, D, H, W, C, _ptr(out), _ptr(out16), ypad, ACT[act],
                          _ptr(resid), rpad, _ptr(mean), _ptr(rstd), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="in_fwd", cls=f"instnorm_fwd C{C} [{N}x{D}x{H}x{W}] pad{ypad} op16",
                        bytes=4.0 * x.numel() * (2 if resid is not None else 1) + out16.numel() * (6 if want_f32 else 2)),
           fn)
    return out, out16, mean, rstd


def instnorm_bwd_op16(x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, dy: torch.Tensor, dypad: int = 0,
                      dy_add: Optional[torch.Tensor] = None, act=None, g_out: Optional[torch.Tensor] = None):
    """instnorm_bwd writing dx only as its operand plane (returned); g_out as in instnorm_bwd."""
    _check(x, "instnorm_bwd.x")
    dt = op16_dtype()
    if dt is None:
        raise ValueError("instnorm_bwd_op16: 16-bit operand planes need the bf16 or fp16 precision mode")
    N, D, H, W, C = x.shape
    if tuple(dy.shape) != (N, D + 2 * dypad, H + 2 * dypad, W + 2 * dypad, C):
        raise ValueError(f"instnorm_bwd: dy shape {tuple(dy.shape)} does not match pad {dypad}")
    if g_out is not None:
        _check(g_out, "instnorm_bwd.g_out")
        if tuple(g_out.shape) != tuple(x.shape):
            raise ValueError("instnorm_bwd: g_out shape mismatch")
    dx16 = torch.empty(x.shape, device=x.device, dtype=dt)
    nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_instnorm_bwd_op16", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy), dypad,
                      _ptr(dy_add), ACT[act], _ptr(dx16), _ptr(g_out), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="in_bwd", cls=f"instnorm_bwd C{C} [{N}x{D}x{H}x{W}] pad{dypad} op16",
                        bytes=4.0 * (x.numel() + dy.numel() + (x.numel() if dy_add is not None else 0)
                                     + (x.numel() if g_out is not None else 0)) + 2.0 * x.numel()), fn)
    return dx16


def _instnorm_apply_op16(x, act, ypad, resid, rpad, want_f32, stats):
    _check(x, "instnorm.x")
    dt = op16_dtype()
    if dt is None:
        raise ValueError("instnorm_apply_op16: 16-bit operand planes need the bf16 or fp16 precision mode")
    mean, rstd = stats
    N, D, H, W, C = x.shape
    if tuple(mean.shape) != (N, C) or tuple(rstd.shape) != (N, C):
        raise ValueError("instnorm_apply_op16: statistics shape mismatch")
    shp = (N, D + 2 * ypad, H + 2 * ypad, W + 2 * ypad, C)
    out = torch.empty(shp, device=x.device, dtype=torch.float32) if want_f32 else None
    out16 = torch.empty(shp, device=x.device, dtype=dt)
    if resid is not None:
        _check(resid, "instnorm.resid")
        if tuple(resid.shape) != (N, D + 2 * rpad, H + 2 * rpad, W + 2 * rpad, C):
            raise ValueError("instnorm: residual shape mismatch")
    fn = lambda: call("mragan_instnorm_apply_op16", _ptr(x), N, D, H, W, C, _ptr(out), _ptr(out16), ypad, ACT[act],
                      _ptr(resid), rpad, _ptr(mean), _ptr(rstd), _stream())
    _timed(lambda: dict(op="in_fwd", cls=f"instnorm_fwd C{C} [{N}x{D}x{H}x{W}] pad{ypad} op16 fin",
                        bytes=4.0 * x.numel() * (2 if resid is not None else 1) + out16.numel() * (6 if want_f32 else 2)),
           fn)
    return out, out16, mean, rstd


_SPLIT_CACHE = {}


def dgrad_split(N: int, D: int, H: int, W: int, cin: int, cout: int) -> bool:
    """Does the whole-grid k3 s1 data gradient from the plane of dY [N, D, H, W, cin] (→ cout
    channels on the padded grid) run as interior brick + shell pass in the current mode?  The
    library's own rule (mragan_conv3d_dgrad_split, ABI 19), cached per shape and mode."""
    key = (N, D, H, W, cin, cout, get_conv_precision())
    v = _SPLIT_CACHE.get(key)
    if v is None:
        v = _SPLIT_CACHE[key] = bool(query("mragan_conv3d_dgrad_split", N, D, H, W, cin, cout))
    return v


def conv3d_op16(x16: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int, out_spatial: Sequence[int],
                wsplit: torch.Tensor, part: Optional[torch.Tensor] = None, transposed: bool = False, fin: bool = False):
    """conv3d (pre-split weights if any, no bias / act) on the operand plane x16 of its input (the
    k3 s1 brick kernel; the implicit GEMM for other forward-form convs, ABI 14); with `part` also the
    InstanceNorm statistics partials.  Returns (out, chunks); with fin (ABI 15) (out, chunks, stats):
    stats = (mean, rstd) when the launch finalized them (then instnorm_fwd_op16(stats=…)), else None."""
    if fin and part is not None:
        return _conv3d_op16_fin(x16, wp, cout, k, s, p, out_spatial, wsplit, part, transposed)
    _check16(x16, "conv3d_op16.x16")
    N, Di, Hi, Wi, cin = x16.shape
    Do, Ho, Wo = out_spatial
    _check_weights(wp, wsplit, k ** 3 * cin * cout, "conv3d_op16")
    if part is not None and (part.dtype != torch.float64 or not part.is_cuda):
        raise ValueError("conv3d_op16: part must be a float64 device tensor")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x16.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_op16", _ptr(x16), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), cout, k, s, p,
                      _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _ptr(part),
                      0 if part is None else part.numel() * 8, None if part is None else _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out, chunks.value


def _conv3d_op16_fin(x16, wp, cout, k, s, p, out_spatial, wsplit, part, transposed):
    _check16(x16, "conv3d_op16.x16")
    N, Di, Hi, Wi, cin = x16.shape
    Do, Ho, Wo = out_spatial
    _check_weights(wp, wsplit, k ** 3 * cin * cout, "conv3d_op16")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("conv3d_op16: part must be a float64 device tensor")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x16.device, dtype=torch.float32)
    mean = torch.empty((N, cout), device=x16.device, dtype=torch.float32)
    rstd = torch.empty((N, cout), device=x16.device, dtype=torch.float32)
    tick = _ticket_ptr(N * max(1, cout // 32), x16.device)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    chunks, done = _ct.c_int(0), _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_op16_fin", _ptr(x16), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), cout, k, s, p,
                      _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _ptr(part), part.numel() * 8,
                      _ct.byref(chunks), tick, _ptr(mean), _ptr(rstd), _ct.byref(done), _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out, chunks.value, ((mean, rstd) if done.value else None)


def conv3d_op16_dgrad_in_stats(dy16: torch.Tensor, wp: torch.Tensor, cout: int, wsplit: torch.Tensor,
                               x_in: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, act, part: torch.Tensor,
                               fin: bool = False, x_add: Optional[torch.Tensor] = None):
    """Whole-grid data gradient (k3 s1 p0 transposed form, output = input + 2 per dim) from the
    plane dy16 that also leaves, in `part`, the backward-statistics partials of the InstanceNorm
    (+act) whose output was this conv's input: x_in (pre-norm, [N, D, H, W, cout]), mean, rstd.
    Returns (dz, chunks); chunks = 0: no partials (run instnorm_bwd_op16).  With fin (ABI 15):
    (dz, chunks, coef) — coef [N, cout, 2] when the launch finalized the IN backward's coefficients
    (then instnorm_bwd_partials_op16(coef=…)), else None.  x_add (ABI 18, same shape as x_in): a
    gradient that joins the fold before act' — the statistics are then those of fold(dz) + x_add
    (instnorm_bwd_partials_op16 with dy_add=x_add); chunks = 0 where no brick epilogue runs."""
    _check16(dy16, "dgrad_in_stats.dy16")
    _check(x_in, "dgrad_in_stats.x_in")
    N, Di, Hi, Wi, cin = dy16.shape
    if tuple(x_in.shape) != (N, Di, Hi, Wi, cout):
        raise ValueError(f"dgrad_in_stats: x_in shape {tuple(x_in.shape)} != {(N, Di, Hi, Wi, cout)}")
    if x_add is not None:
        _check(x_add, "dgrad_in_stats.x_add")
        if tuple(x_add.shape) != tuple(x_in.shape):
            raise ValueError(f"dgrad_in_stats: x_add shape {tuple(x_add.shape)} != {tuple(x_in.shape)}")
    if wsplit is None:
        raise ValueError("dgrad_in_stats: the pre-split weight is required")
    _check_weights(wp, wsplit, 27 * cin * cout, "dgrad_in_stats")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("dgrad_in_stats: part must be a float64 device tensor")
    osp = (Di + 2, Hi + 2, Wi + 2)
    out = torch.empty((N,) + osp + (cout,), device=dy16.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, 3, 1, 0, *osp, 1)
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    if x_add is not None:
        coef = torch.empty((N, cout, 2), device=dy16.device, dtype=torch.float32) if fin else None
        tick = _ticket_ptr(N * max(1, cout // 32), dy16.device) if fin else None
        done = _ct.c_int(0)
        fn = lambda: call("mragan_conv3d_op16_dgrad_in_stats_add", _ptr(dy16), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit),
                          cout, _ptr(out), _ptr(ws), nbytes, _ptr(x_in), _ptr(mean), _ptr(rstd), ACT[act], _ptr(x_add),
                          _ptr(part), part.numel() * 8, _ct.byref(chunks), tick, _ptr(coef),
                          _ct.byref(done) if fin else None, _stream())
        _timed(lambda: _conv_info(cin, cout, 3, 1, 0, True, N, (Di, Hi, Wi), osp), fn)
        if fin:
            return out, chunks.value, (coef if done.value else None)
        return out, chunks.value
    if fin:
        coef = torch.empty((N, cout, 2), device=dy16.device, dtype=torch.float32)
        tick = _ticket_ptr(N * max(1, cout // 32), dy16.device)
        done = _ct.c_int(0)
        fn = lambda: call("mragan_conv3d_op16_dgrad_in_stats_fin", _ptr(dy16), N, Di, Hi, Wi, cin, _ptr(wp),
                          _ptr(wsplit), cout, _ptr(out), _ptr(ws), nbytes, _ptr(x_in), _ptr(mean), _ptr(rstd), ACT[act],
                          _ptr(part), part.numel() * 8, _ct.byref(chunks), tick, _ptr(coef), _ct.byref(done), _stream())
        _timed(lambda: _conv_info(cin, cout, 3, 1, 0, True, N, (Di, Hi, Wi), osp), fn)
        return out, chunks.value, (coef if done.value else None)
    fn = lambda: call("mragan_conv3d_op16_dgrad_in_stats", _ptr(dy16), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), cout,
                      _ptr(out), _ptr(ws), nbytes, _ptr(x_in), _ptr(mean), _ptr(rstd), ACT[act], _ptr(part),
                      part.numel() * 8, _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, 3, 1, 0, True, N, (Di, Hi, Wi), osp), fn)
    return out, chunks.value


def instnorm_bwd_partials_op16(x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, dy: torch.Tensor, dypad: int,
                               dy_add: Optional[torch.Tensor], act, part: torch.Tensor, chunks: int,
                               g_out: Optional[torch.Tensor] = None, coef: Optional[torch.Tensor] = None):
    """instnorm_bwd_op16 from backward-statistics partials (conv3d_op16_dgrad_in_stats): no
    statistics pass; with coef (ABI 15, finalized in that launch) the apply pass alone.  Returns
    the dx plane."""
    if coef is not None:
        return _instnorm_bwd_apply_op16(x, mean, rstd, dy, dypad, dy_add, act, g_out, coef)
    _check(x, "instnorm_bwd.x")
    dt = op16_dtype()
    if dt is None:
        raise ValueError("instnorm_bwd_partials_op16: 16-bit operand planes need the bf16 or fp16 precision mode")
    N, D, H, W, C = x.shape
    if tuple(dy.shape) != (N, D + 2 * dypad, H + 2 * dypad, W + 2 * dypad, C):
        raise ValueError(f"instnorm_bwd: dy shape {tuple(dy.shape)} does not match pad {dypad}")
    dx16 = torch.empty(x.shape, device=x.device, dtype=dt)
    nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_instnorm_bwd_partials_op16", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy),
                      dypad, _ptr(dy_add), ACT[act], _ptr(dx16), _ptr(g_out), _ptr(part), chunks, _ptr(ws), ws.numel(),
                      _stream())
    _timed(lambda: dict(op="in_bwd", cls=f"instnorm_bwd C{C} [{N}x{D}x{H}x{W}] pad{dypad} op16 partials",
                        bytes=4.0 * (x.numel() + dy.numel() + (x.numel() if dy_add is not None else 0)
                                     + (x.numel() if g_out is not None else 0)) + 2.0 * x.numel()), fn)
    return dx16


def _instnorm_bwd_apply_op16(x, mean, rstd, dy, dypad, dy_add, act, g_out, coef):
    _check(x, "instnorm_bwd.x")
    dt = op16_dtype()
    if dt is None:
        raise ValueError("instnorm_bwd_apply_op16: 16-bit operand planes need the bf16 or fp16 precision mode")
    N, D, H, W, C = x.shape
    if tuple(dy.shape) != (N, D + 2 * dypad, H + 2 * dypad, W + 2 * dypad, C):
        raise ValueError(f"instnorm_bwd: dy shape {tuple(dy.shape)} does not match pad {dypad}")
    if tuple(coef.shape) != (N, C, 2) or coef.dtype != torch.float32:
        raise ValueError("instnorm_bwd_apply_op16: coef must be float32 [N, C, 2]")
    dx16 = torch.empty(x.shape, device=x.device, dtype=dt)
    fn = lambda: call("mragan_instnorm_bwd_apply_op16", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy), dypad,
                      _ptr(dy_add), ACT[act], _ptr(dx16), _ptr(g_out), _ptr(coef), _stream())
    _timed(lambda: dict(op="in_bwd", cls=f"instnorm_bwd C{C} [{N}x{D}x{H}x{W}] pad{dypad} op16 fin",
                        bytes=4.0 * (x.numel() + dy.numel() + (x.numel() if dy_add is not None else 0)
                                     + (x.numel() if g_out is not None else 0)) + 2.0 * x.numel()), fn)
    return dx16


def conv3d_dgrad_in_stats(dy: torch.Tensor, wp: torch.Tensor, cout: int, k: int, x_in: torch.Tensor,
                          mean: torch.Tensor, rstd: torch.Tensor, act, fold_pad: int, part: torch.Tensor):
    """Data gradient (transposed form, stride 1, pad 0: output = input + k − 1 per dim) of a valid
    conv whose input was ReplicationPad(fold_pad)(act(IN(x_in))), that also leaves that IN's
    backward-statistics partials when its kernel has the epilogue (ABI 12: thin1_x3, the G head).
    Returns (dz, chunks); chunks = 0: no partials (run instnorm_bwd)."""
    _check(dy, "dgrad_in_stats.dy")
    _check(x_in, "dgrad_in_stats.x_in")
    N, Di, Hi, Wi, cin = dy.shape
    osp = (Di + k - 1, Hi + k - 1, Wi + k - 1)
    if tuple(x_in.shape) != (N,) + tuple(o - 2 * fold_pad for o in osp) + (cout,):
        raise ValueError(f"dgrad_in_stats: x_in shape {tuple(x_in.shape)} does not match fold {fold_pad}")
    if wp.numel() != k ** 3 * cin * cout:
        raise ValueError("dgrad_in_stats: packed weight size mismatch")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("dgrad_in_stats: part must be a float64 device tensor")
    out = torch.empty((N,) + osp + (cout,), device=dy.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, 1, 0, *osp, 1)
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_dgrad_in_stats", _ptr(dy), N, Di, Hi, Wi, cin, _ptr(wp), cout, k, _ptr(out),
                      _ptr(ws), nbytes, _ptr(x_in), _ptr(mean), _ptr(rstd), ACT[act], fold_pad, _ptr(part),
                      part.numel() * 8, _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, k, 1, 0, True, N, (Di, Hi, Wi), osp), fn)
    return out, chunks.value


def conv3d_bwd_stats(x: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int, out_spatial: Sequence[int],
                     wsplit: Optional[torch.Tensor], x_in: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, act,
                     part: torch.Tensor, transposed: bool = False):
    """conv3d (presplit weights, no bias / act) whose output is the data gradient of the
    InstanceNorm(+act) of x_in (same shape): also leaves that norm's backward-statistics partials
    when its kernel has the epilogue (ABI 12: the stride-2 implicit GEMM).  Returns (out, chunks);
    chunks = 0: no partials (run instnorm_bwd)."""
    _check(x, "conv3d.x")
    _check(x_in, "bwd_stats.x_in")
    N, Di, Hi, Wi, cin = x.shape
    Do, Ho, Wo = out_spatial
    if tuple(x_in.shape) != (N, Do, Ho, Wo, cout):
        raise ValueError(f"bwd_stats: x_in shape {tuple(x_in.shape)} != {(N, Do, Ho, Wo, cout)}")
    if wp.numel() != k ** 3 * cin * cout:
        raise ValueError("bwd_stats: packed weight size mismatch")
    if wsplit is not None and wsplit.numel() * wsplit.element_size() != wp.numel() * 4:
        raise ValueError("bwd_stats: wsplit size does not match the packed weight")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("bwd_stats: part must be a float64 device tensor")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_presplit_bwd_stats", _ptr(x), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(wsplit), cout, k,
                      s, p, _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _ptr(x_in), _ptr(mean),
                      _ptr(rstd), ACT[act], _ptr(part), part.numel() * 8, _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out, chunks.value


def conv3d_op16_bwd_stats(x16: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int,
                          out_spatial: Sequence[int], x_in: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, act,
                          part: torch.Tensor, transposed: bool = False):
    """conv3d_bwd_stats on the operand plane x16 of its input (ABI 16).  Returns (out, chunks)."""
    _check16(x16, "conv3d_op16_bwd_stats.x16")
    _check(x_in, "bwd_stats.x_in")
    N, Di, Hi, Wi, cin = x16.shape
    Do, Ho, Wo = out_spatial
    if tuple(x_in.shape) != (N, Do, Ho, Wo, cout):
        raise ValueError(f"bwd_stats: x_in shape {tuple(x_in.shape)} != {(N, Do, Ho, Wo, cout)}")
    if wp.numel() != k ** 3 * cin * cout:
        raise ValueError("bwd_stats: packed weight size mismatch")
    if part.dtype != torch.float64 or not part.is_cuda:
        raise ValueError("bwd_stats: part must be a float64 device tensor")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x16.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    chunks = _ct.c_int(0)
    fn = lambda: call("mragan_conv3d_op16_bwd_stats", _ptr(x16), N, Di, Hi, Wi, cin, _ptr(wp), cout, k, s, p, _ptr(out),
                      Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _ptr(x_in), _ptr(mean), _ptr(rstd), ACT[act],
                      _ptr(part), part.numel() * 8, _ct.byref(chunks), _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out, chunks.value


def instnorm_bwd_partials(x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, dy: torch.Tensor, dypad: int,
                          dy_add: Optional[torch.Tensor], act, part: torch.Tensor, chunks: int,
                          g_out: Optional[torch.Tensor] = None):
    """instnorm_bwd (fp32 dx) from backward-statistics partials (conv3d_dgrad_in_stats)."""
    _check(x, "instnorm_bwd.x")
    N, D, H, W, C = x.shape
    if tuple(dy.shape) != (N, D + 2 * dypad, H + 2 * dypad, W + 2 * dypad, C):
        raise ValueError(f"instnorm_bwd: dy shape {tuple(dy.shape)} does not match pad {dypad}")
    dx = torch.empty(x.shape, device=x.device, dtype=torch.float32)
    nbytes = query("mragan_instnorm_workspace", N, D, H, W, C)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_instnorm_bwd_partials", _ptr(x), _ptr(mean), _ptr(rstd), N, D, H, W, C, _ptr(dy),
                      dypad, _ptr(dy_add), ACT[act], _ptr(dx), _ptr(g_out), _ptr(part), chunks, _ptr(ws), ws.numel(),
                      _stream())
    _timed(lambda: dict(op="in_bwd", cls=f"instnorm_bwd C{C} [{N}x{D}x{H}x{W}] pad{dypad} partials",
                        bytes=4.0 * (2 * x.numel() + dy.numel() + (x.numel() if dy_add is not None else 0)
                                     + (x.numel() if g_out is not None else 0))), fn)
    return dx


def conv3d_wgrad_op16(dense16: torch.Tensor, gathered16: torch.Tensor, k: int, s: int, p: int, dw: torch.Tensor,
                      accumulate: bool) -> torch.Tensor:
    """conv3d_wgrad on the operand planes of dense and gathered (the k3 s1 valid weight gradient)."""
    _check16(dense16, "wgrad_op16.dense")
    _check16(gathered16, "wgrad_op16.gathered")
    N, Dd, Hd, Wd, Cd = dense16.shape
    Ng, Dg, Hg, Wg, Cg = gathered16.shape
    if Ng != N:
        raise ValueError("wgrad: batch mismatch")
    if dw.numel() != Cd * Cg * k ** 3 or not dw.is_contiguous():
        raise ValueError(f"wgrad: dw has {dw.numel()} elements, expected {Cd}x{Cg}x{k}^3 (contiguous)")
    nbytes = query("mragan_conv3d_wgrad_workspace", N, Dd, Hd, Wd, Cd, Cg, k, s)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_conv3d_wgrad_op16", _ptr(dense16), N, Dd, Hd, Wd, Cd, _ptr(gathered16), Dg, Hg, Wg, Cg,
                      k, s, p, _ptr(dw), int(accumulate), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="wgrad", cls=f"wgrad {Cd}x{Cg} k{k} s{s} [{N}x{Dd}x{Hd}x{Wd}]",
                        flops=2.0 * N * Dd * Hd * Wd * Cd * Cg * k ** 3), fn)
    return dw


def conv3d_wgrad_op16_pair(dense16: torch.Tensor, gathered16: torch.Tensor, dense16_b: torch.Tensor,
                           gathered16_b: torch.Tensor, k: int, s: int, p: int, dw: torch.Tensor,
                           accumulate: bool) -> torch.Tensor:
    """conv3d_wgrad_op16 summed over two instance sets of one per-instance shape (ABI 19): a
    generator's first-pass and cycle-pass operands of one ResnetBlock conv in one launch."""
    for t, n in ((dense16, "dense"), (gathered16, "gathered"), (dense16_b, "dense_b"), (gathered16_b, "gathered_b")):
        _check16(t, f"wgrad_op16_pair.{n}")
    N, Dd, Hd, Wd, Cd = dense16.shape
    Nb = dense16_b.shape[0]
    _, Dg, Hg, Wg, Cg = gathered16.shape
    if gathered16.shape[0] != N or gathered16_b.shape[0] != Nb:
        raise ValueError("wgrad_pair: batch mismatch")
    if tuple(dense16_b.shape[1:]) != (Dd, Hd, Wd, Cd) or tuple(gathered16_b.shape[1:]) != (Dg, Hg, Wg, Cg):
        raise ValueError("wgrad_pair: the two instance sets differ in shape")
    if dw.numel() != Cd * Cg * k ** 3 or not dw.is_contiguous():
        raise ValueError(f"wgrad: dw has {dw.numel()} elements, expected {Cd}x{Cg}x{k}^3 (contiguous)")
    nbytes = query("mragan_conv3d_wgrad_workspace", N + Nb, Dd, Hd, Wd, Cd, Cg, k, s)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_conv3d_wgrad_op16_pair", _ptr(dense16), N, _ptr(gathered16), _ptr(dense16_b), Nb,
                      _ptr(gathered16_b), Dd, Hd, Wd, Cd, Dg, Hg, Wg, Cg, k, s, p, _ptr(dw), int(accumulate), _ptr(ws),
                      ws.numel(), _stream())
    _timed(lambda: dict(op="wgrad", cls=f"wgrad {Cd}x{Cg} k{k} s{s} [{N}+{Nb}x{Dd}x{Hd}x{Wd}]",
                        flops=2.0 * (N + Nb) * Dd * Hd * Wd * Cd * Cg * k ** 3), fn)
    return dw


def conv3d_wgrad_g16(dense: torch.Tensor, gathered16: torch.Tensor, k: int, s: int, p: int, dw: torch.Tensor,
                     accumulate: bool) -> torch.Tensor:
    """conv3d_wgrad (k3 s2 p1) with the gathered operand as its 16-bit plane, dense fp32 (ABI 14)."""
    _check(dense, "wgrad_g16.dense")
    _check16(gathered16, "wgrad_g16.gathered")
    N, Dd, Hd, Wd, Cd = dense.shape
    Ng, Dg, Hg, Wg, Cg = gathered16.shape
    if Ng != N:
        raise ValueError("wgrad: batch mismatch")
    if dw.numel() != Cd * Cg * k ** 3 or not dw.is_contiguous():
        raise ValueError(f"wgrad: dw has {dw.numel()} elements, expected {Cd}x{Cg}x{k}^3 (contiguous)")
    nbytes = query("mragan_conv3d_wgrad_workspace", N, Dd, Hd, Wd, Cd, Cg, k, s)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_conv3d_wgrad_g16", _ptr(dense), N, Dd, Hd, Wd, Cd, _ptr(gathered16), Dg, Hg, Wg, Cg,
                      k, s, p, _ptr(dw), int(accumulate), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="wgrad", cls=f"wgrad {Cd}x{Cg} k{k} s{s} [{N}x{Dd}x{Hd}x{Wd}]",
                        flops=2.0 * N * Dd * Hd * Wd * Cd * Cg * k ** 3), fn)
    return dw


def conv3d_thin_op16(x16: torch.Tensor, wp: torch.Tensor, cout: int, k: int, s: int, p: int, out_spatial: Sequence[int],
                     bias: Optional[torch.Tensor] = None, act=None, transposed: bool = False) -> torch.Tensor:
    """conv3d of the 32 → nc k7 layers (G head forward, G stem data gradient) from the operand
    plane of their 32-channel input (ABI 17): bit-identical to conv3d on the fp32 tensor."""
    _check16(x16, "conv3d_thin_op16.x16")
    N, Di, Hi, Wi, cin = x16.shape
    Do, Ho, Wo = out_spatial
    if wp.numel() != k ** 3 * cin * cout:
        raise ValueError(f"conv3d_thin_op16: packed weight has {wp.numel()} elements, expected {k**3}x{cout}x{cin}")
    out = torch.empty((N, Do, Ho, Wo, cout), device=x16.device, dtype=torch.float32)
    nbytes = query("mragan_conv3d_workspace", N, Di, Hi, Wi, cin, cout, k, s, p, Do, Ho, Wo, int(transposed))
    ws = WS.get(nbytes) if nbytes else None
    fn = lambda: call("mragan_conv3d_thin_op16", _ptr(x16), N, Di, Hi, Wi, cin, _ptr(wp), _ptr(bias), cout, k, s, p,
                      ACT[act], _ptr(out), Do, Ho, Wo, int(transposed), _ptr(ws), nbytes, _stream())
    _timed(lambda: _conv_info(cin, cout, k, s, p, transposed, N, (Di, Hi, Wi), (Do, Ho, Wo)), fn)
    return out


def conv3d_wgrad_thin_op16(dense, gathered, k: int, s: int, p: int, dw: torch.Tensor, accumulate: bool) -> torch.Tensor:
    """conv3d_wgrad of the k7 layers (nc ↔ 32 channels) with the 32-channel operand as its 16-bit
    plane and the nc-channel one fp32 (ABI 17)."""
    N, Dd, Hd, Wd, Cd = dense.shape
    Ng, Dg, Hg, Wg, Cg = gathered.shape
    if Ng != N:
        raise ValueError("wgrad: batch mismatch")
    wide, thin = (dense, gathered) if Cd >= Cg else (gathered, dense)
    _check16(wide, "wgrad_thin_op16.wide")
    _check(thin, "wgrad_thin_op16.thin")
    if dw.numel() != Cd * Cg * k ** 3 or not dw.is_contiguous():
        raise ValueError(f"wgrad: dw has {dw.numel()} elements, expected {Cd}x{Cg}x{k}^3 (contiguous)")
    nbytes = query("mragan_conv3d_wgrad_workspace", N, Dd, Hd, Wd, Cd, Cg, k, s)
    ws = WS.get(nbytes)
    fn = lambda: call("mragan_conv3d_wgrad_thin_op16", _ptr(dense), N, Dd, Hd, Wd, Cd, _ptr(gathered), Dg, Hg, Wg, Cg,
                      k, s, p, _ptr(dw), int(accumulate), _ptr(ws), ws.numel(), _stream())
    _timed(lambda: dict(op="wgrad", cls=f"wgrad {Cd}x{Cg} k{k} s{s} [{N}x{Dd}x{Hd}x{Wd}] op16",
                        flops=2.0 * N * Dd * Hd * Wd * Cd * Cg * k ** 3), fn)
    return dw


def rpad(x: torch.Tensor, p: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(x, "rpad.x")
    N, D, H, W, C = x.shape
    if out is None:
        out = torch.empty((N, D + 2 * p, H + 2 * p, W + 2 * p, C), device=x.device, dtype=torch.float32)
    call("mragan_rpad", _ptr(x), N, D, H, W, C, p, _ptr(out), _stream())
    return out


def rpad_fold(yp: torch.Tensor, p: int, add: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(yp, "rpad_fold.y")
    N, Dp, Hp, Wp, C = yp.shape
    D, H, W = Dp - 2 * p, Hp - 2 * p, Wp - 2 * p
    if out is None:
        out = torch.empty((N, D, H, W, C), device=yp.device, dtype=torch.float32)
    call("mragan_rpad_fold", _ptr(yp), N, D, H, W, C, p, _ptr(add), _ptr(out), _stream())
    return out


def act_bwd(y: Optional[torch.Tensor], grads: Sequence[Optional[torch.Tensor]], act, out: torch.Tensor) -> torch.Tensor:
    g = list(grads) + [None] * (3 - len(grads))
    call("mragan_act_bwd", _ptr(y), _ptr(g[0]), _ptr(g[1]), _ptr(g[2]), out.numel(), ACT[act], _ptr(out), _stream())
    return out


def channel_concat(a: torch.Tensor, act_a, b: torch.Tensor, act_b, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NDHWC channel concatenation [act_a(a) | act_b(b)] (UNet skip, networks3D.py:340-343)."""
    _check(a, "concat.a")
    _check(b, "concat.b")
    if a.shape[:4] != b.shape[:4]:
        raise ValueError(f"concat: spatial mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    Ca, Cb = a.shape[4], b.shape[4]
    if out is None:
        out = torch.empty(tuple(a.shape[:4]) + (Ca + Cb,), device=a.device, dtype=torch.float32)
    M = a.numel() // Ca
    call("mragan_channel_concat", _ptr(a), Ca, ACT[act_a], _ptr(b), Cb, ACT[act_b], M, _ptr(out), _stream())
    return out


def channel_split(g: torch.Tensor, Ca: int, ya: Optional[torch.Tensor], act_a, yb: Optional[torch.Tensor], act_b,
                  da: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None):
    """Backward of channel_concat: (g[..., :Ca]·act_a'(ya), g[..., Ca:]·act_b'(yb))."""
    _check(g, "split.g")
    Co = g.shape[4]
    Cb = Co - Ca
    sp = tuple(g.shape[:4])
    if da is None:
        da = torch.empty(sp + (Ca,), device=g.device, dtype=torch.float32)
    if db is None:
        db = torch.empty(sp + (Cb,), device=g.device, dtype=torch.float32)
    for t, c in ((ya, Ca), (yb, Cb)):
        if t is not None and tuple(t.shape) != sp + (c,):
            raise ValueError("split: activation shape mismatch")
    M = g.numel() // Co
    call("mragan_channel_split", _ptr(g), Ca, Cb, M, _ptr(ya), ACT[act_a], _ptr(da), _ptr(yb), ACT[act_b], _ptr(db),
         _stream())
    return da, db


def l1_loss(a: torch.Tensor, b: torch.Tensor, scale: float, loss_slot: torch.Tensor, grad: Optional[torch.Tensor],
            loss_accumulate=False, grad_accumulate=False):
    ws = WS.get(1 << 14)
    call("mragan_l1_loss", _ptr(a), _ptr(b), a.numel(), float(scale), _ptr(loss_slot), int(loss_accumulate), _ptr(grad),
         int(grad_accumulate), _ptr(ws), _stream())


def gan_loss(p: torch.Tensor, target: float, lsgan: bool, scale: float, loss_slot: torch.Tensor,
             dlogit: Optional[torch.Tensor], loss_accumulate=False):
    ws = WS.get(1 << 14)
    call("mragan_gan_loss", _ptr(p), p.numel(), float(target), int(lsgan), float(scale), _ptr(loss_slot),
         int(loss_accumulate), _ptr(dlogit), _ptr(ws), _stream())


def channel_sum(x: torch.Tensor, out: torch.Tensor, accumulate=False):
    C = x.shape[-1]
    M = x.numel() // C
    ws = WS.get(query("mragan_channel_sum_workspace", M, C))
    call("mragan_channel_sum", _ptr(x), M, C, _ptr(out), int(accumulate), _ptr(ws), ws.numel(), _stream())
    return out


def adam(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, lr: float, beta1: float, beta2: float,
         eps: float, step: int, grad_scale: float = 1.0):
    call("mragan_adam", _ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), float(lr), float(beta1), float(beta2), float(eps),
         int(step), float(grad_scale), _stream())


def adam_hyper(lr: float, beta1: float, beta2: float, eps: float, step: int, grad_scale: float = 1.0):
    """Host: the six per-step Adam scalars mragan_adam_dev reads (see include/mragan_hip.h)."""
    import ctypes as C
    out = (C.c_float * 6)()
    call("mragan_adam_hyper", float(lr), float(beta1), float(beta2), float(eps), int(step), float(grad_scale), out)
    return list(out)


def adam_dev(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, hyper: torch.Tensor):
    """Adam step whose scalars live in device memory (hyper: 6 fp32 values) — graph-replayable."""
    if hyper.dtype != torch.float32 or hyper.numel() < 6 or not hyper.is_cuda:
        raise ValueError("adam_dev: hyper must be a device float32 tensor of 6 values")
    call("mragan_adam_dev", _ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(hyper), _stream())


def adam_dev_checked(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, hyper: torch.Tensor,
                     flag: torch.Tensor):
    """adam_dev that leaves p, m, v untouched when the device int `flag` is non-zero."""
    if flag.dtype != torch.int32 or not flag.is_cuda:
        raise ValueError("adam_dev_checked: flag must be a device int32 tensor")
    call("mragan_adam_dev_checked", _ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), _ptr(hyper), _ptr(flag), _stream())


def adam_rebias(base: torch.Tensor, skipped: torch.Tensor, hyper: torch.Tensor):
    """hyper (device, 6 fp32) ← adam_hyper(lr, beta1, beta2, eps, step − skipped, grad_scale) from
    base = device {lr, beta1, beta2, eps, step, grad_scale} and the device skip counter."""
    if base.dtype != torch.float32 or base.numel() < 6 or hyper.dtype != torch.float32 or hyper.numel() < 6:
        raise ValueError("adam_rebias: base and hyper must be float32 tensors of 6 values")
    if skipped.dtype != torch.int32 or not (base.is_cuda and hyper.is_cuda and skipped.is_cuda):
        raise ValueError("adam_rebias: device tensors (skipped int32) expected")
    call("mragan_adam_rebias", _ptr(base), _ptr(skipped), _ptr(hyper), _stream())


def nonfinite_flag(g: torch.Tensor, flag: torch.Tensor):
    """flag |= 1 (device int32) when g holds an inf / NaN."""
    call("mragan_nonfinite_flag", _ptr(g), g.numel(), _ptr(flag), _stream())


def skip_count(flag: torch.Tensor, counter: torch.Tensor):
    """counter += (flag != 0); flag = 0 (both device int32)."""
    call("mragan_skip_count", _ptr(flag), _ptr(counter), _stream())


def fill(t: torch.Tensor, value: float):
    call("mragan_fill", _ptr(t), t.numel(), float(value), _stream())


def patch_gather(vol: torch.Tensor, starts: torch.Tensor, patch, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """vol [X, Y, Z] fp32 (device), starts int32 [n, 3] (device) → [n, px, py, pz, 1] NDHWC patches
    scaled (v − 127.5)/127.5 (test.py:150)."""
    _check(vol, "patch_gather.vol", ndim=3)
    if starts.dtype != torch.int32 or not starts.is_cuda or starts.dim() != 2 or starts.shape[1] != 3:
        raise ValueError("patch_gather: starts must be a device int32 [n, 3] tensor")
    n = starts.shape[0]
    px, py, pz = patch
    if out is None:
        out = torch.empty((n, px, py, pz, 1), device=vol.device, dtype=torch.float32)
    X, Y, Z = vol.shape
    call("mragan_patch_gather", _ptr(vol), X, Y, Z, _ptr(starts.contiguous()), n, px, py, pz, _ptr(out), _stream())
    return out


def patch_combine(pred: torch.Tensor, shape, patch, stride_inplane: int, stride_layer: int,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """pred: [n_patches, px, py, pz] (any trailing singleton) fp32 for the full patch grid in
    the reference's visit order → overlap-averaged label volume [X, Y, Z] (test.py:160-173)."""
    _check(pred, "patch_combine.pred", ndim=0)
    X, Y, Z = shape
    px, py, pz = patch
    if out is None:
        out = torch.empty((X, Y, Z), device=pred.device, dtype=torch.float32)
    call("mragan_patch_combine", _ptr(pred), X, Y, Z, px, py, pz, int(stride_inplane), int(stride_layer), _ptr(out),
         _stream())
    return out


def crop_patches(vol: torch.Tensor, starts: torch.Tensor, patch, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """vol [X, Y, Z] fp32 (device), starts int32 [n, 3] (device; patches inside the volume) →
    [n, px, py, pz] crops (no scaling)."""
    _check(vol, "crop_patches.vol", ndim=3)
    if starts.dtype != torch.int32 or not starts.is_cuda or starts.dim() != 2 or starts.shape[1] != 3:
        raise ValueError("crop_patches: starts must be a device int32 [n, 3] tensor")
    n = starts.shape[0]
    px, py, pz = patch
    if out is None:
        out = torch.empty((n, px, py, pz), device=vol.device, dtype=torch.float32)
    X, Y, Z = vol.shape
    call("mragan_crop_patches", _ptr(vol), X, Y, Z, _ptr(starts.contiguous()), n, px, py, pz, _ptr(out), _stream())
    return out
