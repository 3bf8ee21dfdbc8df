"""Tensor-level launchers for the HIP kernels in libespnet_amd.so.

Torch tensors are used only as device-memory handles (data_ptr / shape / stride) and for
the current HIP stream; every computation is one of the library's kernels.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch

from ._lib import (ACT_NONE, BF16, EPI_ACT, EPI_DACT, EPI_RESID, EPI_STORE, F32, ColsumProb, Epilogue,
                   GroupGemm, HipError, ReduceProb, lib)

__all__ = ["dt", "stream", "gemm", "linear", "linear_dx", "linear_dw", "workspace"]

_DT = {torch.float32: F32, torch.bfloat16: BF16}


class KernelProbe:
    """Measures named GEMM launches from inside the kernel (bench.py): the launch stamps its
    first-block start and last-block end on the GPU's constant 100 MHz clock
    (ea_gemm_set_probe); stream-ordered begin/end kernels accumulate the span, so a launch
    captured into a hipGraph is re-measured on every replay."""

    TICK_MS = 1e-5  # s_memrealtime: 100 MHz

    def __init__(self, names, device=None):
        self.names = set(names)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.slots = {n: torch.zeros(4, dtype=torch.int64, device=dev) for n in names}
        self.active = True

    def begin(self, name):
        if self.active and name in self.names:
            s = self.slots[name].data_ptr()
            lib.ea_probe_begin(s, stream())
            lib.ea_gemm_set_probe(s)

    def end(self, name):
        if self.active and name in self.names:
            lib.ea_gemm_set_probe(None)
            lib.ea_probe_end(self.slots[name].data_ptr(), stream())

    def reset(self):
        for t in self.slots.values():
            t.zero_()

    def mean_ms(self, name):
        tot, cnt = (int(x) for x in self.slots[name][2:4].tolist())
        return (tot / cnt * self.TICK_MS if cnt else float("nan")), cnt


class EventProbe:
    """The same begin/end interface as KernelProbe, timed with HIP events recorded on the
    launch stream around the named launch (eager launches only: not inside a graph capture).
    bench.py reports it beside the in-kernel probe and the rocprof average."""

    def __init__(self, names):
        self.names = set(names)
        self.pairs = {n: [] for n in names}
        self.active = True

    def begin(self, name):
        if self.active and name in self.names:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            self.pairs[name].append([ev, None])

    def end(self, name):
        if self.active and name in self.names:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream())
            self.pairs[name][-1][1] = ev

    def reset(self):
        for v in self.pairs.values():
            v.clear()

    def mean_ms(self, name):
        torch.cuda.synchronize()
        ts = [a.elapsed_time(b) for a, b in self.pairs[name] if b is not None]
        return (sum(ts) / len(ts) if ts else float("nan")), len(ts)


PROBE = None
# Stream-ordering diagnostics (tests/test_dp_streams_gpu.py): EA_DEBUG_DELAY_NS holds every side /
# auxiliary stream segment for that long before its first launch (ea_debug_spin), so a consumer
# that misses its dependency on a side-stream producer reads stale data in every run;
# EA_DEBUG_SERIAL=1 makes the main stream join the side / auxiliary stream at the end of every
# segment (the overlap keeps its launch order but nothing runs concurrently).  Read at call time.
DEBUG_DELAY_NS = int(os.environ.get("EA_DEBUG_DELAY_NS", "0"))
DEBUG_SERIAL = os.environ.get("EA_DEBUG_SERIAL", "0") != "0"


def _debug_enter(side):
    if DEBUG_DELAY_NS:
        lib.ea_debug_spin(DEBUG_DELAY_NS, side.cuda_stream)


def _debug_exit(main, side):
    if DEBUG_SERIAL:
        main.wait_stream(side)


# run weight-gradient GEMMs / bias reductions on a side stream (EA_OVERLAP_WGRAD=0: serial, for profiling)
OVERLAP_WGRAD = os.environ.get("EA_OVERLAP_WGRAD", "1") != "0"
_SIDE = {}
_SIDE_DIRTY = {}  # device -> the side stream forked since the main stream last joined it


class wgrad:
    """Context for weight-gradient work (dW GEMMs, bias column sums) that is off the
    backward critical path: it runs on a side HIP stream, ordered after everything the
    main stream has issued so far; `join()` makes the main stream wait for it.
    Tensors read on the side stream are record_stream()-ed so the caching allocator does
    not recycle them under it.

    While the pass's weight gradients and reductions are deferred (deferred_wgrad), a block
    of linear_dw / colsum calls only queues work, and the fork is skipped unless `launches`
    says the block launches kernels of its own: in a captured step every fork is a graph
    dependency whose event costs the main chain ~5 us even when nothing runs on the side
    (a launch inside a skipped fork simply runs on the current stream, in order)."""

    def __init__(self, *tensors, after=None, launches=False):
        self.tensors = tensors
        self.after = after  # fork from this event (fork_event) instead of the stream's current point
        self.launches = launches

    def __enter__(self):
        if not OVERLAP_WGRAD or not torch.cuda.is_available():  # (CPU: the gloo DP tests)
            self.ctx = None
            return self
        if not self.launches and WGRAD_Q.active and REDUCE_Q.active:
            self.ctx = None  # only deferred work inside: no fork
            return self
        main = torch.cuda.current_stream()
        dev = main.device
        side = _SIDE.get(dev)
        if side is None:
            side = _SIDE[dev] = torch.cuda.Stream(device=dev)
        if self.after is not None:
            side.wait_event(self.after)
        else:
            side.wait_stream(main)
        _SIDE_DIRTY[dev] = True
        for t in self.tensors:
            if t is not None:
                t.record_stream(side)
        self.ctx = torch.cuda.stream(side)
        self.ctx.__enter__()
        self.streams = (main, side)
        _debug_enter(side)
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            _debug_exit(*self.streams)
        return False


def fork_event():
    """An event at the main stream's current point for a later wgrad(after=...), or None: a
    side-stream GEMM forked from an earlier point of the main stream is issued after the main
    stream's next kernel, so in the captured graph the main chain's kernel is the first successor
    of the fork point.  Single process only: with the data-parallel hooks (GRAD_READY) the side
    stream also carries the bucket all-reduces, and the late fork measured 4% slower there
    (1811 -> 1739 utt/s in the DP rehearsal, profiles/r5_fork_after_dp_ab.txt)."""
    if not OVERLAP_WGRAD or GRAD_READY is not None or not torch.cuda.is_available():
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    return ev


def join_wgrad(device=None):
    """Main stream waits for all weight-gradient work issued so far (nothing to wait for —
    and no graph dependency — when the side stream was not forked since the last join)."""
    if not _SIDE:
        return
    main = torch.cuda.current_stream()
    side = _SIDE.get(main.device)
    if side is not None and _SIDE_DIRTY.get(main.device, True):
        main.wait_stream(side)
        _SIDE_DIRTY[main.device] = False
    WGRAD_Q.side_events = []  # whatever the side stream produced is ordered before main now


def on_side() -> bool:
    """The current stream is the weight-gradient side stream."""
    if not _SIDE or not torch.cuda.is_available():
        return False
    cur = torch.cuda.current_stream()
    side = _SIDE.get(cur.device)
    return side is not None and cur == side


# latency-bound work that leaves most CUs idle (the CTC lattice: 2 workgroups per utterance)
# overlaps independent work on an auxiliary stream (EA_OVERLAP_AUX=0: serial)
OVERLAP_AUX = os.environ.get("EA_OVERLAP_AUX", "1") != "0"
_AUX = {}


class aux:
    """Context: the enclosed launches run on the auxiliary stream, ordered after everything the
    main stream has issued so far (or, with `after=event`, only after that event); `join_aux()`
    makes the main stream wait for them.  The tensors it touches are record_stream()-ed for
    the caching allocator."""

    def __init__(self, *tensors, after=None):
        self.tensors = tensors
        self.after = after

    def __enter__(self):
        if not OVERLAP_AUX or not torch.cuda.is_available():
            self.ctx = None
            return self
        main = torch.cuda.current_stream()
        dev = main.device
        st = _AUX.get(dev)
        if st is None:
            st = _AUX[dev] = torch.cuda.Stream(device=dev)
        if self.after is not None:
            st.wait_event(self.after)
        else:
            st.wait_stream(main)
        for t in self.tensors:
            if t is not None:
                t.record_stream(st)
        self.ctx = torch.cuda.stream(st)
        self.ctx.__enter__()
        self.streams = (main, st)
        _debug_enter(st)
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            _debug_exit(*self.streams)
        return False


# the CTC head's backward (gradient kernel + ctc_lo input gradient) overlaps the attention
# decoder's backward on the auxiliary stream (EA_OVERLAP_CTC_BWD=0: serial)
OVERLAP_CTC_BWD = os.environ.get("EA_OVERLAP_CTC_BWD", "1") != "0"
_AUX_FORK = {}


def mark_aux_fork():
    """Record where the loss gradients exist on the main stream (the hybrid combination's
    backward): a backward issued later on the host can fork from this point onto the
    auxiliary stream instead of queueing behind everything issued in between."""
    if not (OVERLAP_AUX and OVERLAP_CTC_BWD) or not torch.cuda.is_available():
        return
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    _AUX_FORK[torch.cuda.current_device()] = ev


def take_aux_fork():
    """The event mark_aux_fork() recorded on this device (consumed), or None."""
    if not _AUX_FORK or not torch.cuda.is_available():
        return None
    return _AUX_FORK.pop(torch.cuda.current_device(), None)


def join_aux():
    """Main stream waits for all auxiliary-stream work issued so far."""
    if not _AUX:
        return
    main = torch.cuda.current_stream()
    st = _AUX.get(main.device)
    if st is not None:
        main.wait_stream(st)


GRAD_READY = None  # callable(prefix): a block's parameter gradients are final (DP overlap)


def grad_ready(bound):
    """A block's backward is done.  Data parallel (GRAD_READY set): the hook flushes the
    deferred weight gradients and issues the bucket all-reduces from the side stream, so the
    main stream goes on with the backward.  Single process: the main stream joins the side
    stream here, once per block (the deferred queues flush at the end of the pass; flushing
    them per block on the side stream, or joining only once per pass, measured slower:
    profiles/r3_stream_wgrad_ab.txt)."""
    if GRAD_READY is not None:
        GRAD_READY(bound.prefix)
        return
    join_wgrad()


def flush_wgrad_side(after=None):
    """Launch the weight gradients queued so far (one grouped GEMM) on the side stream, forked
    from `after` (fork_event); single process only (the data-parallel hooks flush per bucket)."""
    if not (WGRAD_Q.active and WGRAD_Q.items) or GRAD_READY is not None:
        return
    if not OVERLAP_WGRAD or not torch.cuda.is_available():
        return
    with wgrad(*WGRAD_Q.tensors(), after=after, launches=True):
        WGRAD_Q.flush()


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise HipError(f"unsupported dtype {t.dtype}") from None


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


_WS = {}


def workspace(numel: int, device) -> torch.Tensor:
    """Persistent f32 scratch (split-K slabs), one per (device, stream); grows monotonically."""
    key = (str(device), "f32", stream())
    ws = _WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


_SPLITK_WS = 1 << 25  # 32M floats


def make_epi(kind=EPI_STORE, *, alpha=1.0, beta=0.0, bias=None, post_scale=1.0, act=ACT_NONE,
             aux=None, resid=None, rscale=1.0, drop_p=0.0, seed=0):
    e = Epilogue()
    e.kind = kind
    e.act = act
    e.alpha = alpha
    e.beta = beta
    e.post_scale = post_scale
    e.rscale = rscale
    e.drop_p = drop_p
    e.seed = seed & 0xFFFFFFFFFFFFFFFF
    e.bias = ptr(bias)
    if aux is not None:
        e.aux = aux.data_ptr()
        e.aux_dtype = dt(aux)
        e.ldaux = aux.stride(-2)
    if resid is not None:
        e.resid = resid.data_ptr()
        e.ldr = resid.stride(-2)
    return e


MN_TAIL_COPIES = 0  # operands re-homed by _mn_tail_guard (tests read it)


def _mn_tail_guard(X, MN, K, ld, s, batch, nh):
    """ea_gemm's contract for an MN-major bf16 operand whose width MN is not a multiple of 8
    (include/espnet_amd.h): the LDS-DMA loads move whole 16-B chunks, so the last chunk of a
    row reads up to 7 elements past MN — every row, the last one included, must be readable to
    MN rounded up to 8.  A view ending closer than that to the end of its storage (a
    column-offset slice at the end of an allocation) is copied, with its strides, into a
    buffer padded by 8 elements; the GEMM then reads the copy."""
    global MN_TAIL_COPIES
    if X.dtype != torch.bfloat16 or MN % 8 == 0 or K <= 0:
        return X
    esz = X.element_size()
    total = X.untyped_storage().nbytes() // esz
    off = X.storage_offset()
    last = off + (batch - 1) * s[0] + (nh - 1) * s[1] + (K - 1) * ld  # start of the last row read
    if last + (MN + 7) // 8 * 8 <= total:
        return X
    span = last + MN - off
    buf = torch.empty(span + 8, dtype=X.dtype, device=X.device)
    buf[:span].copy_(torch.as_strided(X, (span,), (1,), off))  # same strides from the new base
    buf[span:].zero_()
    MN_TAIL_COPIES += 1
    return buf


def gemm(A, B, C, *, M, N, K, a_kmajor, b_kmajor, lda, ldb, ldc,
         batch=1, nh=1, sA=(0, 0), sB=(0, 0), sC=(0, 0), epi: Epilogue = None, splitk=True):
    """Raw batched GEMM (see include/espnet_amd.h: ea_gemm).  An MN-major bf16 operand whose
    last row cannot be read to its width rounded up to 8 is re-homed first (_mn_tail_guard)."""
    if A.dtype != B.dtype:
        raise HipError(f"gemm operand dtypes differ: {A.dtype} vs {B.dtype}")
    if epi is None:
        epi = make_epi()
    if not a_kmajor:
        A = _mn_tail_guard(A, M, K, lda, sA, batch, nh)
    if not b_kmajor:
        B = _mn_tail_guard(B, N, K, ldb, sB, batch, nh)
    ws = workspace(_SPLITK_WS, A.device) if splitk else None
    lib.ea_gemm(dt(A), int(a_kmajor), int(b_kmajor), M, N, K,
                A.data_ptr(), lda, sA[0], sA[1],
                B.data_ptr(), ldb, sB[0], sB[1],
                batch, nh,
                C.data_ptr(), dt(C), ldc, sC[0], sC[1],
                ctypes.byref(epi), ptr(ws), 0 if ws is None else ws.numel(), stream())
    return C


def _rows(x):
    """(…, K) tensor with unit inner stride -> (rows, K, ld)."""
    if x.stride(-1) != 1:
        raise HipError("inner dimension must be contiguous")
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    ld = x.stride(-2) if x.dim() >= 2 else K
    if x.dim() > 2:
        # leading dims must collapse onto a single row stride
        exp = ld
        for d in range(x.dim() - 2, 0, -1):
            exp *= x.shape[d]
            if x.shape[d - 1] > 1 and x.stride(d - 1) != exp:
                raise HipError("leading dims do not collapse onto one row stride")
    return rows, K, ld


def linear(x, w, out, *, epi: Epilogue = None):
    """out[r, n] = epi(sum_k x[r, k] * w[n, k]) — torch.nn.Linear forward."""
    M, K, lda = _rows(x)
    N = w.shape[0]
    _, _, ldc = _rows(out)
    return gemm(x, w, out, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=lda, ldb=w.stride(0),
                ldc=ldc, epi=epi)


# ----------------------------------------------------------------------------- transposed shadow
# The Linear input gradient dX = dY . W has N = K_in: for K_in <= 512 it runs on the narrow
# 64x128 / 32x128 tiles, where W read MN-major (128-wide panels, transposed LDS reads) costs
# about a third of the launch.  A bf16 W^T copy per such weight, rewritten by one grouped
# transpose after every optimizer step (and shadow refresh), lets those GEMMs read both
# operands K-major.  EA_WT_SHADOW=0 turns it off (A/B).
WT_SHADOW = os.environ.get("EA_WT_SHADOW", "1") != "0"
WT_MAX_KIN = 512  # 2048-wide inputs too measured neutral (round 4): the FFN w_2 epilogue sets its time
TSHADOWS = {}  # arena shadow storage pointer -> weakref(TransposedShadow) (the arena owns it)


class TransposedShadow:
    def __init__(self, shadow):
        self.shadow = shadow  # the arena's bf16 weight shadow (flat)
        self.items = {}  # (element offset, R, C) -> (C, R) bf16 tensor
        self.tiles = self.probs = None
        self.ntiles = 0
        # set once a hipGraph captured refresh(): that graph holds this tile / problem table
        # and its count, so no weight may be registered afterwards (its W^T would never be
        # refreshed by the graph, and a rebuilt table would free the captured one) — such a
        # weight keeps the MN-major path instead
        self.frozen = False

    def _rebuild(self):
        probs, tiles = [], []
        for pi, ((off, R, C), dst) in enumerate(self.items.items()):
            probs.append((off, dst.data_ptr(), R | (C << 32)))
            tiles += [(pi, tr, tc, 0) for tr in range((R + 63) // 64) for tc in range((C + 63) // 64)]
        dev = self.shadow.device
        self.probs = torch.tensor(probs, dtype=torch.int64).to(dev)
        self.tiles = torch.tensor(tiles, dtype=torch.int32).to(dev)
        self.ntiles = len(tiles)

    def get(self, w):
        """W^T (C x R, row-major) of a contiguous (R x C) view of the shadow, created (and
        transposed from the current shadow) on first use."""
        off = (w.data_ptr() - self.shadow.data_ptr()) // w.element_size()
        key = (off, int(w.shape[0]), int(w.shape[1]))
        wt = self.items.get(key)
        if wt is None:
            if self.frozen or torch.cuda.is_current_stream_capturing():
                return None  # registration happens in the eager warm-up steps
            wt = torch.empty(key[2], key[1], dtype=w.dtype, device=w.device)
            self.items[key] = wt
            self._rebuild()
            self.refresh()
        return wt

    def refresh(self):
        if torch.cuda.is_current_stream_capturing():
            self.frozen = True
        if self.ntiles:
            lib.ea_transpose_bf16_grouped(self.ntiles, self.tiles.data_ptr(), self.probs.data_ptr(),
                                          self.shadow.data_ptr(), stream())


def attach_transposed_shadow(shadow):
    """Register an arena's bf16 shadow for transposed copies (returns the registry, or None)."""
    if not WT_SHADOW or shadow is None or shadow.dtype != torch.bfloat16:
        return None
    ts = TransposedShadow(shadow)
    TSHADOWS[shadow.untyped_storage().data_ptr()] = weakref.ref(ts)
    return ts


def _transposed(w):
    if not TSHADOWS or w.dtype != torch.bfloat16 or w.dim() != 2 or w.shape[1] > WT_MAX_KIN:
        return None
    if w.stride(1) != 1 or w.stride(0) != w.shape[1] or w.shape[0] % 8 or w.shape[1] % 8:
        return None
    ref = TSHADOWS.get(w.untyped_storage().data_ptr())
    ts = None if ref is None else ref()
    if ts is None or ts.shadow.untyped_storage().data_ptr() != w.untyped_storage().data_ptr():
        return None
    return ts.get(w)


def linear_dx(dy, w, out, *, epi: Epilogue = None):
    """out[r, k] = epi(sum_n dy[r, n] * w[n, k]) — Linear input gradient (W^T K-major from the
    transposed shadow when the arena keeps one for w)."""
    M, N, lda = _rows(dy)
    K = w.shape[1]
    _, _, ldc = _rows(out)
    wt = _transposed(w)
    if wt is not None:
        return gemm(dy, wt, out, M=M, N=K, K=N, a_kmajor=1, b_kmajor=1, lda=lda, ldb=wt.stride(0),
                    ldc=ldc, epi=epi)
    return gemm(dy, w, out, M=M, N=K, K=N, a_kmajor=1, b_kmajor=0, lda=lda, ldb=w.stride(0),
                ldc=ldc, epi=epi)


def linear_dw(dy, x, dw, *, accumulate=False, post=None):
    """dw[n, k] (+)= sum_r dy[r, n] * x[r, k] — Linear weight gradient (f32 out).  While the
    weight-gradient queue is active (a training backward pass) the GEMM is deferred and
    launched with the others of the pass by WGRAD_Q.flush(); `post` (a callable consuming dw,
    e.g. a permute into the gradient arena) then runs right after that launch."""
    R, N, lddy = _rows(dy)
    R2, K, ldx = _rows(x)
    if R != R2:
        raise HipError("row mismatch in linear_dw")
    beta = 1.0 if accumulate else 0.0
    if WGRAD_Q.active and WGRAD_Q.add(dy, x, dw, M=N, N=K, K=R, lda=lddy, ldb=ldx, ldc=dw.stride(0), beta=beta,
                                      post=post):
        return dw
    gemm(dy, x, dw, M=N, N=K, K=R, a_kmajor=0, b_kmajor=0, lda=lddy, ldb=ldx,
         ldc=dw.stride(0), epi=make_epi(beta=beta))
    if post is not None:
        post()
    return dw


# ----------------------------------------------------------------------------- deferred weight gradients
DEFER_WGRAD = os.environ.get("EA_DEFER_WGRAD", "1") != "0"
# bytes the deferred queues may keep alive (queued operands / partial buffers) before they
# flush early: a pass whose queued dY / X / LayerNorm partials exceed it launches what it has
# and continues (C3 queues ~3.5 GB per backward, under the default)
DEFER_BUDGET = int(float(os.environ.get("EA_DEFER_BUDGET_MB", "8192")) * 2 ** 20)
_GWS = {}


def _nbytes(t):
    return t.numel() * t.element_size()


class WgradQueue:
    """The Linear weight gradients of one backward pass (linear_dw: dW (+)= dY^T X, K = the
    pass's token count), deferred and launched together as ONE grouped GEMM
    (ea_gemm_grouped: every 256x256 tile over its problem's whole K on the pipelined main
    loop) instead of one split-K GEMM + combine pass per Linear.  The queue keeps dY and X
    alive until the flush.  Problems are ordered longest-K first; a problem whose output
    overlaps a queued one flushes the queue first (a launch never holds two writers of one
    element)."""

    def __init__(self):
        self.active = False
        self.items = []
        self.posts = []
        self.pending = 0  # bytes of queued dY / X kept alive
        # events recorded on the side stream where items were queued there (their operands may
        # be side-stream products, e.g. the linear_pos GEMM's dpp) since the main stream last
        # joined it: a flush on another stream waits for them first (data parallel: no
        # per-block joins)
        self.side_events = []

    def add(self, dy, x, dw, *, M, N, K, lda, ldb, ldc, beta, post=None) -> bool:
        if not (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dw.dtype == torch.float32):
            return False
        if (lda % 8 or ldb % 8 or dy.data_ptr() % 16 or x.data_ptr() % 16 or N % 4 or ldc % 4
                or dw.data_ptr() % 16 or M <= 0 or N <= 0 or K <= 0):
            return False
        if 2.0 * K * lda >= 4.0e9 or 2.0 * K * ldb >= 4.0e9:
            return False
        lo = dw.data_ptr()
        hi = lo + ((M - 1) * ldc + N) * 4
        if any(lo < it[-1] and it[-2] < hi for it in self.items):
            self.flush()
        if on_side():
            ev = torch.cuda.Event()
            ev.record()
            self.side_events.append(ev)
        self.items.append((K, dy, x, dw, M, N, lda, ldb, ldc, beta, lo, hi))
        if post is not None:
            self.posts.append(post)
        self.pending += _nbytes(dy) + _nbytes(x)
        if self.pending > DEFER_BUDGET:
            self.flush()
        return True

    def flush(self):
        """Launch the queued GEMMs on the current stream."""
        if not self.items:
            return
        if self.side_events:
            if not on_side():
                cur = torch.cuda.current_stream()
                for ev in self.side_events:
                    cur.wait_event(ev)
            self.side_events = []
        items = sorted(self.items, key=lambda t: -t[0])
        posts = self.posts
        self.items = []
        self.posts = []
        self.pending = 0
        n = len(items)
        cur = torch.cuda.current_stream()
        for it in items:  # operands may come from another stream's pool: keep them until this launch ran
            for t in it[1:4]:
                t.record_stream(cur)
        arr = (GroupGemm * n)()
        ntiles = 0
        for i, (K, dy, x, dw, M, N, lda, ldb, ldc, beta, _, _) in enumerate(items):
            arr[i] = GroupGemm(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), lda, ldb, ldc, M, N, K, beta)
            ntiles += ((M + 255) // 256) * ((N + 255) // 256)
        nbytes = ctypes.c_long(0)
        lib.ea_gemm_grouped_ws_bytes(n, ntiles, ctypes.addressof(nbytes))
        dev = items[0][1].device
        key = (str(dev), stream())
        ws = _GWS.get(key)
        if ws is None or ws.numel() < nbytes.value:
            ws = torch.empty(max(nbytes.value, 1 << 16), dtype=torch.uint8, device=dev)
            _GWS[key] = ws
        lib.ea_gemm_grouped(0, 0, n, ctypes.addressof(arr), ws.data_ptr(), ws.numel(), stream())
        for post in posts:
            post()

    def tensors(self):
        return [t for it in self.items for t in (it[1], it[2])]


WGRAD_Q = WgradQueue()

# ----------------------------------------------------------------------------- deferred gradient reductions
DEFER_REDUCE = os.environ.get("EA_DEFER_REDUCE", "1") != "0"
_RWS = {}


def _table_ws(kind, nbytes, dev):
    key = (str(dev), stream(), kind)
    ws = _RWS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _RWS[key] = ws
    return ws


class ReduceQueue:
    """The parameter-gradient reductions of one backward pass, deferred: bias column sums
    (colsum: torch.nn.Linear bias.grad = dY summed over tokens) and the ordered sums of the
    LayerNorm (dgamma | dbeta) row-block partials.  flush() runs every queued column sum in
    ONE grouped launch (ea_colsum_grouped), then every reduction in ONE more
    (ea_reduce_grouped) — instead of ~450 launches of a few microseconds per C3 step.  The
    column sums use ea_colsum's row blocking, so results are bit-identical to the per-call
    path.  Outputs that overlap a queued one flush the queue first."""

    def __init__(self):
        self.active = False
        self.colsums = []
        self.reduces = []
        self.spans = []
        self.pending = 0  # bytes of queued inputs / partial buffers kept alive

    def _account(self, t):
        self.pending += _nbytes(t)
        if self.pending > DEFER_BUDGET:
            self.flush()

    def _claim(self, out, n):
        lo = out.data_ptr()
        hi = lo + 4 * n
        if any(lo < h and l_ < hi for l_, h in self.spans):
            self.flush()
        self.spans.append((lo, hi))

    def add_colsum(self, x, out, accumulate) -> bool:
        if x.dtype not in (torch.bfloat16, torch.float32) or out.dtype != torch.float32 or not out.is_contiguous():
            return False
        rows, n, ld = _rows(x)
        if rows <= 0 or n % 4 or ld % 4 or x.data_ptr() % (8 if x.dtype == torch.bfloat16 else 16):
            return False
        self._claim(out, n)
        self.colsums.append((x, rows, n, ld, out, accumulate))
        self._account(x)
        return True

    def add_reduce(self, part, nparts, n, stride, out, accumulate=True):
        self._claim(out, n)
        self.reduces.append((part, nparts, n, stride, out, accumulate))
        self._account(part)

    def tensors(self):
        return [c[0] for c in self.colsums] + [r[0] for r in self.reduces]

    def flush(self):
        if not self.colsums and not self.reduces:
            return
        colsums, reduces = self.colsums, list(self.reduces)
        self.colsums, self.reduces, self.spans = [], [], []
        self.pending = 0
        cur = torch.cuda.current_stream()
        for t in [c[0] for c in colsums] + [r[0] for r in reduces]:
            t.record_stream(cur)
        dev = (colsums[0][0] if colsums else reduces[0][0]).device
        cb, rb = ctypes.c_long(0), ctypes.c_long(0)
        if colsums:
            rpps = [max(32, (c[1] + 127) // 128) for c in colsums]  # ea_colsum's row blocking
            nrbs = [(c[1] + r - 1) // r for c, r in zip(colsums, rpps)]
            part = torch.empty(sum(nrb * c[2] for c, nrb in zip(colsums, nrbs)), dtype=torch.float32, device=dev)
            arr = (ColsumProb * len(colsums))()
            off = 0
            for i, ((x, rows, n, ld, out, acc), rpp, nrb) in enumerate(zip(colsums, rpps, nrbs)):
                arr[i] = ColsumProb(x.data_ptr(), part.data_ptr() + 4 * off, ld, rows, n, dt(x), rpp)
                reduces.append((part, nrb, n, n, out, acc, off))
                off += nrb * n
            lib.ea_grouped_table_bytes(len(colsums), ctypes.addressof(cb), ctypes.addressof(rb))
            ws = _table_ws("colsum", cb.value, dev)
            lib.ea_colsum_grouped(len(colsums), ctypes.addressof(arr), ws.data_ptr(), ws.numel(), stream())
        arr = (ReduceProb * len(reduces))()
        for i, r in enumerate(reduces):
            part, nparts, n, stride, out, acc = r[:6]
            off = r[6] if len(r) > 6 else 0
            arr[i] = ReduceProb(part.data_ptr() + 4 * off, out.data_ptr(), stride, nparts, n, int(acc))
        lib.ea_grouped_table_bytes(len(reduces), ctypes.addressof(cb), ctypes.addressof(rb))
        ws = _table_ws("reduce", rb.value, dev)
        lib.ea_reduce_grouped(len(reduces), ctypes.addressof(arr), ws.data_ptr(), ws.numel(), stream())


REDUCE_Q = ReduceQueue()


def flush_deferred():
    """Launch every deferred weight gradient and gradient reduction (current stream)."""
    WGRAD_Q.flush()
    REDUCE_Q.flush()


def deferred_tensors():
    return WGRAD_Q.tensors() + REDUCE_Q.tensors()


class deferred_wgrad:
    """Context of a training backward pass: linear_dw calls inside are queued
    (EA_DEFER_WGRAD=0 turns this off), so are the bias column sums and LayerNorm
    parameter-gradient reductions (EA_DEFER_REDUCE=0); all are flushed on exit, on the
    current stream."""

    def __enter__(self):
        self.prev = (WGRAD_Q.active, REDUCE_Q.active)
        WGRAD_Q.active = DEFER_WGRAD
        REDUCE_Q.active = DEFER_REDUCE
        return WGRAD_Q

    def __exit__(self, *exc):
        WGRAD_Q.active, REDUCE_Q.active = self.prev
        if exc[0] is None:
            if GRAD_READY is None and OVERLAP_WGRAD and torch.cuda.is_available():
                # the pass's reductions (bias column sums, LayerNorm parameter sums: bandwidth-
                # bound) on the side stream beside the grouped weight-gradient GEMM (MFMA-bound)
                # on this one; disjoint outputs (bias / norm vs weight gradients)
                with wgrad(*REDUCE_Q.tensors(), launches=True):
                    REDUCE_Q.flush()
                WGRAD_Q.flush()
            else:
                flush_deferred()
            if GRAD_READY is None:
                join_wgrad()  # gradients written on the side stream during the pass are final
        else:
            WGRAD_Q.items, WGRAD_Q.posts = [], []
            REDUCE_Q.colsums, REDUCE_Q.reduces, REDUCE_Q.spans = [], [], []
        return False


# ----------------------------------------------------------------------------- scratch
_SCRATCH = {}


def scratch(numel: int, device, tag="ws") -> torch.Tensor:
    """Stream-ordered f32 scratch shared by consecutive kernels (partials, reductions); one
    per (device, stream) so the weight-gradient side stream never races the main one."""
    key = (str(device), tag, stream())
    t = _SCRATCH.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1 << 22), dtype=torch.float32, device=device)
        _SCRATCH[key] = t
    return t


def _ws(device, numel=1 << 22):
    w = scratch(numel, device)
    return w.data_ptr(), w.numel()


# ----------------------------------------------------------------------------- norms
def layernorm_fwd(x, gamma, beta, y, mean, rstd, eps=1e-12):
    rows, d, ldx = _rows(x)
    lib.ea_layernorm_fwd(rows, d, x.data_ptr(), ldx, gamma.data_ptr(), beta.data_ptr(), eps,
                         y.data_ptr(), dt(y), y.stride(-2) if y.dim() > 1 else d,
                         mean.data_ptr(), rstd.data_ptr(), stream())


def linear_ln(x, gamma, beta, w, out, *, epi=None, eps=1e-12):
    """out = epi(LayerNorm(x) . w^T) in one launch (ea_gemm_ln): x f32 (rows, K), w bf16
    (N, K); the normalised rows are rounded to bf16 as the unfused LayerNorm stores them."""
    rows, K, ldx = _rows(x)
    N = w.shape[0]
    if epi is None:
        epi = make_epi()
    lib.ea_gemm_ln(rows, N, K, x.data_ptr(), ldx, gamma.data_ptr(), beta.data_ptr(), ctypes.c_float(eps),
                   w.data_ptr(), w.stride(0), out.data_ptr(), dt(out), out.stride(0), ctypes.byref(epi), stream())
    return out


def layernorm_bwd(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, accumulate=True, drop=None):
    """drop=(y, scale, p, seed[, ycol]): also y = dropout(scale * dx) once dx is final (the next
    residual site's dropout backward, ea_layernorm_bwd_drop), instead of an ea_scale_dropout
    pass; ycol (+)= column sums of y (that site's bias gradient) from the same kernel."""
    rows, d, ldx = _rows(x)
    _, _, lddy = _rows(dy)
    _, _, lddx = _rows(dx)
    if drop is not None:
        y, ysc, yp, yseed = drop[:4]
        ycol = drop[4] if len(drop) > 4 else None
        _, _, ldy = _rows(y)
        dargs = (y.data_ptr(), dt(y), ldy, float(ysc), float(yp), yseed & 0xFFFFFFFFFFFFFFFF,
                 0 if ycol is None else ycol.data_ptr())
    if REDUCE_Q.active and rows > 0 and dbeta.data_ptr() == dgamma.data_ptr() + 4 * d:
        # dx now; the (dgamma | dbeta) row-block partials go to a buffer of their own and are
        # summed with the pass's other parameter-gradient reductions (REDUCE_Q.flush)
        # the vectorized kernel's block count (16-row blocks; ln_bwd_impl), the generic paths'
        # at most 128 blocks
        vec8 = (d % 8 == 0 and d <= 1024 and lddy % 8 == 0 and ldx % 4 == 0 and lddx % 4 == 0
                and x.data_ptr() % 16 == 0 and dy.data_ptr() % 16 == 0 and dx.data_ptr() % 16 == 0
                and gamma.data_ptr() % 16 == 0)
        nparts_max = (rows + 15) // 16 if vec8 else max((rows + 15) // 16, 128)
        part = torch.empty(nparts_max * (3 if drop is not None else 2) * d, dtype=torch.float32, device=x.device)
        np_ = ctypes.c_int(0)
        if drop is not None:
            yparts = ctypes.c_int(0)
            lib.ea_layernorm_bwd_partials_drop(rows, d, dy.data_ptr(), dt(dy), lddy, x.data_ptr(), ldx,
                                               gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                               lddx, int(accumulate), part.data_ptr(), part.numel(),
                                               ctypes.addressof(np_), *dargs, ctypes.addressof(yparts), stream())
            if yparts.value:
                npv = np_.value
                REDUCE_Q.add_reduce(part[npv * 2 * d:], npv, d, d, ycol, accumulate=True)
        else:
            lib.ea_layernorm_bwd_partials(rows, d, dy.data_ptr(), dt(dy), lddy, x.data_ptr(), ldx, gamma.data_ptr(),
                                          mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), lddx, int(accumulate),
                                          part.data_ptr(), part.numel(), ctypes.addressof(np_), stream())
        REDUCE_Q.add_reduce(part, np_.value, 2 * d, 2 * d, dgamma, accumulate=True)
        return
    w, n = _ws(x.device, max(1 << 22, 1024 * d))
    if drop is not None:
        lib.ea_layernorm_bwd_drop(rows, d, dy.data_ptr(), dt(dy), lddy, x.data_ptr(), ldx, gamma.data_ptr(),
                                  mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), lddx, int(accumulate),
                                  dgamma.data_ptr(), dbeta.data_ptr(), 1, w, n, *dargs, stream())
        return
    lib.ea_layernorm_bwd(rows, d, dy.data_ptr(), dt(dy), lddy, x.data_ptr(), ldx, gamma.data_ptr(),
                         mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), lddx, int(accumulate),
                         dgamma.data_ptr(), dbeta.data_ptr(), 1, w, n, stream())


def reduce_rows(part, nparts, n, stride, out, accumulate=True):
    """out[c] (+)= sum_p part[p*stride + c], p in fixed order (deterministic); deferred with the
    pass's other parameter-gradient reductions while the reduction queue is active."""
    if REDUCE_Q.active:
        REDUCE_Q.add_reduce(part, nparts, n, stride, out, accumulate)
        return
    lib.ea_reduce_partials(nparts, n, part.data_ptr(), stride, out.data_ptr(), int(accumulate), stream())


def colsum(x, out, accumulate=True, defer=True):
    """out (+)= column sums of x.  While the reduction queue is active the sum is deferred to
    REDUCE_Q.flush(): pass defer=False when x is modified in place before the pass ends."""
    if defer and REDUCE_Q.active and REDUCE_Q.add_colsum(x, out, accumulate):
        return
    rows, n, ld = _rows(x)
    w, wn = _ws(x.device)
    lib.ea_colsum(rows, n, x.data_ptr(), dt(x), ld, out.data_ptr(), int(accumulate), w, wn, stream())


def batchnorm_fwd(y, gamma, beta, mean, rstd, run_mean, run_var, nbt, z, training, act,
                  eps=1e-5, momentum=0.1):
    rows, C, _ = _rows(y)
    w, wn = _ws(y.device, (min(rows // 16 + 1, 256) + 2) * 2 * C)
    lib.ea_batchnorm_fwd(rows, C, y.data_ptr(), gamma.data_ptr(), beta.data_ptr(), eps, momentum,
                         int(training), mean.data_ptr(), rstd.data_ptr(), ptr(run_mean), ptr(run_var),
                         ptr(nbt), act, z.data_ptr(), dt(z), w, wn, stream())


def batchnorm_bwd(dz, y, mean, rstd, gamma, beta, act, dy, dgamma, dbeta):
    rows, C, _ = _rows(y)
    w, wn = _ws(y.device, (min(rows // 16 + 1, 256) + 2) * 2 * C)
    lib.ea_batchnorm_bwd(rows, C, dz.data_ptr(), dt(dz), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                         gamma.data_ptr(), beta.data_ptr(), act, dy.data_ptr(), dgamma.data_ptr(),
                         dbeta.data_ptr(), 1, w, wn, stream())


# ----------------------------------------------------------------------------- elementwise
def scale_dropout(x, y, scale=1.0, p=0.0, seed=0):
    rows, cols, ldx = _rows(x)
    _, _, ldy = _rows(y)
    lib.ea_scale_dropout(rows, cols, x.data_ptr(), dt(x), ldx, y.data_ptr(), dt(y), ldy,
                         float(scale), float(p), seed & 0xFFFFFFFFFFFFFFFF, stream())
    return y


def scale_dropout_colsum(x, y, out, scale=1.0, p=0.0, seed=0, accumulate=True):
    """y = dropout(scale * x) and out (+)= column sums of y: the two-pass form (ea_scale_dropout,
    then ea_colsum on the weight-gradient side stream).  The one-pass kernel
    (ea_scale_dropout_colsum) puts the reduction on the backward's critical path and measured
    slower on MI355X (C3: 27.43-28.07 vs 27.26 ms/step, round 1)."""
    scale_dropout(x, y, scale=scale, p=p, seed=seed)
    with wgrad(y):
        colsum(y, out, accumulate=accumulate)
    return y


def cast(x, dtype):
    """Copy-convert (f32 <-> bf16) through ea_scale_dropout; returns x if already dtype."""
    if x.dtype == dtype:
        return x
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    scale_dropout(x.reshape(-1, x.shape[-1]), y.view(-1, y.shape[-1]))
    return y


def permute3(src, dst, A, Bd, Cd, accumulate=False):
    lib.ea_permute3(A, Bd, Cd, src.data_ptr(), dt(src), dst.data_ptr(), dt(dst), int(accumulate), stream())
