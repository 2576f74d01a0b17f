"""cairo_amd -- MI355X-native EVX-1 (hinike/cairo) encode path.

The product is ``_lib/libcairo_amd.so``: hand-written HIP kernels for gfx950
(convert, inter search, macroblock wavefront with in-loop deblock), the host entropy stage
and the drop-in ``evx1_encoder`` / ``bit_stream`` C++ API.  This module is a
thin ctypes view of its C ABI (``include/cairo_amd.h``) for tests, the bench
and Python callers.  There is no Python or CPU fallback for the hot path: if
the library is missing, importing the bindings raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libcairo_amd.so")

# evx_block_desc (reference common.h:78-95, pack(2), 16 bytes)
BLOCK_DESC = np.dtype(
    [
        ("block_type", "<u4"),
        ("prediction_target", "u1"),
        ("pad", "u1"),
        ("motion_x", "<i2"),
        ("motion_y", "<i2"),
        ("sp_pred", "u1"),
        ("sp_amount", "u1"),
        ("sp_index", "u1"),
        ("q_index", "u1"),
        ("variance", "<i2"),
    ]
)
assert BLOCK_DESC.itemsize == 16

EVX_SUCCESS = 0
API_VERSION = 3  # include/cairo_amd.h CAIRO_AMD_API_VERSION
OUT_COEF, OUT_FEED = 1, 2  # cairo_ctx_set_outputs
FEED_NONE, FEED_VALID, FEED_OVERFLOW = 0, 1, 2
MAX_COEF_CHUNKS = 16  # CAIRO_MAX_COEF_CHUNKS
PEER_SIZE = 3 * 4 + 7 * 4 + 2 * 8 + MAX_COEF_CHUNKS * 8 + 2 * 64 + MAX_COEF_CHUNKS * 64  # sizeof(cairo_peer)
# EVX_PEEK_STATE (reference evx1.h:55-64)
PEEK_SOURCE, PEEK_PREDICTION, PEEK_BLOCK_TABLE, PEEK_QUANT_TABLE, PEEK_SPMP_TABLE, PEEK_BLOCK_VARIANCE, \
    PEEK_DESTINATION = range(7)
MAX_BATCH = 48  # kMaxBatch (kernels.h CAIRO_MAX_BATCH): frames per engine launch, stamp layout
EVX_ERROR_HARDWAREFAIL = 5


# In-kernel wait kinds of a timeout record (include/cairo_amd.h CAIRO_WAIT_*)
WAIT_KINDS = {1: "records", 2: "granule", 3: "prev_progress", 4: "row_above", 5: "batch", 6: "injected",
              9: "host_mark"}
TIMEOUT_FIELDS = ("kind", "epoch", "index", "row", "member", "need", "on", "seen_lo", "seen_hi")


class CairoError(RuntimeError):
    def __init__(self, what: str, status: int, timeout: dict | None = None):
        msg = f"{what} failed with evx_status {status}"
        if timeout:
            msg += f" (in-kernel wait timed out: {timeout})"
        super().__init__(msg)
        self.status = status
        self.timeout = timeout  # the first timed-out wait (Context.timeout_info), if one was reported


_lib = None


def lib() -> ctypes.CDLL:
    """Load libcairo_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build()"
        )
    L = ctypes.CDLL(LIB_PATH)
    P, I, U, V = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, None
    sig = {
        "cairo_ctx_create": (I, [U, U, U, I, ctypes.POINTER(P)]),
        "cairo_ctx_create_ex": (I, [U, U, U, I, I, ctypes.POINTER(P)]),
        "cairo_ctx_destroy": (I, [P]),
        "cairo_ctx_reset": (I, [P]),
        "cairo_ctx_submit": (I, [P, P, I, U, U, U, ctypes.POINTER(I)]),
        "cairo_ctx_wait": (I, [P, I, P]),
        "cairo_ctx_release": (I, [P, I]),
        "cairo_ctx_sync": (I, [P]),
        "cairo_ctx_stages": (I, [P]),
        "cairo_ctx_read_planes": (I, [P, I, P, P, P]),
        "cairo_ctx_read_inter": (I, [P, P, P]),
        "cairo_ctx_read_table": (I, [P, P]),
        "cairo_ctx_set_debug": (I, [P, I]),
        "cairo_ctx_read_predeblock": (I, [P, P, P, P]),
        "cairo_ctx_read_stamps": (I, [P, P]),
        "cairo_ctx_set_profiling": (I, [P, I]),
        "cairo_ctx_take_timings": (I, [P, P, ctypes.POINTER(I)]),
        "cairo_ctx_busy_intervals": (I, [P, P, I, ctypes.POINTER(I)]),
        "cairo_ctx_set_workgroups": (I, [P, I]),
        "cairo_ctx_set_batch": (I, [P, I]),
        "cairo_ctx_peer_info": (I, [P, I, P]),
        "cairo_ctx_join_group": (I, [P, I, I, P]),
        "cairo_group_check_queues": (I, [I, I]),
        "cairo_ctx_timeout_info": (I, [P, P, I]),
        "cairo_ctx_read_acct": (I, [P, P, I, I]),
        "cairo_peer_size": (I, []),
        "cairo_ctx_flush": (I, [P]),
        "cairo_ctx_set_helpers": (I, [P, I]),
        "cairo_ctx_max_workgroups": (I, [P]),
        "cairo_default_batch": (I, [U, U]),
        "cairo_task_order": (I, [I, I, P, ctypes.POINTER(I)]),
        "cairo_task_queues": (I, [I, I, I, I, I, P, P, ctypes.POINTER(I)]),
        "cairo_kat_transform": (I, [P, P, P, I, P, P, P, I]),
        "cairo_serialize_slice": (I, [P, U, U, U, P, P, P, P, U, ctypes.POINTER(U)]),
        "cairo_serialize_feed": (I, [P, ctypes.c_uint64, P, U, ctypes.POINTER(U)]),
        "cairo_precode_slice": (I, [P, U, U, U, P, P, P, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
        "cairo_ctx_set_outputs": (I, [P, I]),
        "cairo_ctx_fetch_coef": (I, [P, I, P]),
        "cairo_unserialize_slice": (I, [P, ctypes.POINTER(U), U, U, U, U, P, P, P, P]),
        "cairo_stream_create": (I, [P, I, ctypes.POINTER(P)]),
        "cairo_stream_submit": (I, [P, P, I, U, U, U, ctypes.POINTER(I)]),
        "cairo_stream_collect": (I, [P, I, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
        "cairo_stream_destroy": (I, [P]),
        "cairo_stream_timeline": (I, [P, I, P]),
        "cairo_stream_payload_bits": (I, [P, I, ctypes.POINTER(ctypes.c_uint64)]),
        "cairo_bits_append": (I, [P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), P, ctypes.c_uint64]),
        "evx_encoder_create": (I, [ctypes.POINTER(P)]),
        "evx_encoder_destroy": (I, [P]),
        "evx_encoder_clear": (I, [P]),
        "evx_encoder_insert_intra": (I, [P]),
        "evx_encoder_set_quality": (I, [P, ctypes.c_uint8]),
        "evx_encoder_encode": (I, [P, P, U, U, P]),
        "evx_encoder_set_ring": (I, [P, U]),
        "evx_encoder_peek": (I, [P, I, P]),
        "evx_encoder_set_device": (I, [P, I]),
        "evx_bitstream_create": (P, [U]),
        "evx_bitstream_destroy": (V, [P]),
        "evx_bitstream_data": (P, [P]),
        "evx_bitstream_occupancy": (U, [P]),
        "evx_bitstream_empty": (V, [P]),
        "evx_bitstream_write_bits": (I, [P, P, U]),
        "evx_decoder_create": (I, [ctypes.POINTER(P)]),
        "evx_decoder_destroy": (I, [P]),
        "evx_decoder_clear": (I, [P]),
        "evx_decoder_decode": (I, [P, P, P]),
        "evx_decoder_set_device": (I, [P, I]),
        "cairo_ctx_decode_frame": (I, [P, P, P, U, P]),
        "cairo_make_band4": (V, [P, U, U, U, U]),
        "cairo_version": (ctypes.c_char_p, []),
        "cairo_api_version": (I, []),
        "cairo_device_count": (I, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.cairo_api_version() != API_VERSION:
        raise ImportError(f"{LIB_PATH} has C ABI version {L.cairo_api_version()}, these bindings expect "
                          f"{API_VERSION} (include/cairo_amd.h CAIRO_AMD_API_VERSION): rebuild with `make`")
    _lib = L
    return L


def _ck(status: int, what: str) -> None:
    if status != EVX_SUCCESS:
        raise CairoError(what, status)


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _host_frame(rgb, width: int, height: int) -> int:
    """Address of a host RGB888 frame, after checking that it holds a whole
    width x height frame (the native side copies width*height*3 bytes from
    it asynchronously)."""
    if not isinstance(rgb, np.ndarray):
        raise TypeError("host frames are numpy arrays (pass on_device=True for a device address)")
    if rgb.dtype != np.uint8 or rgb.shape != (height, width, 3) or not rgb.flags["C_CONTIGUOUS"]:
        raise ValueError(f"frame must be a C-contiguous uint8 array of shape ({height}, {width}, 3), "
                         f"got {rgb.dtype} {rgb.shape}")
    return rgb.ctypes.data


def make_band4(w: int, h: int, t: int, seed: int = 1234) -> np.ndarray:
    """band4 synthetic RGB888 frame, shape (h, w, 3)."""
    out = np.empty((h, w, 3), np.uint8)
    lib().cairo_make_band4(_ptr(out), w, h, t, seed)
    return out


class _FrameResult(ctypes.Structure):
    _fields_ = [
        ("block_table", ctypes.c_void_p),
        ("coef_y", ctypes.c_void_p),
        ("coef_u", ctypes.c_void_p),
        ("coef_v", ctypes.c_void_p),
        ("wa", ctypes.c_uint32),
        ("ha", ctypes.c_uint32),
        ("wmb", ctypes.c_uint32),
        ("hmb", ctypes.c_uint32),
        ("index", ctypes.c_uint32),
        ("type", ctypes.c_uint32),
        ("quality", ctypes.c_uint32),
        ("feed", ctypes.c_void_p),
        ("feed_bits", ctypes.c_uint64),
        ("feed_status", ctypes.c_int32),
    ]


@dataclass
class FrameOutputs:
    """Host copies of one frame's outputs (block table + output_cache)."""

    table: np.ndarray  # (mbs,) BLOCK_DESC
    coef_y: np.ndarray | None  # None without OUT_COEF (Context.fetch_coef)
    coef_u: np.ndarray | None
    coef_v: np.ndarray | None
    feed: np.ndarray | None = None  # OUT_FEED: the GPU precode's feed words (uint32, LSB-first)
    feed_bits: int = 0
    feed_status: int = 0  # FEED_NONE / FEED_VALID / FEED_OVERFLOW


def _view(addr: int, dtype, count: int) -> np.ndarray:
    buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(addr)
    return np.frombuffer(buf, dtype=dtype, count=count)


class Context:
    """The encode-path backend (``cairo_ctx_*``): one encoder's device state."""

    def __init__(self, width: int, height: int, ring: int = 4, device: int = 0, stages: int = 96):
        self.L = lib()
        self.width, self.height, self.ring, self.device = width, height, ring, device
        self.wa, self.ha = (width + 15) & ~15, (height + 15) & ~15
        self.wmb, self.hmb = self.wa // 16, self.ha // 16
        p = ctypes.c_void_p()
        _ck(self.L.cairo_ctx_create_ex(width, height, ring, device, stages, ctypes.byref(p)), "cairo_ctx_create")
        self.h = p
        self._keep = {}  # ticket -> host RGB frame still being copied

    def close(self) -> None:
        if self.h:
            self.L.cairo_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stages(self) -> int:
        return int(self.L.cairo_ctx_stages(self.h))

    def submit(self, rgb, index: int, inter: bool, quality: int, on_device: bool = False) -> int:
        t = ctypes.c_int()
        ptr = rgb if on_device else _host_frame(rgb, self.width, self.height)
        _ck(
            self.L.cairo_ctx_submit(self.h, ptr, int(on_device), index, int(inter), quality, ctypes.byref(t)),
            "cairo_ctx_submit",
        )
        if not on_device:  # the H2D copy is asynchronous: keep the host frame alive
            self._keep[t.value] = rgb
        return t.value

    def wait(self, ticket: int, copy: bool = True) -> FrameOutputs:
        r = _FrameResult()
        st = self.L.cairo_ctx_wait(self.h, ticket, ctypes.byref(r))
        if st != EVX_SUCCESS:
            raise CairoError("cairo_ctx_wait", st, self.timeout_info() if st == EVX_ERROR_HARDWAREFAIL else None)
        self._keep.pop(ticket, None)
        return self._outputs(r, copy)

    ACCT_FIELDS = ("coder_tasks", "coder_total", "coder_group_wait", "coder_window", "coder_search", "coder_inter",
                   "coder_dequeue", "coder_mbs", "helper_tasks", "helper_total", "helper_wait", "helper_deblock",
                   "helper_search", "helper_catchup", "helper_dequeue", "helper_chunks",
                   "win_bytes", "win_spec_unused_bytes", "zero_mv_bytes", "gran_poll_bytes", "rec_poll_bytes",
                   "win_stages", "searched_tasks", "inter_tasks", "coder_xform", "coder_publish", "coder_drain",
                   "coder_vm0", "coder_records", "coder_prebarrier", "coder_store_tail",
                   "search_eval", "search_barrier", "search_select", "subpel_eval", "subpel_barrier",
                   "subpel_select", "db_inputs", "db_filter", "db_write")

    def read_acct(self, reset: bool = False) -> dict:
        """Engine time accounting (set_debug(32) on a CAIRO_ACCT=1 build): 10 ns
        ticks per role and phase summed over all tasks (kernels.h Acct)."""
        w = np.zeros(len(self.ACCT_FIELDS), np.uint64)
        _ck(self.L.cairo_ctx_read_acct(self.h, _ptr(w), len(w), int(reset)), "cairo_ctx_read_acct")
        return {k: int(w[i]) for i, k in enumerate(self.ACCT_FIELDS)}

    def timeout_info(self) -> dict | None:
        """The in-kernel wait that timed out first, as last reported
        (cairo_ctx_timeout_info): kind (WAIT_KINDS name), the waiting frame's
        epoch, index and MB row, the group member, what it needed, what it
        waited on, the last value seen; None if none since create / reset."""
        w = np.zeros(16, np.int32)
        _ck(self.L.cairo_ctx_timeout_info(self.h, _ptr(w), 16), "cairo_ctx_timeout_info")
        if not w[0]:
            return None
        d = {k: int(w[i]) for i, k in enumerate(TIMEOUT_FIELDS)}
        d["kind"] = WAIT_KINDS.get(d["kind"], str(d["kind"]))
        d["seen"] = (d.pop("seen_hi") & 0xFFFFFFFF) << 32 | (d.pop("seen_lo") & 0xFFFFFFFF)
        return d

    def _outputs(self, r, copy: bool) -> FrameOutputs:
        ny, nc = r.wa * r.ha, (r.wa // 2) * (r.ha // 2)
        mbs = r.wmb * r.hmb
        has_coef = bool(r.coef_y)
        feed = _view(r.feed, np.uint32, (r.feed_bits + 31) // 32) if r.feed_status == FEED_VALID else None
        out = FrameOutputs(
            _view(r.block_table, BLOCK_DESC, mbs),
            _view(r.coef_y, np.int16, ny).reshape(r.ha, r.wa) if has_coef else None,
            _view(r.coef_u, np.int16, nc).reshape(r.ha // 2, r.wa // 2) if has_coef else None,
            _view(r.coef_v, np.int16, nc).reshape(r.ha // 2, r.wa // 2) if has_coef else None,
            feed, int(r.feed_bits), int(r.feed_status),
        )
        if copy:
            cp = lambda a: None if a is None else a.copy()  # noqa: E731
            out = FrameOutputs(cp(out.table), cp(out.coef_y), cp(out.coef_u), cp(out.coef_v), cp(out.feed),
                               out.feed_bits, out.feed_status)
        return out

    def set_outputs(self, outputs: int) -> None:
        """OUT_COEF and/or OUT_FEED for frames submitted from now on."""
        _ck(self.L.cairo_ctx_set_outputs(self.h, outputs), "cairo_ctx_set_outputs")

    def fetch_coef(self, ticket: int):
        """(y, u, v) output_cache planes of a waited, unreleased frame (copies)."""
        r = _FrameResult()
        _ck(self.L.cairo_ctx_fetch_coef(self.h, ticket, ctypes.byref(r)), "cairo_ctx_fetch_coef")
        ny, nc = self.wa * self.ha, (self.wa // 2) * (self.ha // 2)
        return (_view(r.coef_y, np.int16, ny).reshape(self.ha, self.wa).copy(),
                _view(r.coef_u, np.int16, nc).reshape(self.ha // 2, self.wa // 2).copy(),
                _view(r.coef_v, np.int16, nc).reshape(self.ha // 2, self.wa // 2).copy())

    def release(self, ticket: int) -> None:
        _ck(self.L.cairo_ctx_release(self.h, ticket), "cairo_ctx_release")

    def encode_frame(self, rgb, index: int, inter: bool, quality: int, on_device: bool = False) -> FrameOutputs:
        t = self.submit(rgb, index, inter, quality, on_device)
        try:
            return self.wait(t, copy=True)
        finally:
            self.release(t)

    def sync(self) -> None:
        _ck(self.L.cairo_ctx_sync(self.h), "cairo_ctx_sync")

    def reset(self) -> None:
        """Fresh-encoder state (cairo_ctx_reset): planes zeroed, tickets from 0,
        any group left (its members reset and rejoin together)."""
        _ck(self.L.cairo_ctx_reset(self.h), "cairo_ctx_reset")
        self._keep.clear()

    def read_planes(self, which: int):
        """which: 0 input, 1 output_cache, 2+k ring slot k -> (y, u, v)."""
        y = np.empty((self.ha, self.wa), np.int16)
        u = np.empty((self.ha // 2, self.wa // 2), np.int16)
        v = np.empty_like(u)
        _ck(self.L.cairo_ctx_read_planes(self.h, which, _ptr(y), _ptr(u), _ptr(v)), "read_planes")
        return y, u, v

    def read_inter(self):
        n = self.wmb * self.hmb * max(self.ring - 1, 0)
        d = np.zeros(n, BLOCK_DESC)
        s = np.zeros(n, np.int32)
        if n:
            _ck(self.L.cairo_ctx_read_inter(self.h, _ptr(d), _ptr(s)), "read_inter")
        return d, s

    def read_table(self):
        t = np.zeros(self.wmb * self.hmb, BLOCK_DESC)
        _ck(self.L.cairo_ctx_read_table(self.h, _ptr(t)), "read_table")
        return t

    def set_debug(self, flags: int) -> None:
        _ck(self.L.cairo_ctx_set_debug(self.h, flags), "set_debug")

    def read_predeblock(self):
        y = np.empty((self.ha, self.wa), np.int16)
        u = np.empty((self.ha // 2, self.wa // 2), np.int16)
        v = np.empty_like(u)
        _ck(self.L.cairo_ctx_read_predeblock(self.h, _ptr(y), _ptr(u), _ptr(v)), "read_predeblock")
        return y, u, v

    def read_stamps(self):
        """-> (per-MB stamps (MAX_BATCH, hmb, wmb, 12), per-row deblock chunk stamps (MAX_BATCH, hmb, 256),
        engine [entry, exit], inter-task stamps (MAX_BATCH, hmb, ng, 12): dequeue, ready,
        done, zero-MV checked, window staged, level-2 wait start / end, level-2
        count, step 16 done, integer steps done, sub-pel done) for the frames of the last batch; 100 MHz ticks."""
        n_mb, n_db = self.hmb * self.wmb * 12, self.hmb * 256
        fw = n_mb + n_db
        ng = (self.wmb + 3) // 4
        n_it = MAX_BATCH * self.hmb * ng * 12
        out = np.zeros(MAX_BATCH * fw + 2 + n_it, np.uint64)
        _ck(self.L.cairo_ctx_read_stamps(self.h, _ptr(out)), "read_stamps")
        fr = out[: MAX_BATCH * fw].reshape(MAX_BATCH, fw)
        return (fr[:, :n_mb].reshape(MAX_BATCH, self.hmb, self.wmb, 12), fr[:, n_mb:].reshape(MAX_BATCH, self.hmb, 256),
                out[MAX_BATCH * fw:MAX_BATCH * fw + 2], out[MAX_BATCH * fw + 2:].reshape(MAX_BATCH, self.hmb, ng, 12))

    def set_profiling(self, enable: bool) -> None:
        _ck(self.L.cairo_ctx_set_profiling(self.h, int(enable)), "set_profiling")

    def take_timings(self):
        """-> ([convert ms, 0, engine ms summed over launches, engine busy ms
        (union of the launch intervals)], frames) since the last call."""
        ms = (ctypes.c_double * 4)()
        n = ctypes.c_int()
        _ck(self.L.cairo_ctx_take_timings(self.h, ms, ctypes.byref(n)), "take_timings")
        return list(ms), n.value

    def busy_intervals(self) -> np.ndarray:
        """(n, 2) engine launch [start, end) ms since profiling started, not reset."""
        n = ctypes.c_int()
        _ck(self.L.cairo_ctx_busy_intervals(self.h, None, 0, ctypes.byref(n)), "busy_intervals")
        out = np.zeros((max(n.value, 1), 2), np.float64)
        _ck(self.L.cairo_ctx_busy_intervals(self.h, _ptr(out), n.value, ctypes.byref(n)), "busy_intervals")
        return out[: n.value]

    def set_batch(self, frames: int) -> None:
        _ck(self.L.cairo_ctx_set_batch(self.h, frames), "set_batch")

    def set_workgroups(self, rows: int = 0) -> None:
        _ck(self.L.cairo_ctx_set_workgroups(self.h, rows), "set_workgroups")

    def set_helpers(self, helpers: int = 0) -> None:
        _ck(self.L.cairo_ctx_set_helpers(self.h, helpers), "set_helpers")

    def max_workgroups(self) -> int:
        return int(self.L.cairo_ctx_max_workgroups(self.h))

    def flush(self) -> None:
        _ck(self.L.cairo_ctx_flush(self.h), "cairo_ctx_flush")

    # ---- frame-interleaved groups (include/cairo_amd.h) ----
    def peer_info(self, cross_device: bool = False) -> bytes:
        """This member's cairo_peer record (plain bytes, to exchange)."""
        rec = (ctypes.c_uint8 * PEER_SIZE)()
        _ck(self.L.cairo_ctx_peer_info(self.h, int(cross_device), rec), "cairo_ctx_peer_info")
        return bytes(rec)

    def join_group(self, rank: int, peers: list) -> None:
        """Join the group of len(peers) members as `rank` (records in rank order)."""
        buf = b"".join(peers)
        assert len(buf) == PEER_SIZE * len(peers)
        arr = (ctypes.c_uint8 * len(buf)).from_buffer_copy(buf)
        _ck(self.L.cairo_ctx_join_group(self.h, len(peers), rank, arr), "cairo_ctx_join_group")


MIRROR_SLOTS = 16  # kMirrorSlots (backend.hip): reconstruction slots of a member over devices / processes


def group_layout(n: int, size: int, ring: int, stages: int, mirror: bool = False) -> dict:
    """Where frame n of a frame-interleaved group of `size` members lives
    (backend.hip frame_links): its member, that member's ticket, staging
    slot and reconstruction slot, and whether it reconstructs in place over
    frame n - ring (the reference's ring reuse, common.cpp:192-195).  mirror:
    members on other devices or processes, whose rings all share one layout
    (slot (n % N) * S + (n / N) % S: the producer's own block, a mirror block
    on every other member); `readers` are the members its deblock pushes it
    to (the frames n+1..n+R-1 reference it, n+R reads its stale rows)."""
    slots = -(-ring // size)  # S = ceil(R / N) reconstruction slots per member (per block when mirrored)
    t = n // size
    slot = (n % size) * slots + t % slots if mirror else t % slots
    readers = []
    if mirror:
        for d in range(1, ring + 1):
            j = (n + d) % size
            if j != n % size and j not in readers:
                readers.append(j)
    return {"member": n % size, "ticket": t, "staging_slot": t % stages, "recon_slot": slot,
            "recon_slots": slots * size if mirror else slots, "in_place": size * slots == ring, "readers": readers}


class Group:
    """A frame-interleaved group of member contexts in this process (one per
    device, or several on one device) encoding ONE stream: frame n goes to
    member n % N (include/cairo_amd.h).  Processes that each own
    one member exchange Context.peer_info() records themselves."""

    def __init__(self, width: int, height: int, ring: int, devices, stages: int = 64, batch: int = 0):
        self.members = [Context(width, height, ring, device=d, stages=stages) for d in devices]
        n = len(self.members)
        per_dev = {d: list(devices).count(d) for d in devices}
        cross = len(per_dev) > 1
        for m, d in zip(self.members, devices):
            if batch:
                m.set_batch(batch)
            if per_dev[d] > 1:  # members on one device share its workgroup slots
                m.set_workgroups(max(1, m.max_workgroups() // per_dev[d]))
        self.cross = cross
        self._join()
        self.size, self.ring, self.stages = n, ring, stages
        self.tickets = {}

    def _join(self) -> None:
        recs = [m.peer_info(cross_device=self.cross) for m in self.members]
        for r, m in enumerate(self.members):
            m.join_group(r, recs)

    def reset(self) -> None:
        """Every member back to the fresh-encoder state and the group rejoined
        (cairo_ctx_reset leaves it): the next frame is frame 0 of a new stream."""
        for m in self.members:
            m.reset()
        self._join()
        self.tickets = {}

    def submit(self, rgb, index: int, inter: bool, quality: int, on_device: bool = False) -> None:
        m = self.members[index % self.size]
        self.tickets[index] = m.submit(rgb, index, inter, quality, on_device)

    def wait(self, index: int, copy: bool = True) -> FrameOutputs:
        """Outputs of frame `index`; launches every member's pending frames first
        (the frame may depend on any earlier frame of the stream)."""
        for m in self.members:
            m.flush()
        return self.members[index % self.size].wait(self.tickets[index], copy)

    def release(self, index: int) -> None:
        self.members[index % self.size].release(self.tickets.pop(index))

    def recon(self, n: int):
        """Frame n's deblocked reconstruction (y, u, v), while still held."""
        lay = group_layout(n, self.size, self.ring, self.stages, mirror=self.cross)
        return self.members[lay["member"]].read_planes(2 + lay["recon_slot"])

    def close(self) -> None:
        for m in self.members:
            m.close()


def default_batch(width: int, height: int) -> int:
    """Frames per engine launch the library uses by default for this frame size."""
    return int(lib().cairo_default_batch(width, height))


def task_order(hmb: int, frames: int):
    """-> (the engine's task order of a launch: int32 (frame << 16 | row) per
    task, the order slope)."""
    out = np.zeros(frames * hmb, np.int32)
    slope = ctypes.c_int()
    _ck(lib().cairo_task_order(hmb, frames, _ptr(out), ctypes.byref(slope)), "cairo_task_order")
    return out, slope.value


def task_queues(hmb: int, frames: int, helpers: int = 192, rows: int = 192, pool: int = 0):
    """-> (one pool's tasks (0 helpers, 1 row coders) of a launch with
    `helpers` + `rows` workers, partitioned into per-label queues: int32
    (frame << 16 | row), the 9 segment bounds, the number of labels) -- the
    layout the engine's launch uses (backend.hip banded_pool)."""
    out = np.zeros(frames * hmb, np.int32)
    seg = np.zeros(9, np.int32)
    nlab = ctypes.c_int()
    _ck(lib().cairo_task_queues(hmb, frames, helpers, rows, pool, _ptr(out), _ptr(seg), ctypes.byref(nlab)),
        "cairo_task_queues")
    return out, seg, nlab.value


def serialize_slice(table: np.ndarray, wmb: int, hmb: int, ring: int, cy, cu, cv, capacity_bytes: int | None = None):
    """Host entropy stage on explicit inputs -> (bytes, nbits)."""
    cap = capacity_bytes or (cy.size * 4 + 65536)
    out = np.zeros(cap, np.uint8)  # bits past the payload's end are left as they are: zeros
    pos = ctypes.c_uint32(0)
    t = np.ascontiguousarray(table).view(np.uint8)
    cy, cu, cv = (np.ascontiguousarray(a, dtype=np.int16) for a in (cy, cu, cv))
    _ck(
        lib().cairo_serialize_slice(_ptr(t), wmb, hmb, ring, _ptr(cy), _ptr(cu), _ptr(cv), _ptr(out), cap, ctypes.byref(pos)),
        "cairo_serialize_slice",
    )
    n = pos.value
    return out[: (n + 7) // 8].tobytes(), n


def serialize_feed(feed: np.ndarray, feed_bits: int, capacity_bytes: int | None = None):
    """The arithmetic coder over a GPU-precoded feed (FrameOutputs.feed) -> (bytes, nbits)."""
    cap = capacity_bytes or (feed_bits // 8 * 2 + 65536)
    out = np.zeros(cap, np.uint8)
    pos = ctypes.c_uint32(0)
    f = np.ascontiguousarray(feed, dtype=np.uint32)
    _ck(lib().cairo_serialize_feed(_ptr(f), feed_bits, _ptr(out), cap, ctypes.byref(pos)), "cairo_serialize_feed")
    return out[: (pos.value + 7) // 8].tobytes(), pos.value


def precode_slice(table: np.ndarray, wmb: int, hmb: int, ring: int, cy, cu, cv):
    """The host precode alone -> (feed words uint32, feed bits): what the GPU
    precode hands over for a FEED_VALID frame."""
    t = np.ascontiguousarray(table).view(np.uint8)
    cy, cu, cv = (np.ascontiguousarray(a, dtype=np.int16) for a in (cy, cu, cv))
    nb = ctypes.c_uint64(0)
    L = lib()
    L.cairo_precode_slice(_ptr(t), wmb, hmb, ring, _ptr(cy), _ptr(cu), _ptr(cv), None, 0, ctypes.byref(nb))
    out = np.zeros((nb.value + 31) // 32 + 1, np.uint32)
    _ck(L.cairo_precode_slice(_ptr(t), wmb, hmb, ring, _ptr(cy), _ptr(cu), _ptr(cv), _ptr(out), out.size,
                              ctypes.byref(nb)), "cairo_precode_slice")
    return out[: (nb.value + 31) // 32], nb.value


def unserialize_slice(payload: bytes, nbits: int, wmb: int, hmb: int, ring: int, table=None, planes=None,
                      start: int = 0):
    """Host entropy decode of one frame's payload (bits [start, nbits) of
    payload) into a persistent (table, (y, u, v)) state (zeros when None) ->
    (table, planes, bits consumed)."""
    if table is None:
        table = np.zeros(wmb * hmb, BLOCK_DESC)
    if planes is None:
        planes = (np.zeros((hmb * 16, wmb * 16), np.int16), np.zeros((hmb * 8, wmb * 8), np.int16),
                  np.zeros((hmb * 8, wmb * 8), np.int16))
    buf = np.frombuffer(payload, np.uint8) if len(payload) else np.zeros(1, np.uint8)
    rd = ctypes.c_uint32(start)
    _ck(lib().cairo_unserialize_slice(_ptr(np.ascontiguousarray(buf)), ctypes.byref(rd), nbits, wmb, hmb, ring,
                                      _ptr(table), *(_ptr(p) for p in planes)), "cairo_unserialize_slice")
    return table, planes, rd.value - start


def bits_append(dst: np.ndarray, pos: int, src: bytes, nbits: int) -> int:
    """Append nbits of src (LSB-first) at bit pos of the uint8 array dst -> new pos."""
    p = ctypes.c_uint64(pos)
    s = np.frombuffer(src, np.uint8) if len(src) else np.zeros(1, np.uint8)
    _ck(lib().cairo_bits_append(_ptr(dst), dst.size * 8, ctypes.byref(p), _ptr(s), nbits), "cairo_bits_append")
    return p.value


class Stream:
    """Frame pipeline (``cairo_stream_*``): GPU hot path + host entropy on
    native worker threads.  Drives ``ctx`` exclusively while open."""

    def __init__(self, ctx: "Context", threads: int = 0):
        self.L = lib()
        self.ctx = ctx
        p = ctypes.c_void_p()
        _ck(self.L.cairo_stream_create(ctx.h, threads, ctypes.byref(p)), "cairo_stream_create")
        self.h = p
        self._keep = {}

    def submit(self, rgb, index: int, inter: bool, quality: int, on_device: bool = False) -> int:
        t = ctypes.c_int()
        ptr = rgb if on_device else _host_frame(rgb, self.ctx.width, self.ctx.height)
        _ck(self.L.cairo_stream_submit(self.h, ptr, int(on_device), index, int(inter), quality, ctypes.byref(t)),
            "cairo_stream_submit")
        if not on_device:
            self._keep[t.value] = rgb
        return t.value

    def collect(self, ticket: int, out: np.ndarray | None = None, pos: int = 0):
        """Append the frame's payload at bit pos of out -> new pos; with out
        None, return (bytes, nbits) of the payload alone."""
        if out is None:
            p = ctypes.c_uint64(0)
            _ck(self.L.cairo_stream_payload_bits(self.h, ticket, ctypes.byref(p)), "cairo_stream_payload_bits")
            buf = np.zeros(p.value // 8 + 8, np.uint8)
            p = ctypes.c_uint64(0)
            _ck(self.L.cairo_stream_collect(self.h, ticket, _ptr(buf), buf.size, ctypes.byref(p)),
                "cairo_stream_collect")
            self._keep.pop(ticket, None)
            return buf[: (p.value + 7) // 8].tobytes(), p.value
        p = ctypes.c_uint64(pos)
        _ck(self.L.cairo_stream_collect(self.h, ticket, _ptr(out), out.size, ctypes.byref(p)), "cairo_stream_collect")
        self._keep.pop(ticket, None)
        return p.value

    def payload_bits(self, ticket: int) -> int:
        """The frame's payload length in bits (waits for its entropy stage)."""
        p = ctypes.c_uint64(0)
        _ck(self.L.cairo_stream_payload_bits(self.h, ticket, ctypes.byref(p)), "cairo_stream_payload_bits")
        return p.value

    def timeline(self, ticket: int):
        """(submitted, outputs on host, entropy start, entropy end, collected), us."""
        t = (ctypes.c_double * 5)()
        _ck(self.L.cairo_stream_timeline(self.h, ticket, t), "cairo_stream_timeline")
        return list(t)

    def close(self) -> None:
        if self.h:
            r = self.L.cairo_stream_destroy(self.h)
            self.h = None
            self._keep.clear()
            _ck(r, "cairo_stream_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BitStream:
    """evx::bit_stream owned from Python."""

    def __init__(self, size_bits: int):
        self.L = lib()
        self.h = self.L.evx_bitstream_create(size_bits)
        if not self.h:
            raise MemoryError("evx_bitstream_create")

    def bits(self) -> int:
        return self.L.evx_bitstream_occupancy(self.h)

    def write(self, data: bytes, nbits: int | None = None) -> None:
        """Append nbits (default: all) of data, LSB-first."""
        n = len(data) * 8 if nbits is None else nbits
        buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        _ck(self.L.evx_bitstream_write_bits(self.h, _ptr(np.ascontiguousarray(buf)), n), "write_bits")

    def data(self) -> bytes:
        n = (self.bits() + 7) // 8
        return ctypes.string_at(self.L.evx_bitstream_data(self.h), n) if n else b""

    def empty(self) -> None:
        self.L.evx_bitstream_empty(self.h)

    def __del__(self):
        try:
            if self.h:
                self.L.evx_bitstream_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Encoder:
    """The drop-in evx1_encoder (reference evx1.h:66-94) through its C view."""

    def __init__(self, ring: int = 4, device: int = 0):
        self.L = lib()
        p = ctypes.c_void_p()
        _ck(self.L.evx_encoder_create(ctypes.byref(p)), "create_encoder")
        self.h = p
        if ring != 4:
            _ck(self.L.evx_encoder_set_ring(self.h, ring), "set_ring")
        if device:
            _ck(self.L.evx_encoder_set_device(self.h, device), "set_device")

    def set_quality(self, q: int) -> None:
        _ck(self.L.evx_encoder_set_quality(self.h, q), "set_quality")

    def insert_intra(self) -> None:
        _ck(self.L.evx_encoder_insert_intra(self.h), "insert_intra")

    def clear(self) -> None:
        _ck(self.L.evx_encoder_clear(self.h), "clear")

    def encode(self, rgb: np.ndarray, bs: BitStream) -> None:
        if rgb.ndim != 3 or rgb.shape[2] != 3:
            raise ValueError(f"frame must have shape (height, width, 3), got {rgb.shape}")
        h, w = rgb.shape[:2]
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8) if rgb.dtype == np.uint8 else None
        if rgb is None:
            raise ValueError("frame must be uint8 RGB888")
        _ck(self.L.evx_encoder_encode(self.h, _ptr(rgb), w, h, bs.h), "encode")
        self._shape = (w, h)

    def peek(self, state: int, width: int, height: int) -> np.ndarray:
        """Debug view of the last encoded frame (EVX_PEEK_*, evx1.h) -> RGB (h, w, 3)."""
        # the native peek writes the encoder's frame size: refuse a smaller view
        if getattr(self, "_shape", None) != (width, height):
            raise ValueError(f"peek size {width}x{height} differs from the last encoded frame "
                             f"{getattr(self, '_shape', None)}")
        out = np.zeros((height, width, 3), np.uint8)
        _ck(self.L.evx_encoder_peek(self.h, state, _ptr(out)), "peek")
        return out

    def close(self) -> None:
        if self.h:
            self.L.evx_encoder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Decoder:
    """The drop-in evx1_decoder (reference evx1.h:97-112) through its C view."""

    def __init__(self, device: int = 0):
        self.L = lib()
        p = ctypes.c_void_p()
        _ck(self.L.evx_decoder_create(ctypes.byref(p)), "create_decoder")
        self.h = p
        if device:
            _ck(self.L.evx_decoder_set_device(self.h, device), "set_device")

    def decode(self, bs: "BitStream", width: int, height: int) -> np.ndarray:
        """Decode [header +] one frame record of bs (emptied afterwards) -> RGB (h, w, 3)."""
        out = np.zeros((height, width, 3), np.uint8)
        _ck(self.L.evx_decoder_decode(self.h, bs.h, _ptr(out)), "decode")
        return out

    def clear(self) -> None:
        _ck(self.L.evx_decoder_clear(self.h), "clear")

    def close(self) -> None:
        if self.h:
            self.L.evx_decoder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def yuv_to_rgb(y: np.ndarray, u: np.ndarray, v: np.ndarray, width: int, height: int) -> np.ndarray:
    """convert_image YUV -> RGB (reference convert.cpp:16-19, 162-223), numpy
    restatement for tests: saturate narrows to int16, then clips to 0..255."""
    yy = y[:height, :width].astype(np.int32) - 16
    uu = np.repeat(np.repeat(u.astype(np.int32) - 128, 2, 0), 2, 1)[:height, :width]
    vv = np.repeat(np.repeat(v.astype(np.int32) - 128, 2, 0), 2, 1)[:height, :width]

    def sat(x):
        x = ((x + 32768) & 0xFFFF) - 32768
        return np.clip(x, 0, 255).astype(np.uint8)

    return np.stack([sat((256 * yy + 358 * vv + 128) >> 8),
                     sat((256 * yy - 88 * uu - 182 * vv + 128) >> 8),
                     sat((256 * yy + 452 * uu + 128) >> 8)], axis=-1)


def device_count() -> int:
    return lib().cairo_device_count()
