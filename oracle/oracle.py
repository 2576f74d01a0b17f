"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes view of liboracle.so, the plain-C CPU restatement of the reference
EVX-1 encoder (oracle/evx_oracle.c).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module, and only as the
checker / CPU baseline.  The product (cairo_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
FNV_OFFSET = 0xCBF29CE484222325

# evx_block_desc (reference common.h:78-95, pack(2), 16 bytes)
BLOCK_DESC = np.dtype(
    [("block_type", "<u4"), ("prediction_target", "u1"), ("pad", "u1"), ("motion_x", "<i2"),
     ("motion_y", "<i2"), ("sp_pred", "u1"), ("sp_amount", "u1"), ("sp_index", "u1"),
     ("q_index", "u1"), ("variance", "<i2")]
)

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make oracle/liboracle.so`")
        L = ctypes.CDLL(LIB_PATH)
        P, I, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32
        L.orc_create.restype = P
        L.orc_create.argtypes = [I]
        L.orc_destroy.argtypes = [P]
        L.orc_clear.argtypes = [P]
        L.orc_insert_intra.argtypes = [P]
        L.orc_set_quality.argtypes = [P, I]
        L.orc_encode.restype = I
        L.orc_encode.argtypes = [P, P, I, I, P, U, ctypes.POINTER(U)]
        for n in ("orc_plane",):
            getattr(L, n).restype = P
            getattr(L, n).argtypes = [P, I, I]
        L.orc_predeblock_plane.restype = P
        L.orc_predeblock_plane.argtypes = [P, I]
        for n in ("orc_block_table", "orc_inter_descs", "orc_inter_sads"):
            getattr(L, n).restype = P
            getattr(L, n).argtypes = [P]
        L.orc_dims.restype = I
        L.orc_dims.argtypes = [P] + [ctypes.POINTER(I)] * 4
        L.orc_make_frame.argtypes = [P, I, I, U, U]
        L.orc_fnv1a64.restype = ctypes.c_uint64
        L.orc_fnv1a64.argtypes = [ctypes.c_uint64, P, ctypes.c_uint64]
        L.orc_abac_feed.restype = U
        L.orc_abac_feed.argtypes = [P, ctypes.c_uint64, P, U, ctypes.POINTER(I)]
        L.orc_transform_8x8.argtypes = [P, I, P, I]
        L.orc_sub_transform_8x8.argtypes = [P, I, P, I, P, I]
        L.orc_inverse_transform_8x8.argtypes = [P, I, P, I]
        L.orc_inverse_transform_add_8x8.argtypes = [P, I, P, I, P, I]
        L.orc_variance2.restype = ctypes.c_int32
        L.orc_variance2.argtypes = [P, I]
        L.orc_vaq.restype = ctypes.c_uint8
        L.orc_vaq.argtypes = [ctypes.c_uint8, P, I]
        L.orc_quantize_mb.argtypes = [ctypes.c_uint8, I, P, P, P, P, P, P]
        L.orc_dequantize_mb.argtypes = [ctypes.c_uint8, I, P, P, P, P, P, P]
        L.orc_deblock.argtypes = [P, P, P, P, I, I]
        L.orc_convert_rgb.argtypes = [P, I, I, P, P, P, I, I]
        L.orc_op_counts.argtypes = [P, I]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def make_frame(w: int, h: int, t: int, seed: int = 1234) -> np.ndarray:
    out = np.empty((h, w, 3), np.uint8)
    lib().orc_make_frame(_ptr(out), w, h, t, seed)
    return out


def fnv1a64(data: bytes, h: int = FNV_OFFSET) -> int:
    buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    return lib().orc_fnv1a64(h, _ptr(np.ascontiguousarray(buf)), len(data))


PIXEL_OPS_PER_CALL = (256, 384, 256, 384)  # SAD, MAD, zero-SAD, lerp


def op_counts(reset: bool = False) -> dict:
    """Oracle work since the last reset: helper calls and the algorithmic
    pixel-op total (one abs-difference, max or lerp per pixel)."""
    out = np.zeros(4, np.uint64)
    lib().orc_op_counts(_ptr(out), int(reset))
    calls = [int(x) for x in out]
    return {"sad": calls[0], "mad": calls[1], "sad0": calls[2], "lerp": calls[3],
            "pixel_ops": sum(c * k for c, k in zip(calls, PIXEL_OPS_PER_CALL))}


def canonical_frame_bytes(data: bytes, nbits: int, first: bool) -> bytes:
    """Mask a frame's bytes for comparison: tail bits beyond nbits zeroed,
    header byte 7 (an unwritten pad in the reference, common.h:50-62) zeroed."""
    b = bytearray(data[: (nbits + 7) // 8])
    if nbits % 8:
        b[-1] &= (1 << (nbits % 8)) - 1
    if first and len(b) > 7:
        b[7] = 0
    return bytes(b)


class OracleEncoder:
    def __init__(self, ring: int = 4):
        self.L = lib()
        self.h = self.L.orc_create(ring)
        self.ring = ring
        self.first = True

    def __del__(self):
        try:
            if self.h:
                self.L.orc_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def set_quality(self, q: int) -> None:
        self.L.orc_set_quality(self.h, q)

    def insert_intra(self) -> None:
        self.L.orc_insert_intra(self.h)

    def encode(self, rgb: np.ndarray):
        """Encode one frame into a fresh buffer -> (bytes, nbits)."""
        h, w = rgb.shape[:2]
        cap = w * h * 8 + 4096
        out = np.zeros(cap, np.uint8)
        pos = ctypes.c_uint32(0)
        st = self.L.orc_encode(self.h, _ptr(np.ascontiguousarray(rgb)), w, h, _ptr(out), cap, ctypes.byref(pos))
        if st:
            raise RuntimeError(f"oracle encode failed: {st}")
        self.first = False
        return out[: (pos.value + 7) // 8].tobytes(), pos.value

    def dims(self):
        a = [ctypes.c_int() for _ in range(4)]
        self.L.orc_dims(self.h, *[ctypes.byref(x) for x in a])
        return tuple(x.value for x in a)  # wa, ha, ring, index

    def _plane(self, addr: int, shape):
        n = shape[0] * shape[1]
        buf = (ctypes.c_int16 * n).from_address(addr)
        return np.frombuffer(buf, np.int16, n).reshape(shape).copy()

    def planes(self, which: int):
        """which: 0 input, 1 output_cache, 2+k ring slot k -> (y, u, v) copies."""
        wa, ha, _, _ = self.dims()
        return tuple(
            self._plane(self.L.orc_plane(self.h, which, p), (ha, wa) if p == 0 else (ha // 2, wa // 2))
            for p in range(3)
        )

    def predeblock(self):
        wa, ha, _, _ = self.dims()
        return tuple(
            self._plane(self.L.orc_predeblock_plane(self.h, p), (ha, wa) if p == 0 else (ha // 2, wa // 2))
            for p in range(3)
        )

    def block_table(self) -> np.ndarray:
        wa, ha, _, _ = self.dims()
        n = (wa // 16) * (ha // 16)
        raw = ctypes.string_at(self.L.orc_block_table(self.h), n * 16)
        return np.frombuffer(raw, BLOCK_DESC).copy()

    def inter_records(self):
        wa, ha, ring, _ = self.dims()
        n = (wa // 16) * (ha // 16) * max(ring - 1, 0)
        d = np.frombuffer(ctypes.string_at(self.L.orc_inter_descs(self.h), n * 16), BLOCK_DESC).copy()
        s = np.frombuffer(ctypes.string_at(self.L.orc_inter_sads(self.h), n * 4), np.int32).copy()
        return d, s


def abac_feed(words: np.ndarray, nbits: int) -> tuple[bytes, int]:
    """The reference coder (abac.cpp) alone over a raw LSB-first feed -> (bytes, bits)."""
    w = np.ascontiguousarray(words, dtype=np.uint32)
    cap = nbits * 2 + 4096
    out = np.zeros(cap // 8 + 8, np.uint8)
    err = ctypes.c_int(0)
    n = lib().orc_abac_feed(_ptr(w), nbits, _ptr(out), cap, ctypes.byref(err))
    assert not err.value
    return out[: (n + 7) // 8].tobytes(), int(n)
