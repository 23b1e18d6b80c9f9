"""TEST INFRASTRUCTURE ONLY -- ctypes/numpy front-end of the C restatement
``oracle/inccl_oracle.c``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product package
``container_inc_amd`` never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc.so")

PAYLOAD_COUNT = 1024   # api.h:40
LANES = 256            # nts.c:55
SW_SLOTS = 16          # nts.c:22
SW_ABSORBED, SW_BROADCAST, SW_REPLAY, SW_DROPPED, SW_ACK, SW_IGNORED, SW_INVALID, SW_FORWARD, SW_DOWN = range(9)
SW_WIRE_ORDER, SW_RECYCLE = 1, 2   # non-root flags (orc_switch_init_nonroot)
FRAME_ROW = 1152       # an output row of orc_switch_pipeline (the longest frame is 1098 B)

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        sz = ctypes.c_size_t
        L.orc_encode_be32.argtypes = [P, P, sz]
        L.orc_decode_be32.argtypes = [P, P, sz]
        L.orc_quantise_one.argtypes = [ctypes.c_float, ctypes.c_int]
        L.orc_quantise_one.restype = ctypes.c_int32
        L.orc_quantise_f32.argtypes = [P, P, sz, ctypes.c_int]
        L.orc_dequantise_one.argtypes = [ctypes.c_int32, ctypes.c_int]
        L.orc_dequantise_one.restype = ctypes.c_float
        L.orc_dequantise_q32.argtypes = [P, P, sz, ctypes.c_int]
        L.orc_sum_q32.argtypes = [P, ctypes.c_int, P, sz]
        L.orc_reduce_f32.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_quant_sum.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_absmax_f32.argtypes = [P, ctypes.c_int, sz]
        L.orc_absmax_f32.restype = ctypes.c_float
        L.orc_bf16_to_f32.argtypes = [ctypes.c_uint16]
        L.orc_bf16_to_f32.restype = ctypes.c_float
        L.orc_f32_to_bf16.argtypes = [ctypes.c_float]
        L.orc_f32_to_bf16.restype = ctypes.c_uint16
        L.orc_reduce_bf16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_quant_sum_bf16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_sum_dequant_bf16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_absmax_bf16.argtypes = [P, ctypes.c_int, sz]
        L.orc_absmax_bf16.restype = ctypes.c_float
        L.orc_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.orc_f16_to_f32.restype = ctypes.c_float
        L.orc_f32_to_f16.argtypes = [ctypes.c_float]
        L.orc_f32_to_f16.restype = ctypes.c_uint16
        L.orc_f16_to_f32_n.argtypes = [P, P, sz]
        L.orc_f32_to_f16_n.argtypes = [P, P, sz]
        L.orc_reduce_f16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_quant_sum_f16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_sum_dequant_f16.argtypes = [P, ctypes.c_int, P, sz, ctypes.c_int]
        L.orc_absmax_f16.argtypes = [P, ctypes.c_int, sz]
        L.orc_absmax_f16.restype = ctypes.c_float
        L.orc_choose_scale.argtypes = [ctypes.c_float, ctypes.c_int]
        L.orc_choose_scale.restype = ctypes.c_int
        L.orc_checksum_q32.argtypes = [P, sz, ctypes.c_uint64]
        L.orc_checksum_q32.restype = ctypes.c_uint32
        L.orc_switch_init.argtypes = [P, ctypes.c_int]
        L.orc_switch_bytes.argtypes = []
        L.orc_switch_bytes.restype = sz
        L.orc_switch_init_ring.argtypes = [P, ctypes.c_int, ctypes.c_uint32]
        L.orc_switch_init_ring.restype = ctypes.c_int
        L.orc_switch_init_nonroot.argtypes = [P, ctypes.c_int, ctypes.c_uint32, ctypes.c_int]
        L.orc_switch_init_nonroot.restype = ctypes.c_int
        L.orc_switch_slot.argtypes = [P, ctypes.c_uint32]
        L.orc_switch_slot.restype = P
        L.orc_switch_pipeline.argtypes = [P, P, ctypes.c_int, P, sz, P, sz, P]
        L.orc_switch_pipeline.restype = ctypes.c_int
        L.orc_build_ack_frame.argtypes = [P, P, ctypes.c_uint32]
        L.orc_build_ack_frame.restype = sz
        L.orc_switch_ingress.argtypes = [P, ctypes.c_int, ctypes.c_uint32, P, P]
        L.orc_switch_ingress.restype = ctypes.c_int
        L.orc_crc32.argtypes = [P, sz]
        L.orc_crc32.restype = ctypes.c_uint32
        L.orc_icrc.argtypes = [P]
        L.orc_icrc.restype = ctypes.c_uint32
        L.orc_build_data_frame.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, P]
        L.orc_build_data_frame.restype = sz
        L.orc_allreduce_write_loopback.argtypes = [ctypes.c_int, P, ctypes.c_uint32, P, ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        L.orc_allreduce_write_loopback.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


# ---- wire codec (api.c:300-302, :428-430) ----
def encode_be32(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.int32)
    out = np.empty(x.shape, np.uint32)
    lib().orc_encode_be32(_p(x), _p(out), x.size)
    return out


def decode_be32(w: np.ndarray) -> np.ndarray:
    w = np.ascontiguousarray(w, dtype=np.uint32)
    out = np.empty(w.shape, np.int32)
    lib().orc_decode_be32(_p(w), _p(out), w.size)
    return out


# ---- quantise / dequantise / reduce ----
def quantise(x: np.ndarray, k: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    q = np.empty(x.shape, np.int32)
    lib().orc_quantise_f32(_p(x), _p(q), x.size, int(k))
    return q


def dequantise(q: np.ndarray, k: int) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int32)
    f = np.empty(q.shape, np.float32)
    lib().orc_dequantise_q32(_p(q), _p(f), q.size, int(k))
    return f


def sum_q32(srcs) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.int32) for s in srcs]
    out = np.empty(srcs[0].shape, np.int32)
    lib().orc_sum_q32(_ptr_array(srcs), len(srcs), _p(out), out.size)
    return out


def reduce_f32(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.float32) for s in srcs]
    out = np.empty(srcs[0].shape, np.float32)
    lib().orc_reduce_f32(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def quant_sum(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.float32) for s in srcs]
    out = np.empty(srcs[0].shape, np.int32)
    lib().orc_quant_sum(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def absmax(srcs) -> float:
    srcs = [np.ascontiguousarray(s, dtype=np.float32) for s in srcs]
    return float(lib().orc_absmax_f32(_ptr_array(srcs), len(srcs), srcs[0].size))


# ---- bfloat16 buckets (uint16 bit patterns) ----
def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    L = lib()
    return np.array([L.orc_f32_to_bf16(float(v)) for v in x], np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(h, dtype=np.uint16)
    return (h.astype(np.uint32) << 16).view(np.float32)


def reduce_bf16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    out = np.empty(srcs[0].shape, np.uint16)
    lib().orc_reduce_bf16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def quant_sum_bf16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    out = np.empty(srcs[0].shape, np.int32)
    lib().orc_quant_sum_bf16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def sum_dequant_bf16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.int32) for s in srcs]
    out = np.empty(srcs[0].shape, np.uint16)
    lib().orc_sum_dequant_bf16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def absmax_bf16(srcs) -> float:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    return float(lib().orc_absmax_bf16(_ptr_array(srcs), len(srcs), srcs[0].size))


# ---- IEEE binary16 buckets (uint16 bit patterns) ----
def f16_to_f32(h: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(h, dtype=np.uint16).ravel()
    out = np.empty(h.size, np.float32)
    lib().orc_f16_to_f32_n(_p(h), _p(out), h.size)
    return out


def f32_to_f16(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.empty(x.size, np.uint16)
    lib().orc_f32_to_f16_n(_p(x), _p(out), x.size)
    return out


def reduce_f16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    out = np.empty(srcs[0].shape, np.uint16)
    lib().orc_reduce_f16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def quant_sum_f16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    out = np.empty(srcs[0].shape, np.int32)
    lib().orc_quant_sum_f16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def sum_dequant_f16(srcs, k: int) -> np.ndarray:
    srcs = [np.ascontiguousarray(s, dtype=np.int32) for s in srcs]
    out = np.empty(srcs[0].shape, np.uint16)
    lib().orc_sum_dequant_f16(_ptr_array(srcs), len(srcs), _p(out), out.size, int(k))
    return out


def absmax_f16(srcs) -> float:
    srcs = [np.ascontiguousarray(s, dtype=np.uint16) for s in srcs]
    return float(lib().orc_absmax_f16(_ptr_array(srcs), len(srcs), srcs[0].size))


# ---- non-finite inputs under INCCL_NONFINITE_NAN (this library's own spec,
# include/inccl_amd.h inccl_comm_set_nonfinite / INCCL_ABSMAX_FLAG_NONFINITE;
# the reference has no floats) ----
def widened_bits(src, kind: str = "f32") -> np.ndarray:
    """fp32 bit patterns of an fp32 / bf16 / fp16 bucket's elements, widened exactly"""
    if kind == "f32":
        return np.ascontiguousarray(src, dtype=np.float32).view(np.uint32).ravel()
    if kind == "bf16":
        return np.ascontiguousarray(src, dtype=np.uint16).astype(np.uint32).ravel() << 16
    return f16_to_f32(src).view(np.uint32)


def absmax_word_flagged(srcs, kind: str = "f32") -> int:
    """The absmax word with INCCL_ABSMAX_FLAG_NONFINITE: max over |x| bits, where a
    NaN or +-Inf element counts as bit 31 | its |x| bits"""
    m = 0
    for s in srcs:
        a = widened_bits(s, kind) & np.uint32(0x7FFFFFFF)
        w = np.where(a >= np.uint32(0x7F800000), a | np.uint32(0x80000000), a)
        if w.size:
            m = max(m, int(w.max()))
    return m


def any_nonfinite(srcs, kind: str = "f32") -> bool:
    return bool(absmax_word_flagged(srcs, kind) >> 31)


def choose_scale(amax: float, R: int) -> int:
    return int(lib().orc_choose_scale(ctypes.c_float(amax), int(R)))


def checksum_q32(q: np.ndarray, index_base: int = 0) -> int:
    q = np.ascontiguousarray(q, dtype=np.int32)
    return int(lib().orc_checksum_q32(_p(q), q.size, int(index_base)))


# ---- switch (nts.c:303-501) ----
class Switch:
    """Root switch with `fan_in` children (nts.c state, restated); `slots` is
    the PSN ring (the reference's is 16, window 8: nts.c:21-22).  nonroot=True:
    a non-root switch (nts.c:376-400, :408-423, :457-499) whose parent is port
    fan_in; `flags` SW_WIRE_ORDER / SW_RECYCLE (0: the reference exactly)."""

    def __init__(self, fan_in: int, slots: int = SW_SLOTS, nonroot: bool = False, flags: int = 0):
        self.fan_in = int(fan_in)
        self.nonroot = bool(nonroot)
        self.rows = self.fan_in + (1 if self.nonroot else 0)
        self._buf = np.zeros(int(lib().orc_switch_bytes()), np.uint8)
        if self.nonroot:
            rc = lib().orc_switch_init_nonroot(_p(self._buf), self.fan_in, int(slots), int(flags))
        else:
            rc = lib().orc_switch_init_ring(_p(self._buf), self.fan_in, int(slots))
        if rc != 0:
            raise ValueError(f"orc switch: fan_in {fan_in}, slots {slots}, flags {flags}")

    def ingress(self, port: int, psn: int, payload_be: np.ndarray):
        payload_be = np.ascontiguousarray(payload_be, dtype=np.uint32)
        assert payload_be.size == LANES
        egress = np.zeros(LANES, np.uint32)
        rc = lib().orc_switch_ingress(_p(self._buf), int(port), int(psn), _p(payload_be), _p(egress))
        return rc, egress

    def slot(self, psn: int) -> np.ndarray:
        """The aggregator words of `psn`'s slot (uint32 copy)."""
        a = lib().orc_switch_slot(_p(self._buf), int(psn))
        return np.ctypeslib.as_array((ctypes.c_uint32 * LANES).from_address(a)).copy()

    def pipeline(self, conns: np.ndarray, port: int, frame: bytes, row_len: int | None = None):
        """nts.c:303-501 on one frame (orc_switch_pipeline): (action, [frame
        bytes sent to row c, or None]).  `conns` holds one 28-byte connection
        record per row (the engine's FRAME_TEMPLATE_DTYPE layout): fan_in
        children, and for a non-root the parent last."""
        c = np.ascontiguousarray(conns).view(np.uint8)
        assert c.size == 28 * self.rows
        row = max(len(frame), 64) if row_len is None else int(row_len)
        fb = np.zeros(max(row, len(frame), 64), np.uint8)
        fb[: len(frame)] = np.frombuffer(bytes(frame), np.uint8)
        out = np.zeros((self.rows, FRAME_ROW), np.uint8)
        ln = np.zeros(self.rows, np.int32)
        rc = lib().orc_switch_pipeline(_p(self._buf), _p(c), int(port), _p(fb), row, _p(out), FRAME_ROW, _p(ln))
        return rc, [out[i, : ln[i]].tobytes() if ln[i] else None for i in range(self.rows)]


# ---- framing (util.c) ----
def crc32(data: bytes) -> int:
    b = np.frombuffer(bytes(data), np.uint8).copy()
    return int(lib().orc_crc32(_p(b), b.size))


def icrc(frame: bytes) -> int:
    b = np.zeros(max(len(frame), 64), np.uint8)
    b[: len(frame)] = np.frombuffer(bytes(frame), np.uint8)
    return int(lib().orc_icrc(_p(b)))


class FrameHdr(ctypes.Structure):
    _fields_ = [("src_mac", ctypes.c_uint8 * 6), ("dst_mac", ctypes.c_uint8 * 6),
                ("src_ip", ctypes.c_uint32), ("dst_ip", ctypes.c_uint32),
                ("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16),
                ("qp", ctypes.c_uint32), ("psn", ctypes.c_uint32), ("opcode", ctypes.c_uint8)]


def build_data_frame(payload_host: np.ndarray, psn: int, opcode: int, qp: int = 0x11,
                     with_reth: bool = False, reth: bytes | None = None,
                     src_ip: int = 0, dst_ip: int = 0, src_port: int = 4791, dst_port: int = 4791,
                     src_mac: bytes = bytes(6), dst_mac: bytes = bytes(6)) -> bytes:
    payload_host = np.ascontiguousarray(payload_host, dtype=np.int32)
    h = FrameHdr()
    for i in range(6):
        h.src_mac[i] = src_mac[i]
        h.dst_mac[i] = dst_mac[i]
    h.src_ip, h.dst_ip, h.src_port, h.dst_port = src_ip, dst_ip, src_port, dst_port
    h.qp, h.psn, h.opcode = qp, psn, opcode
    frame = np.zeros(4096 + 128, np.uint8)
    rb = None
    if reth is not None:
        rb = np.frombuffer(reth, np.uint8).copy()
    n = lib().orc_build_data_frame(_p(frame), ctypes.byref(h), _p(payload_host), payload_host.size,
                                   1 if with_reth else 0, _p(rb) if rb is not None else None)
    return frame[:n].tobytes()


def build_ack_frame(psn: int, msn: int | None = None, qp: int = 0x11, src_ip: int = 0, dst_ip: int = 0,
                    src_port: int = 4791, dst_port: int = 4791, src_mac: bytes = bytes(6),
                    dst_mac: bytes = bytes(6)) -> bytes:
    """util.c:331-442 PACKET_TYPE_ACK (send_roce_ack: msn = psn + 1, nts.c:292)."""
    h = FrameHdr()
    for i in range(6):
        h.src_mac[i] = src_mac[i]
        h.dst_mac[i] = dst_mac[i]
    h.src_ip, h.dst_ip, h.src_port, h.dst_port = src_ip, dst_ip, src_port, dst_port
    h.qp, h.psn, h.opcode = qp, psn, 0x11
    frame = np.zeros(128, np.uint8)
    n = lib().orc_build_ack_frame(_p(frame), ctypes.byref(h), (psn + 1) if msn is None else int(msn))
    return frame[:n].tobytes()


# ---- loopback driver (api.c:403-452 + nts.c) ----
def allreduce_write_loopback(srcs, len_elems: int | None = None, dup_every: int = 0,
                             dst_init=None, with_icrc: bool = False):
    srcs = [np.ascontiguousarray(s, dtype=np.int32) for s in srcs]
    R = len(srcs)
    n = srcs[0].size if len_elems is None else int(len_elems)
    if dst_init is None:
        dsts = [np.zeros(srcs[0].size, np.int32) for _ in range(R)]
    else:
        dsts = [np.array(d, dtype=np.int32, copy=True) for d in dst_init]
    frames = ctypes.c_uint64(0)
    rc = lib().orc_allreduce_write_loopback(R, _ptr_array(srcs), n, _ptr_array(dsts), int(dup_every),
                                            ctypes.byref(frames), 1 if with_icrc else 0)
    return rc, dsts, int(frames.value)
