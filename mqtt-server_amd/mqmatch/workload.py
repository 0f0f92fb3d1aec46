"""Synthetic workloads from mqtt-server_amd/lib/libmqgen.so.

Generates subscriptions, publish topics, retained topics and Messages filters as columnar
numpy arrays (concatenated bytes + u64 offsets). Input generation only.
"""
import ctypes as C
import os

import numpy as np

from ._paths import LIB_DIR

BASE_SEED = 0x6D716D61
MIX_MQTT = 0   # config-2/3 mix
MIX_IOT = 1    # config-4 IoT fan-in

_LIB = None
_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(LIB_DIR, "libmqgen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        L = C.CDLL(path)
        L.mqgen_subs.restype = C.c_void_p
        L.mqgen_subs.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_int]
        for f in ("mqgen_subs_n", "mqgen_subs_nbytes", "mqgen_subs_unique_filters",
                  "mqgen_batch_n", "mqgen_batch_nbytes"):
            getattr(L, f).restype = C.c_uint64
            getattr(L, f).argtypes = [C.c_void_p]
        L.mqgen_subs_copy.argtypes = [C.c_void_p, _u8p, _u64p, _u32p, _u32p, _u8p, _u8p, _i32p]
        L.mqgen_subs_free.argtypes = [C.c_void_p]
        L.mqgen_topics.restype = C.c_void_p
        L.mqgen_topics.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int]
        L.mqgen_retained.restype = C.c_void_p
        L.mqgen_retained.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
        L.mqgen_msg_filters.restype = C.c_void_p
        L.mqgen_msg_filters.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.mqgen_batch_copy.argtypes = [C.c_void_p, _u8p, _u64p, _u64p]
        L.mqgen_batch_free.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


class _Handle:
    def __init__(self, h, free):
        self.h, self._free = h, free

    def __del__(self):
        if self.h:
            self._free(self.h)
            self.h = None


def gen_subscriptions(n_subs, n_clients, seed=BASE_SEED, mix=MIX_MQTT):
    """Columnar subscriptions: bytes, offs, client_ids, filter_ids, qos, flags, idents.
    flags = nolocal | rap<<1 | rh<<2 (include/mqmatch.h MQ_SUB_*)."""
    L = _lib()
    h = L.mqgen_subs(n_subs, n_clients, seed, mix)
    n, nb = L.mqgen_subs_n(h), L.mqgen_subs_nbytes(h)
    w = {
        "bytes": np.empty(max(nb, 1), np.uint8), "offs": np.empty(n + 1, np.uint64),
        "client_ids": np.empty(n, np.uint32), "filter_ids": np.empty(n, np.uint32),
        "qos": np.empty(n, np.uint8), "flags": np.empty(n, np.uint8),
        "idents": np.empty(n, np.int32),
    }
    L.mqgen_subs_copy(h, _p(w["bytes"], _u8p), _p(w["offs"], _u64p), _p(w["client_ids"], _u32p),
                      _p(w["filter_ids"], _u32p), _p(w["qos"], _u8p), _p(w["flags"], _u8p),
                      _p(w["idents"], _i32p))
    w["n_unique_filters"] = int(L.mqgen_subs_unique_filters(h))
    w["_handle"] = _Handle(h, L.mqgen_subs_free)  # kept for topic generation
    return w


def _batch(h):
    L = _lib()
    n, nb = L.mqgen_batch_n(h), L.mqgen_batch_nbytes(h)
    b = np.empty(max(nb, 1), np.uint8)
    o = np.empty(n + 1, np.uint64)
    hd = np.zeros(n, np.uint64)
    L.mqgen_batch_copy(h, _p(b, _u8p), _p(o, _u64p), _p(hd, _u64p))
    return b, o, hd


def gen_topics(subs, n_topics, seed=BASE_SEED, mix=MIX_MQTT):
    """Publish topics (bytes, offs) instantiated from `subs`."""
    L = _lib()
    h = L.mqgen_topics(subs["_handle"].h if subs is not None else None, n_topics, seed, mix)
    b, o, _ = _batch(h)
    L.mqgen_batch_free(h)
    return b, o


def gen_retained(n, n_sys=1000, seed=BASE_SEED, mix=MIX_MQTT):
    """Retained topic names (bytes, offs, handles) plus the generator handle for filters."""
    L = _lib()
    h = L.mqgen_retained(n, n_sys, seed, mix)
    b, o, hd = _batch(h)
    return b, o, hd, _Handle(h, L.mqgen_batch_free)


def gen_msg_filters(retained_handle, n, seed=BASE_SEED):
    L = _lib()
    h = L.mqgen_msg_filters(retained_handle.h, n, seed)
    b, o, _ = _batch(h)
    L.mqgen_batch_free(h)
    return b, o


def strings(bytes_, offs):
    """Decode a columnar string batch into a Python list (small batches only)."""
    raw = bytes_.tobytes()
    return [raw[int(offs[i]):int(offs[i + 1])].decode("utf-8", "surrogateescape")
            for i in range(len(offs) - 1)]
