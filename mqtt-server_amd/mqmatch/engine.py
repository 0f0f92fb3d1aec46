"""ctypes binding of lib/libmqmatch.so (include/mqmatch.h) and a host-side mirror of the
reference Go `TopicsIndex` API (/root/reference/topics.go:349-698).

The mirror does what the Go cgo shim does: it interns client-ID and filter
strings to u32 ids, keeps the stored packets.Subscription values host-side, calls the engine
through the C-ABI, and rematerialises the engine's id rows as Go-shaped `Subscribers`
(topics.go:312-317). There is no CPU matching path: if the library or a GPU is missing, the
calls raise.
"""
import ctypes as C
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from ._paths import LIB_DIR

SHARE_PREFIX = "$SHARE"  # topics.go:16
SYS_PREFIX = "$SYS"      # topics.go:17

META_QOS = 0x3
META_NOLOCAL = 0x100
META_RAP = 0x200
META_RH_SHIFT = 10

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class MqConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32), ("expected_subs", C.c_uint64),
                ("expected_nodes", C.c_uint64), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32)]


class XList(C.Structure):
    """mq_xlist: a shard's exported cross-shard nodes per topic (device pointers)."""
    _fields_ = [("n_topics", C.c_uint32), ("shard", C.c_uint32), ("counts", C.c_void_p), ("ents", C.c_void_p),
                ("n_ents", C.c_uint64)]


class TopicResult(C.Structure):
    _fields_ = [("sub_base", C.c_uint64), ("shared_base", C.c_uint64), ("inline_base", C.c_uint64),
                ("sub_cap", C.c_uint32), ("n_client", C.c_uint32), ("n_ident", C.c_uint32),
                ("n_shared", C.c_uint32), ("n_inline", C.c_uint32), ("reserved", C.c_uint32)]


class MatchResult(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("reserved", C.c_uint32),
                ("topics", C.c_void_p), ("sub_rows", C.c_void_p), ("shared_rows", C.c_void_p),
                ("inline_rows", C.c_void_p), ("n_sub_rows", C.c_uint64),
                ("n_shared_rows", C.c_uint64), ("n_inline_rows", C.c_uint64)]


class TopicSpans(C.Structure):
    _fields_ = [("span_base", C.c_uint64), ("patch_base", C.c_uint64), ("inline_base", C.c_uint64),
                ("picked_base", C.c_uint64), ("n_spans", C.c_uint32), ("n_patches", C.c_uint32),
                ("n_inline", C.c_uint32), ("n_rows", C.c_uint32), ("n_client", C.c_uint32),
                ("n_ident", C.c_uint32), ("n_shared", C.c_uint32), ("flags", C.c_uint32)]


class SpanResult(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("flags", C.c_uint32), ("topics", C.c_void_p), ("spans", C.c_void_p),
                ("patches", C.c_void_p), ("inline_rows", C.c_void_p), ("picked_rows", C.c_void_p),
                ("sub_pool", C.c_void_p), ("shared_pool", C.c_void_p), ("n_spans", C.c_uint64),
                ("n_patches", C.c_uint64), ("n_inline_rows", C.c_uint64), ("n_picked_rows", C.c_uint64),
                ("sub_pool_len", C.c_uint64), ("shared_pool_len", C.c_uint64),
                ("set_patches", C.c_void_p), ("merge_rows", C.c_void_p), ("n_set_patches", C.c_uint64),
                ("merge_row_base", C.c_void_p), ("n_merge_rows", C.c_uint64)]


SPANS_PICKED = 1  # MQ_SPANS_PICKED
MQ_EINVAL, MQ_ENOMEM, MQ_ENODEV, MQ_EIO = -22, -12, -19, -5  # include/mqmatch.h return codes
PROF_TIMES, PROF_WORK, PROF_WALK = 1, 2, 4  # mq_profile_enable

# mq_set_option: product options (include/mqmatch.h) and development ones (include/mqmatch_dev.h)
OPT_CHUNK_ROWS, OPT_PATCH_CAP, OPT_EDGE_LOAD = 1, 6, 13
OPT_SUBBATCH_TOPICS, OPT_MSG_SPEC_MB, OPT_MSG_WAVES, OPT_SERIAL, OPT_MERGE_WAVES = 2, 3, 4, 5, 7
OPT_MSG_IMAGE, OPT_WALK_WAVES, OPT_WALK_LISTS, OPT_MERGE_DEDUP = 8, 9, 10, 12
OPT_SET_GRID, OPT_WALK_GROUP, OPT_ONE_SYNC, OPT_FUSE_DESC, OPT_SET_EXP, OPT_MSG_EXPORT = 14, 15, 16, 17, 18, 19
OPT_PATCH_CODES = 20
OPT_MSG_EDGES = 21
OPT_MSG_EDGE_BUDGET, OPT_FAIL_NEXT, OPT_WALK_EXP, OPT_MSG_KEYIDX = 22, 23, 24, 25
OPT_MAX = 25  # (include/mqmatch_dev.h MQ_OPT_MAX)


class MsgResult(C.Structure):
    _fields_ = [("n_filters", C.c_uint32), ("reserved", C.c_uint32), ("base", C.c_void_p),
                ("count", C.c_void_p), ("handles", C.c_void_p), ("n_handles", C.c_uint64)]


class MsgRunsResult(C.Structure):  # mq_msg_runs_result
    _fields_ = [("n_filters", C.c_uint32), ("reserved", C.c_uint32), ("run_base", C.c_void_p),
                ("n_runs", C.c_void_p), ("base", C.c_void_p), ("count", C.c_void_p), ("runs", C.c_void_p),
                ("n_runs_total", C.c_uint64), ("handles", C.c_void_p), ("n_handles", C.c_uint64),
                ("n_expanded", C.c_uint64)]


# mq_msg_run: first handle, count, where the run starts in the batch's expanded output
MSG_RUN_DT = np.dtype([("first", np.uint32), ("count", np.uint32), ("at", np.uint64)])


class AclResult(C.Structure):
    _fields_ = [("n_pairs", C.c_uint64), ("matched", C.c_void_p), ("n_elems", C.c_void_p),
                ("elem_base", C.c_void_p), ("elems", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("nodes", "edges", "edge_capacity", "subs", "subs_merge",
                                           "shared", "inlines", "retained", "retained_live",
                                           "device_bytes", "upload_bytes_total", "syncs", "partners",
                                           "foreign")] + \
               [("max_depth", C.c_uint32), ("edge_load", C.c_uint32)]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_uint64), ("total_ms", C.c_double)]


# Every symbol declared in include/mqmatch.h (checked by tests/test_capi.py).
EXPORTS = [
    "mq_index_create", "mq_index_destroy", "mq_last_error", "mq_abi_version", "mq_subscribe",
    "mq_unsubscribe", "mq_inline_subscribe", "mq_inline_unsubscribe", "mq_retain_message",
    "mq_retained_delete", "mq_retained_set", "mq_retained_len", "mq_subscribe_bulk", "mq_retain_bulk",
    "mq_match_batch", "mq_match_device", "mq_match_chunks", "mq_messages_batch",
    "mq_messages_device", "mq_result_free", "mq_sync", "mq_index_stats", "mq_profile_enable",
    "mq_profile_read", "mq_profile_reset", "mq_index_check", "mq_match_device_chunks",
    "mq_acl_match_batch", "mq_select_shared_device", "mq_match_spans", "mq_match_spans_device",
    "mq_spans_expand", "mq_set_option", "mq_match_spans_begin", "mq_match_spans_end",
    "mq_match_spans_end_host", "mq_device_check", "mq_match_spans_submit", "mq_match_spans_wait",
    "mq_unsubscribe_bulk", "mq_thread_warm", "mq_messages_runs_device", "mq_messages_runs_batch",
    "mq_msg_runs_expand",
]

CFG_SELECT_SHARED = 1  # MQ_CFG_SELECT_SHARED
SPANS_PATCH_CODES = 2  # MQ_SPANS_PATCH_CODES
PATCH_OP = 0x20000000  # MQ_PATCH_OP

CHUNK_FN = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(MatchResult), C.c_uint32, C.c_void_p)

_LIB = None


def lib_path():
    return os.path.join(LIB_DIR, "libmqmatch.so")


def lib():
    """Load the engine library; raises if it is missing (there is no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: build it with __graft_entry__.build()")
    L = C.CDLL(path)
    vp = C.c_void_p
    sig = {
        "mq_index_create": (C.c_int, [C.POINTER(MqConfig), C.POINTER(vp)]),
        "mq_index_destroy": (None, [vp]),
        "mq_last_error": (C.c_char_p, []),
        "mq_abi_version": (C.c_uint32, []),
        "mq_subscribe": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint8,
                                   C.c_uint8, C.c_int32]),
        "mq_unsubscribe": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_uint32]),
        "mq_inline_subscribe": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_int32, C.c_uint32]),
        "mq_inline_unsubscribe": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_int32]),
        "mq_retain_message": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                        C.c_uint8, _i64p]),
        "mq_retained_delete": (C.c_int, [vp, C.c_char_p, C.c_uint32]),
        "mq_retained_set": (C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint8]),
        "mq_retained_len": (C.c_uint64, [vp]),
        "mq_subscribe_bulk": (C.c_int, [vp, _u8p, _u64p, _u32p, _u32p, _u8p, _u8p, _i32p,
                                        C.c_uint64, _u8p]),
        "mq_retain_bulk": (C.c_int, [vp, _u8p, _u64p, _u64p, C.c_uint64]),
        "mq_unsubscribe_bulk": (C.c_int, [vp, _u8p, _u64p, _u32p, C.c_uint64, _u8p]),
        "mq_thread_warm": (C.c_int, [vp]),
        "mq_match_batch": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, C.POINTER(C.POINTER(MatchResult))]),
        "mq_match_device": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.POINTER(MatchResult)]),
        "mq_match_spans": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, C.POINTER(C.POINTER(SpanResult))]),
        "mq_match_spans_device": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.POINTER(SpanResult)]),
        "mq_match_spans_submit": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, C.POINTER(vp)]),
        "mq_match_spans_wait": (C.c_int, [vp, C.POINTER(C.POINTER(SpanResult))]),
        "mq_spans_expand": (C.c_int, [C.POINTER(SpanResult), C.c_uint32, C.c_uint32, vp, C.c_uint64, vp,
                                      C.c_uint64, _u64p, _u64p]),
        "mq_set_option": (C.c_int, [vp, C.c_uint32, C.c_uint64]),
        "mq_match_spans_begin": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.POINTER(XList)]),
        "mq_match_spans_end": (C.c_int, [vp, C.POINTER(XList), C.c_uint32, vp, C.POINTER(SpanResult)]),
        "mq_match_spans_end_host": (C.c_int, [vp, C.POINTER(XList), C.c_uint32, C.POINTER(C.POINTER(SpanResult))]),
        "mq_match_chunks": (C.c_uint32, [vp]),
        "mq_select_shared_device": (C.c_int, [vp, C.POINTER(MatchResult), vp, vp, vp]),
        "mq_match_device_chunks": (C.c_int, [vp, vp, vp, C.c_uint32, vp, CHUNK_FN, vp]),
        "mq_acl_match_batch": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, _u8p, _u64p, C.c_uint32, _u32p, _u32p,
                                         C.c_uint64, C.POINTER(C.POINTER(AclResult))]),
        "mq_messages_batch": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, C.POINTER(C.POINTER(MsgResult))]),
        "mq_messages_device": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.POINTER(MsgResult)]),
        "mq_messages_runs_device": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.POINTER(MsgRunsResult)]),
        "mq_messages_runs_batch": (C.c_int, [vp, _u8p, _u64p, C.c_uint32, C.POINTER(C.POINTER(MsgRunsResult))]),
        "mq_msg_runs_expand": (C.c_int, [C.POINTER(MsgRunsResult), C.c_uint32, C.c_uint32, _u64p, C.c_uint64,
                                         _u64p]),
        "mq_result_free": (None, [vp]),
        "mq_sync": (C.c_int, [vp, vp]),
        "mq_index_stats": (C.c_int, [vp, C.POINTER(Stats)]),
        "mq_index_check": (C.c_int, [vp]),
        "mq_device_check": (C.c_int, [vp]),
        "mq_profile_enable": (C.c_int, [vp, C.c_int]),
        "mq_profile_read": (C.c_int, [vp, C.POINTER(KernelTime), C.c_uint32]),
        "mq_profile_reset": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


class EngineError(RuntimeError):
    pass


def _check(rc, what):
    if rc < 0:
        msg = lib().mq_last_error()
        raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def _b(s):
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s)


def _p(a, t):
    return a.ctypes.data_as(t)


def pack_strings(items):
    """List of str/bytes -> (uint8 bytes, uint64 offsets)."""
    bs = [_b(x) for x in items]
    offs = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        offs[1:] = np.cumsum([len(x) for x in bs], dtype=np.uint64)
    raw = np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy()
    return raw, offs


# ---- Go-shaped values (packets/packets.go:172-182, topics.go:306-317) -----------------------------
@dataclass
class Subscription:
    filter: str = ""
    identifier: int = 0
    qos: int = 0
    no_local: bool = False
    retain_as_published: bool = False
    retain_handling: int = 0
    identifiers: Optional[Dict[str, int]] = None

    def merge(self, n: "Subscription") -> "Subscription":
        """Subscription.Merge (packets/packets.go:254-274)."""
        s = Subscription(self.filter, self.identifier, self.qos, self.no_local,
                         self.retain_as_published, self.retain_handling,
                         None if self.identifiers is None else self.identifiers)
        if s.identifiers is None:
            s.identifiers = {s.filter: s.identifier}
        if n.identifier > 0:
            s.identifiers[n.filter] = n.identifier
        if n.qos > s.qos:
            s.qos = n.qos
        if n.no_local:
            s.no_local = True
        return s


@dataclass
class InlineSubscription:
    filter: str = ""
    identifier: int = 0


@dataclass
class Subscribers:
    shared: Dict[str, Dict[str, Subscription]] = field(default_factory=dict)
    shared_selected: Dict[str, Subscription] = field(default_factory=dict)
    subscriptions: Dict[str, Subscription] = field(default_factory=dict)
    inline_subscriptions: Dict[int, InlineSubscription] = field(default_factory=dict)

    def select_shared(self):
        """SelectShared (topics.go:320-333). Go picks the first member in random map order;
        this picks the first in sorted order, one of the orders Go can produce."""
        self.shared_selected = {}
        for _, subs in sorted(self.shared.items()):
            for client, sub in sorted(subs.items()):
                cls = self.shared_selected.get(client, sub)
                self.shared_selected[client] = cls.merge(sub)
                break

    def merge_shared_selected(self):
        """MergeSharedSelected (topics.go:338-347)."""
        for client, sub in self.shared_selected.items():
            cls = self.subscriptions.get(client, sub)
            self.subscriptions[client] = cls.merge(sub)


def is_share_prefix(seg: str) -> bool:
    """strings.EqualFold(seg, "$SHARE") with Go simple folding (U+017F ~ 's', Q9)."""
    if len(seg) != 6:
        return False
    for a, b in zip(seg, SHARE_PREFIX):
        if a == "ſ" and b == "S":
            continue
        if not a.isascii() or a.lower() != b.lower():
            return False
    return True


class Engine:
    """Thin object wrapper over one mq_index handle (id-level C-ABI)."""

    def __init__(self, device=0, expected_subs=0, expected_nodes=0, select_shared=False, shard=0, n_shards=1):
        """select_shared: MQ_CFG_SELECT_SHARED (results carry one picked member per shared
        filter; SelectShared ran on the device). shard / n_shards: a sharded index (mq_config)."""
        L = lib()
        cfg = MqConfig(device, CFG_SELECT_SHARED if select_shared else 0, expected_subs, expected_nodes,
                       shard, n_shards)
        h = C.c_void_p()
        _check(L.mq_index_create(C.byref(cfg), C.byref(h)), "mq_index_create")
        self.h = h
        # MQ_ENGINE_OPTIONS="opt=value,..." (MQ_OPT_* numbers): engine options for every index this
        # process creates — how a test run exercises a non-default engine path
        for kv in os.environ.get("MQ_ENGINE_OPTIONS", "").split(","):
            if kv.strip():
                k, v = kv.split("=")
                self.set_option(int(k), int(v))

    def close(self):
        if self.h:
            lib().mq_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def subscribe(self, filter, client_id, filter_id, qos=0, flags=0, identifier=0):
        fb = _b(filter)
        return _check(lib().mq_subscribe(self.h, fb, len(fb), client_id, filter_id, qos, flags,
                                         identifier), "mq_subscribe")

    def unsubscribe(self, filter, client_id):
        fb = _b(filter)
        return _check(lib().mq_unsubscribe(self.h, fb, len(fb), client_id), "mq_unsubscribe")

    def inline_subscribe(self, filter, identifier, filter_id):
        fb = _b(filter)
        return _check(lib().mq_inline_subscribe(self.h, fb, len(fb), identifier, filter_id),
                      "mq_inline_subscribe")

    def inline_unsubscribe(self, filter, identifier):
        fb = _b(filter)
        return _check(lib().mq_inline_unsubscribe(self.h, fb, len(fb), identifier),
                      "mq_inline_unsubscribe")

    def retain_message(self, topic, handle, payload_len, retain=True):
        tb = _b(topic)
        out = C.c_int64()
        _check(lib().mq_retain_message(self.h, tb, len(tb), handle, payload_len,
                                       1 if retain else 0, C.byref(out)), "mq_retain_message")
        return out.value

    def retained_delete(self, topic):
        tb = _b(topic)
        return _check(lib().mq_retained_delete(self.h, tb, len(tb)), "mq_retained_delete")

    def retained_set(self, topic, handle, payload_len=1, retain=True):
        """mq_retained_set: Retained.Add outside RetainMessage."""
        tb = _b(topic)
        return _check(lib().mq_retained_set(self.h, tb, len(tb), handle, payload_len, 1 if retain else 0),
                      "mq_retained_set")

    def retained_len(self):
        return int(lib().mq_retained_len(self.h))

    def subscribe_bulk(self, w):
        n = len(w["client_ids"])
        out = np.zeros(max(n, 1), np.uint8)
        _check(lib().mq_subscribe_bulk(self.h, _p(w["bytes"], _u8p), _p(w["offs"], _u64p),
                                       _p(w["client_ids"], _u32p), _p(w["filter_ids"], _u32p),
                                       _p(w["qos"], _u8p), _p(w["flags"], _u8p),
                                       _p(w["idents"], _i32p), n, _p(out, _u8p)),
               "mq_subscribe_bulk")
        return out[:n]

    def unsubscribe_bulk(self, bytes_, offs, client_ids):
        """mq_unsubscribe_bulk: per pair, whether the filter's particle existed (as unsubscribe)."""
        n = len(offs) - 1
        out = np.zeros(max(n, 1), np.uint8)
        _check(lib().mq_unsubscribe_bulk(self.h, _p(bytes_, _u8p), _p(offs, _u64p), _p(client_ids, _u32p), n,
                                         _p(out, _u8p)), "mq_unsubscribe_bulk")
        return out[:n]

    def retain_bulk(self, bytes_, offs, handles):
        _check(lib().mq_retain_bulk(self.h, _p(bytes_, _u8p), _p(offs, _u64p),
                                    _p(handles, _u64p), len(offs) - 1), "mq_retain_bulk")

    def sync(self, stream=None):
        _check(lib().mq_sync(self.h, stream), "mq_sync")

    def device_check(self):
        """mq_device_check: the device arrays equal the host mirror (diagnostic)."""
        _check(lib().mq_device_check(self.h), "mq_device_check")

    def check(self):
        """mq_index_check: host-side invariants of the device-bound image (raises on violation)."""
        _check(lib().mq_index_check(self.h), "mq_index_check")

    def stats(self):
        s = Stats()
        _check(lib().mq_index_stats(self.h, C.byref(s)), "mq_index_stats")
        return {n: getattr(s, n) for n, _ in Stats._fields_}

    def set_option(self, option, value):
        """mq_set_option (MQ_OPT_*)."""
        _check(lib().mq_set_option(self.h, option, int(value)), "mq_set_option")

    def match_spans(self, bytes_, offs):
        """mq_match_spans -> dict of numpy copies of the span-format result (topics as a
        structured array, spans [n,4], patches [n,2], inline rows, picked rows, flags, and the
        merge-set patches with the packed merge rows; host_topic_patches() resolves both kinds)."""
        n = len(offs) - 1
        rp = C.POINTER(SpanResult)()
        _check(lib().mq_match_spans(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)), "mq_match_spans")
        try:
            return _span_arrays(rp.contents, n)
        finally:
            lib().mq_result_free(rp)

    def match_batch_spans(self, bytes_, offs):
        """mq_match_spans, expanded on the host by mq_spans_expand into exactly match_batch()'s
        dict (rows region per topic = its spans' records with the patches applied)."""
        n = len(offs) - 1
        rp = C.POINTER(SpanResult)()
        _check(lib().mq_match_spans(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)), "mq_match_spans")
        return _expand_host_spans(rp, n)

    def match_spans_end_expanded(self, foreign, n):
        """mq_match_spans_end_host with the other shards' XLists, expanded like match_batch_spans."""
        arr = (XList * max(1, len(foreign)))(*foreign)
        rp = C.POINTER(SpanResult)()
        _check(lib().mq_match_spans_end_host(self.h, arr, len(foreign), C.byref(rp)), "mq_match_spans_end_host")
        return _expand_host_spans(rp, n)

    def match_spans_pipelined(self, bytes_, offs, batches, log=None):
        """`batches` consecutive mq_match_spans_submit calls of the same host topics, each waited
        for (mq_match_spans_wait) after the next one is submitted, so that a batch's copy into host
        memory runs beside the next batch's kernels; every result is freed. Returns the results'
        bytes (each batch's are the same). `log` (a list): each batch's (submit ms, ms waiting for
        the batch before it) is appended."""
        n = len(offs) - 1
        pending, nbytes = [], 0

        def finish(t):
            nonlocal nbytes
            rp = C.POINTER(SpanResult)()
            _check(lib().mq_match_spans_wait(t, C.byref(rp)), "mq_match_spans_wait")
            r = rp.contents
            pw = 4 if r.flags & SPANS_PATCH_CODES else 8
            nbytes = (64 * n + 16 * r.n_spans + pw * r.n_patches + 8 * r.n_inline_rows + 8 * r.n_picked_rows +
                      pw * r.n_set_patches + 4 * r.n_merge_rows + (4 * n if r.merge_row_base else 0))
            lib().mq_result_free(rp)
        for _ in range(batches):
            t = C.c_void_p()
            t0 = time.perf_counter()
            _check(lib().mq_match_spans_submit(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(t)),
                   "mq_match_spans_submit")
            t1 = time.perf_counter()
            pending.append(t)
            if len(pending) == 2:
                finish(pending.pop(0))
            if log is not None:
                log.append((round(1e3 * (t1 - t0), 3), round(1e3 * (time.perf_counter() - t1), 3)))
        while pending:
            finish(pending.pop(0))
        return int(nbytes)

    def match_spans_host(self, bytes_, offs, expand=False, block=1024, threads=1):
        """mq_match_spans with its results left in the library's host buffers (the end-to-end
        path: H2D topics, kernels, D2H of the span-format arrays). expand=True also materialises
        every topic's rows with mq_spans_expand, `block` topics per call into a reused buffer per
        thread, on `threads` host threads (mq_spans_expand is thread-safe for disjoint outputs;
        ctypes releases the GIL during the call) — what a consumer that wants rows pays. Returns
        (result bytes, rows expanded)."""
        n = len(offs) - 1
        rp = C.POINTER(SpanResult)()
        _check(lib().mq_match_spans(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)), "mq_match_spans")
        try:
            r = rp.contents
            pw = 4 if r.flags & SPANS_PATCH_CODES else 8  # (4-byte patch codes)
            parts = {"topics": 64 * n, "spans": 16 * r.n_spans, "patches": pw * r.n_patches,
                     "inline_rows": 8 * r.n_inline_rows, "picked_rows": 8 * r.n_picked_rows,
                     "set_patches": pw * r.n_set_patches, "merge_rows": 4 * r.n_merge_rows,
                     "merge_row_base": 4 * n if r.merge_row_base else 0}
            self.last_host_bytes = parts  # the result's bytes per array (bench.py's end_to_end)
            nbytes = sum(parts.values())
            done = 0
            if expand and n:
                buf = (C.c_char * (n * 64)).from_address(r.topics)
                top = np.frombuffer(buf, _TOPIC_SPANS_DT)
                csum = np.concatenate(([0], np.cumsum(top["n_rows"].astype(np.uint64))))
                ssum = np.concatenate(([0], np.cumsum(top["n_shared"].astype(np.uint64))))
                starts = list(range(0, n, block))
                cap_r = max(int(max(csum[min(b + block, n)] - csum[b] for b in starts)), 1)
                cap_s = max(int(max(ssum[min(b + block, n)] - ssum[b] for b in starts)), 1)
                threads = max(1, min(int(threads), len(starts)))

                def work(k):
                    rows = np.empty((cap_r, 4), np.uint32)
                    shared = np.empty((cap_s, 2), np.uint32)
                    nr, ns = C.c_uint64(), C.c_uint64()
                    got = 0
                    for b in starts[k::threads]:
                        _check(lib().mq_spans_expand(rp, b, min(block, n - b), rows.ctypes.data, cap_r,
                                                     shared.ctypes.data, cap_s, C.byref(nr), C.byref(ns)),
                               "mq_spans_expand")
                        got += int(nr.value)
                    return got
                if threads == 1:
                    done = work(0)
                else:
                    from concurrent.futures import ThreadPoolExecutor
                    with ThreadPoolExecutor(threads) as pool:
                        done = sum(pool.map(work, range(threads)))
        finally:
            lib().mq_result_free(rp)
        return int(nbytes), done

    def match_spans_begin(self, d_bytes, d_offs, n, stream=None):
        """mq_match_spans_begin -> XList (this shard's export; device pointers)."""
        x = XList()
        _check(lib().mq_match_spans_begin(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                          C.c_void_p(stream) if stream else None, C.byref(x)),
               "mq_match_spans_begin")
        return x

    def match_spans_end(self, foreign, stream=None):
        """mq_match_spans_end with the other shards' XLists -> SpanResult (device pointers)."""
        arr = (XList * max(1, len(foreign)))(*foreign)
        r = SpanResult()
        _check(lib().mq_match_spans_end(self.h, arr, len(foreign), C.c_void_p(stream) if stream else None,
                                        C.byref(r)), "mq_match_spans_end")
        return r

    def match_spans_device(self, d_bytes, d_offs, n, stream=None):
        """mq_match_spans_device on device pointers (ints); returns the SpanResult struct."""
        r = SpanResult()
        _check(lib().mq_match_spans_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                           C.c_void_p(stream) if stream else None, C.byref(r)),
               "mq_match_spans_device")
        return r

    def match_batch_rows(self, bytes_, offs):
        """mq_match_batch with its results left in the library's host buffers (freed here):
        the end-to-end path (H2D topics, kernels, D2H of every row). Returns the row counts."""
        n = len(offs) - 1
        rp = C.POINTER(MatchResult)()
        _check(lib().mq_match_batch(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)),
               "mq_match_batch")
        r = rp.contents
        counts = (int(r.n_sub_rows), int(r.n_shared_rows), int(r.n_inline_rows))
        lib().mq_result_free(rp)
        return counts

    def match_batch(self, bytes_, offs):
        """mq_match_batch -> dict of numpy arrays (host copies)."""
        n = len(offs) - 1
        rp = C.POINTER(MatchResult)()
        _check(lib().mq_match_batch(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)),
               "mq_match_batch")
        try:
            r = rp.contents
            def arr(ptr, count, dtype, width):
                if count == 0 or not ptr:
                    return np.zeros((0, width), dtype)
                buf = (C.c_char * (count * width * np.dtype(dtype).itemsize)).from_address(ptr)
                return np.frombuffer(buf, dtype).reshape(count, width).copy()
            topics = arr(r.topics, n, np.uint32, 12)
            out = {
                # TopicResult as u32 words: sub_base(0,1) shared_base(2,3) inline_base(4,5)
                # sub_cap(6) n_client(7) n_ident(8) n_shared(9) n_inline(10)
                "sub_base": topics[:, 0].astype(np.uint64) | (topics[:, 1].astype(np.uint64) << np.uint64(32)),
                "shared_base": topics[:, 2].astype(np.uint64) | (topics[:, 3].astype(np.uint64) << np.uint64(32)),
                "inline_base": topics[:, 4].astype(np.uint64) | (topics[:, 5].astype(np.uint64) << np.uint64(32)),
                "sub_cap": topics[:, 6].copy(), "n_client": topics[:, 7].copy(),
                "n_ident": topics[:, 8].copy(), "n_shared": topics[:, 9].copy(),
                "n_inline": topics[:, 10].copy(),
                "rows": arr(r.sub_rows, r.n_sub_rows, np.uint32, 4),
                "shared": arr(r.shared_rows, r.n_shared_rows, np.uint32, 2),
                "inline": arr(r.inline_rows, r.n_inline_rows, np.uint32, 2),
            }
        finally:
            lib().mq_result_free(rp)
        return out

    def messages_batch(self, bytes_, offs):
        """mq_messages_batch -> (base, count, handles): filter i has handles[base[i] : base[i] + count[i]]."""
        n = len(offs) - 1
        rp = C.POINTER(MsgResult)()
        _check(lib().mq_messages_batch(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)),
               "mq_messages_batch")
        try:
            r = rp.contents
            def arr(ptr, count, dtype):
                if count == 0 or not ptr:
                    return np.zeros(0, dtype)
                buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
                return np.frombuffer(buf, dtype).copy()
            base = arr(r.base, n, np.uint64)
            count = arr(r.count, n, np.uint32)
            hs = arr(r.handles, r.n_handles, np.uint64)
        finally:
            lib().mq_result_free(rp)
        return base, count, hs

    def messages_runs_batch(self, bytes_, offs, expand=False):
        """mq_messages_runs_batch -> dict of numpy arrays: run_base, n_runs, base, count, runs
        (MSG_RUN_DT) and handles (the array the runs index); with expand, also the expanded
        (base, count, handles) through mq_msg_runs_expand."""
        n = len(offs) - 1
        rp = C.POINTER(MsgRunsResult)()
        _check(lib().mq_messages_runs_batch(self.h, _p(bytes_, _u8p), _p(offs, _u64p), n, C.byref(rp)),
               "mq_messages_runs_batch")
        try:
            r = rp.contents

            def arr(ptr, count, dtype):
                if count == 0 or not ptr:
                    return np.zeros(0, dtype)
                buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
                return np.frombuffer(buf, dtype).copy()
            out = {"run_base": arr(r.run_base, n, np.uint64), "n_runs": arr(r.n_runs, n, np.uint32),
                   "base": arr(r.base, n, np.uint64), "count": arr(r.count, n, np.uint32),
                   "runs": arr(r.runs, r.n_runs_total, MSG_RUN_DT), "handles": arr(r.handles, r.n_handles, np.uint64),
                   "n_expanded": int(r.n_expanded)}
            if expand:
                hs = np.zeros(int(r.n_expanded), np.uint64)
                got = C.c_uint64(0)
                _check(lib().mq_msg_runs_expand(rp, 0, n, _p(hs, _u64p), len(hs), C.byref(got)), "mq_msg_runs_expand")
                assert got.value <= len(hs)
                out["expanded"] = hs
        finally:
            lib().mq_result_free(rp)
        return out

    def messages_runs_device(self, d_bytes, d_offs, n, stream=None):
        r = MsgRunsResult()
        _check(lib().mq_messages_runs_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                             C.c_void_p(stream) if stream else None, C.byref(r)),
               "mq_messages_runs_device")
        return r

    def messages_device(self, d_bytes, d_offs, n, stream=None):
        r = MsgResult()
        _check(lib().mq_messages_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                        C.c_void_p(stream) if stream else None, C.byref(r)),
               "mq_messages_device")
        return r

    def match_device(self, d_bytes, d_offs, n, stream=None):
        """mq_match_device on device pointers (ints); returns the MatchResult struct."""
        r = MatchResult()
        _check(lib().mq_match_device(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                     C.c_void_p(stream) if stream else None, C.byref(r)),
               "mq_match_device")
        return r

    def match_device_chunks(self, d_bytes, d_offs, n, stream, fn):
        """mq_match_device_chunks: fn(chunk: MatchResult, first_topic, chunk_stream) per chunk."""
        cb = CHUNK_FN(lambda user, chunk, first, cs: fn(chunk.contents, int(first), cs))
        _check(lib().mq_match_device_chunks(self.h, C.c_void_p(d_bytes), C.c_void_p(d_offs), n,
                                            C.c_void_p(stream) if stream else None, cb, None),
               "mq_match_device_chunks")

    def select_shared_device(self, chunk, stream, d_selected, d_n_selected):
        """mq_select_shared_device on a device MatchResult (SelectShared, topics.go:320-333):
        picked rows to d_selected at each topic's shared_base, counts to d_n_selected."""
        _check(lib().mq_select_shared_device(self.h, C.byref(chunk), C.c_void_p(stream) if stream else None,
                                             C.c_void_p(d_selected), C.c_void_p(d_n_selected)),
               "mq_select_shared_device")

    def match_chunks(self):
        return int(lib().mq_match_chunks(self.h))

    def acl_match_batch(self, filters, topics, pair_filter, pair_topic):
        """mq_acl_match_batch (auth.MatchTopic, hooks/auth/ledger.go:90-118) over pairs of the two
        string lists -> list of (elements, matched) per pair, as the reference returns them."""
        fb, fo = pack_strings(filters)
        tb, to = pack_strings(topics)
        pf = np.ascontiguousarray(pair_filter, np.uint32)
        pt = np.ascontiguousarray(pair_topic, np.uint32)
        n = len(pf)
        rp = C.POINTER(AclResult)()
        _check(lib().mq_acl_match_batch(self.h, _p(fb, _u8p), _p(fo, _u64p), len(filters), _p(tb, _u8p),
                                        _p(to, _u64p), len(topics), _p(pf, _u32p), _p(pt, _u32p), n,
                                        C.byref(rp)), "mq_acl_match_batch")
        try:
            r = rp.contents
            def arr(ptr, count, dtype):
                if count == 0 or not ptr:
                    return np.zeros(0, dtype)
                buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
                return np.frombuffer(buf, dtype).copy()
            matched = arr(r.matched, n, np.uint8)
            n_el = arr(r.n_elems, n, np.uint32)
            base = arr(r.elem_base, n, np.uint64)
            total = int((base[-1] + n_el[-1])) if n else 0
            spans = arr(r.elems, 2 * max(total, 1), np.uint32)
        finally:
            lib().mq_result_free(rp)
        raw = [_b(t) for t in topics]
        out = []
        for i in range(n):
            t = raw[int(pt[i])]
            els = [t[spans[2 * (int(base[i]) + k)]:spans[2 * (int(base[i]) + k)] + spans[2 * (int(base[i]) + k) + 1]]
                   .decode("utf-8", "surrogateescape") for k in range(int(n_el[i]))]
            out.append((els, bool(matched[i])))
        return out

    def profile(self, enable=True, work=False, walk_only=False):
        """mq_profile_enable: kernel times (HIP events); work=True adds k_merge's work counters;
        walk_only=True times the walk's launches alone (no events between the other kernels)."""
        mode = (PROF_TIMES | (PROF_WORK if work else 0) | (PROF_WALK if walk_only else 0)) if enable else 0
        _check(lib().mq_profile_enable(self.h, mode), "mq_profile_enable")

    def profile_read(self):
        arr = (KernelTime * 64)()
        n = _check(lib().mq_profile_read(self.h, arr, 64), "mq_profile_read")
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].total_ms)) for i in range(n)}

    def profile_reset(self):
        _check(lib().mq_profile_reset(self.h), "mq_profile_reset")


_TOPIC_SPANS_DT = np.dtype([("span_base", np.uint64), ("patch_base", np.uint64), ("inline_base", np.uint64),
                            ("picked_base", np.uint64), ("n_spans", np.uint32), ("n_patches", np.uint32),
                            ("n_inline", np.uint32), ("n_rows", np.uint32), ("n_client", np.uint32),
                            ("n_ident", np.uint32), ("n_shared", np.uint32), ("flags", np.uint32)])


def _span_arrays(r, n):
    """numpy copies of a host SpanResult's arrays."""
    def arr(ptr, count, dtype, width=None):
        shape = (count,) if width is None else (count, width)
        if count == 0 or not ptr:
            return np.zeros(shape, dtype)
        nbytes = count * np.dtype(dtype).itemsize * (width or 1)
        buf = (C.c_char * nbytes).from_address(ptr)
        return np.frombuffer(buf, dtype).reshape(shape).copy()
    codes = (int(r.flags) & SPANS_PATCH_CODES) != 0

    def patches(ptr, count, set_rows):
        if not codes:
            return arr(ptr, count, np.uint32, 2)
        # 4-byte patch codes (row << 3 | op): as (row, MQ_PATCH_OP | op), set rows as x << 26 | k
        c = arr(ptr, count, np.uint32)
        row = c >> 3
        if set_rows:
            row = ((row >> 23) << 26) | (row & ((1 << 23) - 1))
        return np.stack([row, PATCH_OP | (c & 7)], axis=1).astype(np.uint32) if count else np.zeros((0, 2), np.uint32)
    return {
        "topics": arr(r.topics, n, _TOPIC_SPANS_DT),
        "spans": arr(r.spans, int(r.n_spans), np.uint32, 4),
        "patches": patches(r.patches, int(r.n_patches), False),
        "inline": arr(r.inline_rows, int(r.n_inline_rows), np.uint32, 2),
        "picked": arr(r.picked_rows, int(r.n_picked_rows), np.uint32, 2),
        "flags": int(r.flags),
        "patch_codes": codes,
        "set_patches": patches(r.set_patches, int(r.n_set_patches), True),
        "merge_rows": arr(r.merge_rows, int(r.n_merge_rows), np.uint32),
        "merge_base": arr(r.merge_row_base, n if r.merge_row_base else 0, np.uint32),
    }


def host_topic_patches(a):
    """Every patch of a match_spans() dict as (topic, topic row, meta) arrays: the topics' own
    patches and, for MQ_TOPIC_SET_PATCHES topics, their merge set's patches with rows translated
    through the topic's packed merge rows (include/mqmatch.h mq_topic_patch)."""
    t = a["topics"]
    n = len(t)
    setf = (t["flags"] & 1) != 0
    tids, rows, metas = [], [], []
    for own in (True, False):
        sel = ~setf if own else setf
        tid = np.repeat(np.arange(n)[sel], t["n_patches"][sel].astype(np.int64))
        pr = (a["patches"] if own else a["set_patches"])[_ranges(t["patch_base"][sel], t["n_patches"][sel])]
        row = pr[:, 0].astype(np.int64)
        if not own and len(row):
            row = a["merge_rows"][a["merge_base"][tid].astype(np.int64) + (row >> 26)].astype(np.int64) \
                + (row & ((1 << 26) - 1))
        tids.append(tid)
        rows.append(row)
        metas.append(pr[:, 1])
    return np.concatenate(tids), np.concatenate(rows), np.concatenate(metas)


def _expand_host_spans(rp, n):
    """Expand a host SpanResult (then freed) into match_batch()'s dict via mq_spans_expand."""
    try:
        r = rp.contents
        a = _span_arrays(r, n)
        t = a["topics"]
        n_rows, n_shared = t["n_rows"].astype(np.uint64), t["n_shared"].astype(np.uint64)
        rows = np.zeros((max(int(n_rows.sum()), 1), 4), np.uint32)
        shared = np.zeros((max(int(n_shared.sum()), 1), 2), np.uint32)
        nr, ns = C.c_uint64(), C.c_uint64()
        _check(lib().mq_spans_expand(rp, 0, n, rows.ctypes.data, len(rows), shared.ctypes.data, len(shared),
                                     C.byref(nr), C.byref(ns)), "mq_spans_expand")
    finally:
        lib().mq_result_free(rp)
    excl = lambda c: np.concatenate(([0], np.cumsum(c)[:-1])).astype(np.uint64) if len(c) else np.zeros(0, np.uint64)
    return {
        "sub_base": excl(n_rows), "shared_base": excl(n_shared), "inline_base": t["inline_base"].copy(),
        "sub_cap": t["n_rows"].copy(), "n_client": t["n_client"].copy(), "n_ident": t["n_ident"].copy(),
        "n_shared": t["n_shared"].copy(), "n_inline": t["n_inline"].copy(),
        "rows": rows[:int(nr.value)], "shared": shared[:int(ns.value)], "inline": a["inline"],
        "n_patches": int(t["n_patches"].sum()), "n_spans": int(t["n_spans"].sum()),
    }


def _ranges(starts, counts):
    """Concatenated index ranges [starts[i], starts[i] + counts[i])."""
    counts = np.asarray(counts, np.int64)
    total = int(counts.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    rep = np.repeat(np.asarray(starts, np.int64) - np.concatenate(([0], np.cumsum(counts)[:-1])), counts)
    return rep + np.arange(total, dtype=np.int64)


def expand_device_spans(r, n, count=None):
    """Expand a DEVICE span result of n topics (mq_match_spans_device; r: SpanResult of device
    pointers) into match_batch()'s dict on the host, for its first `count` topics (default all):
    every topic's spans' records with its patches applied — per-topic patches, or set-shared ones
    (MQ_TOPIC_SET_PATCHES) translated through the topic's merge rows. What a device consumer of
    the format does; used by the tests and bench.py's parity sample."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipDeviceSynchronize.argtypes = []
    assert hip.hipDeviceSynchronize() == 0

    def d2h(ptr, count, dtype, width=1):
        out = np.zeros((count, width), dtype) if width > 1 else np.zeros(count, dtype)
        if count and ptr:
            assert hip.hipMemcpy(out.ctypes.data, ptr, out.nbytes, 2) == 0  # hipMemcpyDeviceToHost
        return out
    count = n if count is None else min(count, n)
    t = d2h(r.topics, 64 * count, np.uint8).view(_TOPIC_SPANS_DT)
    n = count
    # a topic's spans are contiguous at span_base (topics in order; one-sync batches place topic t's
    # at t * 64, the walk-fused desc's stride layout)
    sb, ns = t["span_base"].astype(np.int64), t["n_spans"].astype(np.int64)
    n_sp = int((sb + ns).max()) if n else 0
    spans = d2h(r.spans, n_sp, np.uint32, 4)[_ranges(sb, ns)]
    pool = d2h(r.sub_pool, int(r.sub_pool_len), np.uint32, 4)
    spool = d2h(r.shared_pool, int(r.shared_pool_len), np.uint32, 2)
    patches = d2h(r.patches, int(r.n_patches), np.uint32, 2)
    sets = d2h(r.set_patches, int(r.n_set_patches), np.uint32, 2)
    mrows = d2h(r.merge_rows, 64 * n if r.merge_rows else 0, np.uint32)
    inl = d2h(r.inline_rows, int(r.n_inline_rows), np.uint32, 2)
    excl = lambda c: np.concatenate(([0], np.cumsum(c)[:-1])).astype(np.uint64) if len(c) else np.zeros(0, np.uint64)
    rows = pool[_ranges(spans[:, 0], spans[:, 1])].copy() if len(spans) else np.zeros((0, 4), np.uint32)
    shared = spool[_ranges(spans[:, 2], spans[:, 3])] if len(spans) else np.zeros((0, 2), np.uint32)
    sub_base = excl(t["n_rows"].astype(np.uint64))
    setf = (t["flags"] & 1) != 0
    for own in (True, False):
        sel = ~setf if own else setf
        tid = np.repeat(np.arange(n)[sel], t["n_patches"][sel].astype(np.int64))
        src = patches if own else sets
        pr = src[_ranges(t["patch_base"][sel], t["n_patches"][sel])]
        row = pr[:, 0].astype(np.int64)
        if not own:
            row = mrows[tid * 64 + (row >> 26)].astype(np.int64) + (row & ((1 << 26) - 1))
        rows[sub_base[tid].astype(np.int64) + row, 3] = pr[:, 1]
    return {
        "sub_base": sub_base, "shared_base": excl(t["n_shared"].astype(np.uint64)),
        "inline_base": t["inline_base"].copy(), "sub_cap": t["n_rows"].copy(), "n_client": t["n_client"].copy(),
        "n_ident": t["n_ident"].copy(), "n_shared": t["n_shared"].copy(), "n_inline": t["n_inline"].copy(),
        "rows": rows, "shared": shared, "inline": inl, "set_topics": int(setf.sum()),
        "n_patches": int(t["n_patches"].sum()), "n_spans": int(t["n_spans"].sum()),
    }


def device_messages(r, n):
    """Copy a DEVICE Messages result of n filters (mq_messages_device; r: MsgResult of device
    pointers) to the host: (base u64[n], count u32[n], handles u64[n_handles])."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipDeviceSynchronize() == 0
    base, count = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    hs = np.zeros(int(r.n_handles), np.uint64)
    for a, p in ((base, r.base), (count, r.count), (hs, r.handles)):
        if a.nbytes and p:
            assert hip.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return base, count, hs


def device_messages_runs(r, n):
    """Copy a DEVICE Messages runs result (mq_messages_runs_device) to the host: a dict as
    Engine.messages_runs_batch returns (the handle array the runs index copied whole)."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipDeviceSynchronize() == 0
    out = {"run_base": np.zeros(n, np.uint64), "n_runs": np.zeros(n, np.uint32), "base": np.zeros(n, np.uint64),
           "count": np.zeros(n, np.uint32), "runs": np.zeros(int(r.n_runs_total), MSG_RUN_DT),
           "handles": np.zeros(int(r.n_handles), np.uint64), "n_expanded": int(r.n_expanded)}
    for k, p in (("run_base", r.run_base), ("n_runs", r.n_runs), ("base", r.base), ("count", r.count),
                 ("runs", r.runs), ("handles", r.handles)):
        a = out[k]
        if a.nbytes and p:
            assert hip.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


ROW_IDENT = 0x40000000  # MQ_ROW_IDENT (include/mqmatch.h)
ROW_DROP = 0x80000000   # MQ_ROW_DROP
ROW_KIND_MASK = 0xC0000000


def topic_rows(res, t):
    """Row views of topic t from a match_batch() dict: (client rows, ident rows, shared rows,
    inline rows). Client and ident rows are picked out of the topic's row region by kind."""
    b, cap = int(res["sub_base"][t]), int(res["sub_cap"][t])
    sb, ns = int(res["shared_base"][t]), int(res["n_shared"][t])
    ib, nl = int(res["inline_base"][t]), int(res["n_inline"][t])
    region = res["rows"][b:b + cap]
    kind = region[:, 3] & ROW_KIND_MASK
    return (region[kind == 0], region[kind == ROW_IDENT],
            res["shared"][sb:sb + ns], res["inline"][ib:ib + nl])


class TopicsIndex:
    """Mirror of the Go TopicsIndex (topics.go:349-698) over the engine's C-ABI."""

    def __init__(self, device=0, select_shared=False, fmt="spans"):
        """select_shared: SelectShared on the device (MQ_CFG_SELECT_SHARED) — each Shared[filter]
        holds only its picked member, for a broker with no OnSelectSubscribers hook.
        fmt: "spans" (mq_match_spans + mq_spans_expand, the default) or "rows" (mq_match_batch)."""
        if fmt not in ("spans", "rows"):
            raise ValueError(fmt)
        self.fmt = fmt
        self.engine = Engine(device, select_shared=select_shared)
        self.client_ids: Dict[str, int] = {}
        self.clients: List[str] = []
        self.filter_ids: Dict[str, int] = {}
        self.filters: List[str] = []
        self.stored: Dict[tuple, Subscription] = {}  # (client, filter) -> stored subscription
        self.inline_stored: Dict[tuple, InlineSubscription] = {}
        self.handles: Dict[int, object] = {}
        self._next_handle = 1

    def _cid(self, c):
        if c not in self.client_ids:
            self.client_ids[c] = len(self.clients)
            self.clients.append(c)
        return self.client_ids[c]

    def _fid(self, f):
        if f not in self.filter_ids:
            self.filter_ids[f] = len(self.filters)
            self.filters.append(f)
        return self.filter_ids[f]

    def subscribe(self, client: str, sub: Subscription) -> bool:  # topics.go:401
        flags = (1 if sub.no_local else 0) | (2 if sub.retain_as_published else 0) | \
                ((sub.retain_handling & 3) << 2)
        r = self.engine.subscribe(sub.filter, self._cid(client), self._fid(sub.filter), sub.qos,
                                  flags, sub.identifier)
        self.stored[(client, sub.filter)] = Subscription(
            sub.filter, sub.identifier, sub.qos, sub.no_local, sub.retain_as_published,
            sub.retain_handling)
        return r == 1

    def unsubscribe(self, filter: str, client: str) -> bool:  # topics.go:423
        return self.engine.unsubscribe(filter, self._cid(client)) == 1

    def inline_subscribe(self, sub: InlineSubscription) -> bool:  # topics.go:368
        r = self.engine.inline_subscribe(sub.filter, sub.identifier, self._fid(sub.filter))
        self.inline_stored[(sub.identifier, sub.filter)] = sub
        return r == 1

    def inline_unsubscribe(self, identifier: int, filter: str) -> bool:  # topics.go:382
        return self.engine.inline_unsubscribe(filter, identifier) == 1

    def retain_message(self, topic: str, payload: bytes, retain: bool = True, packet=None) -> int:
        h = self._next_handle          # topics.go:453
        self._next_handle += 1
        self.handles[h] = packet if packet is not None else (topic, payload)
        return self.engine.retain_message(topic, h, len(payload), retain)

    def messages(self, filter: str):  # topics.go:525 — retained handles (set semantics)
        return self.messages_batch([filter])[0]

    def messages_batch(self, filters):
        raw, offs = pack_strings(filters)
        base, count, hs = self.engine.messages_batch(raw, offs)
        return [sorted(int(x) for x in hs[int(base[i]):int(base[i]) + int(count[i])])
                for i in range(len(filters))]

    def subscribers(self, topic: str) -> Subscribers:  # topics.go:583
        return self.subscribers_batch([topic])[0]

    def subscribers_batch(self, topics) -> List[Subscribers]:
        """The batching stage's entry point: one engine call for many topics."""
        raw, offs = pack_strings(topics)
        if self.fmt == "spans":
            res = self.engine.match_batch_spans(raw, offs)
        else:
            res = self.engine.match_batch(raw, offs)
        return [self._rebuild(res, t) for t in range(len(topics))]

    def _rebuild(self, res, t) -> Subscribers:
        cli, idn, shr, inl = topic_rows(res, t)
        out = Subscribers()
        for c, f, ident, meta in cli:
            client, filt = self.clients[int(c)], self.filters[int(f)]
            base = self.stored[(client, filt)]
            s = Subscription(filt, int(np.int32(ident)), int(meta) & META_QOS,
                             bool(int(meta) & META_NOLOCAL), bool(int(meta) & META_RAP),
                             (int(meta) >> META_RH_SHIFT) & 3, {filt: int(np.int32(ident))})
            assert base.identifier == s.identifier
            out.subscriptions[client] = s
        for c, f, ident, _ in idn:
            out.subscriptions[self.clients[int(c)]].identifiers[self.filters[int(f)]] = int(np.int32(ident))
        for f, c in shr:
            client, filt = self.clients[int(c)], self.filters[int(f)]
            out.shared.setdefault(filt, {})[client] = self.stored[(client, filt)]
        for ident, f in inl:
            out.inline_subscriptions[int(np.int32(ident))] = InlineSubscription(
                self.filters[int(f)], int(np.int32(ident)))
        return out
