"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle.so, the CPU restatement of the reference Go
`TopicsIndex` (/root/reference/topics.go:349-822, packets/packets.go:254-274). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module: it is the
checker, never the thing measured or shipped.

Parity pinning: the Go toolchain is absent here, so the restatement is pinned
by the reference's own known-answer tests transcribed in tests/test_oracle_kat.py.
"""
import ctypes as C
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(_HERE, "liboracle.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: run `make -C oracle`")
    L = C.CDLL(path)
    L.orc_new.restype = C.c_void_p
    L.orc_free.argtypes = [C.c_void_p]
    L.orc_subscribe.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32,
                                C.c_uint32, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int64]
    L.orc_unsubscribe.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
    L.orc_inline_subscribe.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int64, C.c_uint32]
    L.orc_inline_unsubscribe.argtypes = [C.c_void_p, C.c_int64, C.c_char_p, C.c_uint32]
    L.orc_retain_message.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                     C.c_uint8]
    L.orc_retain_message.restype = C.c_int64
    L.orc_retained_delete.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32]
    L.orc_retained_add.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint8]
    L.orc_retained_len.argtypes = [C.c_void_p]
    L.orc_retained_len.restype = C.c_uint64
    L.orc_particle_count.argtypes = [C.c_void_p]
    L.orc_particle_count.restype = C.c_uint64
    L.orc_subscribe_bulk.argtypes = [C.c_void_p, _u8p, _u64p, _u32p, _u32p, _u8p, _u8p, _i32p,
                                     C.c_uint64, _u8p]
    L.orc_retain_bulk.argtypes = [C.c_void_p, _u8p, _u64p, _u64p, C.c_uint64]
    L.orc_subscribers_json.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint64]
    L.orc_subscribers_json.restype = C.c_uint64
    L.orc_messages.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, _u64p, C.c_uint64]
    L.orc_messages.restype = C.c_uint64
    L.orc_digest_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p, _u32p,
                                   _u64p]
    L.orc_messages_digest_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32,
                                            _u64p, _u32p, _u64p]
    L.orc_bench_subscribers.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    L.orc_bench_subscribers.restype = C.c_double
    L.orc_bench_messages.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    L.orc_bench_messages.restype = C.c_double
    L.orc_isolate_particle.argtypes = [C.c_char_p, C.c_uint32, C.c_int, _u32p, _u32p]
    L.orc_is_valid_filter.argtypes = [C.c_char_p, C.c_uint32, C.c_int]
    L.orc_is_shared_filter.argtypes = [C.c_char_p, C.c_uint32]
    L.orc_match_topic.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, _u32p, C.c_uint32, _u32p]
    L.orc_equal_fold_ascii.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
    L.orc_path_exists.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int]
    L.orc_node_counts.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int, _i64p]
    L.orc_node_counts.restype = C.c_int64
    L.orc_fast_build.argtypes = [C.c_void_p]
    L.orc_fast_build.restype = C.c_void_p
    L.orc_fast_free.argtypes = [C.c_void_p]
    L.orc_fast_digest_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p, _u32p]
    L.orc_fast_bench.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    L.orc_fast_bench.restype = C.c_double
    L.orc_fast_msg_build.argtypes = [C.c_void_p]
    L.orc_fast_msg_build.restype = C.c_void_p
    L.orc_fast_msg_free.argtypes = [C.c_void_p]
    L.orc_fast_msg_digest_batch.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p, _u32p]
    L.orc_fast_msg_bench.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    L.orc_fast_msg_bench.restype = C.c_double
    L.orc_root_children.argtypes = [C.c_void_p]
    L.orc_root_children.restype = C.c_uint64
    L.orc_handle_digests.argtypes = [_u64p, _u32p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    L.orc_run_digests.argtypes = [_u64p, _u32p, _u32p, _u64p, C.c_uint64, C.c_uint32, _u64p]
    _LIB = L
    return L


def _b(s):
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def _ptr(a, t):
    return a.ctypes.data_as(t)


def isolate_particle(f, d):
    fb = _b(f)
    st, ln = C.c_uint32(), C.c_uint32()
    hn = lib().orc_isolate_particle(fb, len(fb), d, C.byref(st), C.byref(ln))
    return fb[st.value:st.value + ln.value].decode("utf-8", "surrogateescape"), bool(hn)


def is_valid_filter(f, for_publish):
    fb = _b(f)
    return bool(lib().orc_is_valid_filter(fb, len(fb), 1 if for_publish else 0))


def match_topic(filter, topic):
    """auth.MatchTopic (hooks/auth/ledger.go:90-118) -> (elements, matched)."""
    fb, tb = _b(filter), _b(topic)
    cap = len(fb) + 1
    el = np.zeros(2 * cap, np.uint32)
    n = C.c_uint32()
    m = lib().orc_match_topic(fb, len(fb), tb, len(tb), _ptr(el, _u32p), cap, C.byref(n))
    elems = [tb[el[2 * i]:el[2 * i] + el[2 * i + 1]].decode("utf-8", "surrogateescape") for i in range(n.value)]
    return elems, bool(m)


def is_shared_filter(f):
    fb = _b(f)
    return bool(lib().orc_is_shared_filter(fb, len(fb)))


def equal_fold(s, t):
    sb, tb = _b(s), _b(t)
    return bool(lib().orc_equal_fold_ascii(sb, len(sb), tb, len(tb)))


def handle_digests(base, count, handles, nthreads=8):
    """Per-filter digests of an engine Messages result (handles[base[i], + count[i]) in any
    order), computed as messages_digest_batch computes the oracle's."""
    n = len(count)
    base = np.ascontiguousarray(base, np.uint64)
    count = np.ascontiguousarray(count, np.uint32)
    handles = np.ascontiguousarray(handles, np.uint64)
    dig = np.zeros(n, np.uint64)
    lib().orc_handle_digests(_ptr(base, _u64p), _ptr(count, _u32p), _ptr(handles, _u64p), n, nthreads,
                             _ptr(dig, _u64p))
    return dig


def run_digests(res, nthreads=8):
    """Per-filter digests of an engine Messages runs result (a dict of run_base, n_runs, runs,
    handles: Engine.messages_runs_batch / engine.device_messages_runs), as handle_digests."""
    n = len(res["n_runs"])
    rb = np.ascontiguousarray(res["run_base"], np.uint64)
    nr = np.ascontiguousarray(res["n_runs"], np.uint32)
    runs = np.ascontiguousarray(res["runs"]).view(np.uint32)
    hs = np.ascontiguousarray(res["handles"], np.uint64)
    dig = np.zeros(n, np.uint64)
    lib().orc_run_digests(_ptr(rb, _u64p), _ptr(nr, _u32p), _ptr(runs, _u32p), _ptr(hs, _u64p), n, nthreads,
                          _ptr(dig, _u64p))
    return dig


class OracleIndex:
    """The reference TopicsIndex restated (topics.go:349). Clients/filters also carry u32 ids
    so digests can be compared with the engine's rows; ids default to interning order."""

    def __init__(self):
        self.h = lib().orc_new()
        self.client_ids = {}
        self.filter_ids = {}

    def close(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _cid(self, c):
        return self.client_ids.setdefault(c, len(self.client_ids))

    def _fid(self, f):
        return self.filter_ids.setdefault(f, len(self.filter_ids))

    def subscribe(self, client, filter, qos=0, identifier=0, no_local=False, rap=False, rh=0,
                  client_id=None, filter_id=None):
        cb, fb = _b(client), _b(filter)
        cid = self._cid(client) if client_id is None else client_id
        fid = self._fid(filter) if filter_id is None else filter_id
        flags = (1 if no_local else 0) | (2 if rap else 0) | ((rh & 3) << 2)
        return bool(lib().orc_subscribe(self.h, cb, len(cb), fb, len(fb), cid, fid, qos, flags,
                                        identifier))

    def unsubscribe(self, filter, client):
        fb, cb = _b(filter), _b(client)
        return bool(lib().orc_unsubscribe(self.h, fb, len(fb), cb, len(cb)))

    def inline_subscribe(self, filter, identifier, filter_id=None):
        fb = _b(filter)
        fid = self._fid(filter) if filter_id is None else filter_id
        return bool(lib().orc_inline_subscribe(self.h, fb, len(fb), identifier, fid))

    def inline_unsubscribe(self, identifier, filter):
        fb = _b(filter)
        return bool(lib().orc_inline_unsubscribe(self.h, identifier, fb, len(fb)))

    def retain_message(self, topic, handle, payload_len, retain=True):
        tb = _b(topic)
        return int(lib().orc_retain_message(self.h, tb, len(tb), handle, payload_len,
                                            1 if retain else 0))

    def retained_delete(self, topic):
        tb = _b(topic)
        lib().orc_retained_delete(self.h, tb, len(tb))

    def retained_add(self, topic, handle, payload_len=1, retain=True):  # Retained.Add
        tb = _b(topic)
        lib().orc_retained_add(self.h, tb, len(tb), handle, payload_len, 1 if retain else 0)

    def retained_len(self):
        return int(lib().orc_retained_len(self.h))

    def particle_count(self):
        return int(lib().orc_particle_count(self.h))

    def root_children(self):
        return int(lib().orc_root_children(self.h))

    def path_exists(self, filter, d=0):
        fb = _b(filter)
        return bool(lib().orc_path_exists(self.h, fb, len(fb), d))

    def node_counts(self, filter, d=0):
        """(children, subs, shared, inline, has_retain_path) of seek(filter, d), or None."""
        fb = _b(filter)
        out = (C.c_int64 * 5)()
        r = lib().orc_node_counts(self.h, fb, len(fb), d, out)
        return None if r < 0 else tuple(out)

    def subscribers(self, topic):
        """Canonical Subscribers(topic) as plain dicts (string keyed)."""
        tb = _b(topic)
        n = lib().orc_subscribers_json(self.h, tb, len(tb), None, 0)
        buf = C.create_string_buffer(int(n))
        lib().orc_subscribers_json(self.h, tb, len(tb), buf, n)
        return json.loads(buf.raw[:n].decode("utf-8", "surrogateescape"))

    def messages(self, filter):
        fb = _b(filter)
        n = lib().orc_messages(self.h, fb, len(fb), None, 0)
        out = (C.c_uint64 * max(int(n), 1))()
        lib().orc_messages(self.h, fb, len(fb), out, n)
        return sorted(out[i] for i in range(int(n)))

    # ---- columnar bulk paths (numpy arrays) ----
    def subscribe_bulk(self, w):
        n = len(w["client_ids"])
        out = np.zeros(n, np.uint8)
        lib().orc_subscribe_bulk(self.h, _ptr(w["bytes"], _u8p), _ptr(w["offs"], _u64p),
                                 _ptr(w["client_ids"], _u32p), _ptr(w["filter_ids"], _u32p),
                                 _ptr(w["qos"], _u8p), _ptr(w["flags"], _u8p),
                                 _ptr(w["idents"], _i32p), n, _ptr(out, _u8p))
        return out

    def retain_bulk(self, bytes_, offs, handles):
        n = len(offs) - 1
        lib().orc_retain_bulk(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p),
                              _ptr(handles, _u64p), n)

    def digest_batch(self, bytes_, offs, nthreads=8):
        n = len(offs) - 1
        dig = np.zeros(n, np.uint64)
        cnt = np.zeros(n * 4, np.uint32)
        tot = np.zeros(4, np.uint64)
        lib().orc_digest_batch(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n, nthreads,
                               _ptr(dig, _u64p), _ptr(cnt, _u32p), _ptr(tot, _u64p))
        return dig, cnt.reshape(n, 4), dict(zip("LPSO", (int(x) for x in tot)))

    def messages_digest_batch(self, bytes_, offs, nthreads=8):
        n = len(offs) - 1
        dig = np.zeros(n, np.uint64)
        cnt = np.zeros(n, np.uint32)
        tot = np.zeros(4, np.uint64)
        lib().orc_messages_digest_batch(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n,
                                        nthreads, _ptr(dig, _u64p), _ptr(cnt, _u32p),
                                        _ptr(tot, _u64p))
        return dig, cnt, dict(zip("LPSO", (int(x) for x in tot)))

    def bench_subscribers(self, bytes_, offs, nthreads):
        n = len(offs) - 1
        sink = C.c_uint64()
        secs = lib().orc_bench_subscribers(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n,
                                           nthreads, C.byref(sink))
        return float(secs), int(sink.value)

    def fast(self):
        """FastIndex snapshot of this index (topics_fast.h): the CPU baseline's restatement."""
        return FastIndex(self)

    def fast_messages(self):
        """FastMsgIndex snapshot of this index (topics_fast.h): bench_messages.py's CPU baseline."""
        return FastMsgIndex(self)

    def bench_messages(self, bytes_, offs, nthreads):
        n = len(offs) - 1
        sink = C.c_uint64()
        secs = lib().orc_bench_messages(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n,
                                        nthreads, C.byref(sink))
        return float(secs), int(sink.value)


class FastIndex:
    """The fast CPU restatement (oracle/topics_fast.h) over a frozen OracleIndex: flat result
    tables per thread, interned client ids. bench.py's cpu_baseline; digest-checked against the
    oracle in tests/test_oracle_kat.py."""

    def __init__(self, orc):
        self.h = lib().orc_fast_build(orc.h)

    def close(self):
        if self.h:
            lib().orc_fast_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def digest_batch(self, bytes_, offs, nthreads=8):
        n = len(offs) - 1
        dig = np.zeros(n, np.uint64)
        cnt = np.zeros(n * 4, np.uint32)
        lib().orc_fast_digest_batch(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n, nthreads,
                                    _ptr(dig, _u64p), _ptr(cnt, _u32p))
        return dig, cnt.reshape(n, 4)

    def bench_subscribers(self, bytes_, offs, nthreads):
        n = len(offs) - 1
        sink = C.c_uint64()
        secs = lib().orc_fast_bench(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n, nthreads, C.byref(sink))
        return float(secs), int(sink.value)


class FastMsgIndex:
    """The fast CPU restatement of Messages (oracle/topics_fast.h) over a frozen OracleIndex:
    bench_messages.py's cpu_baseline; digest-checked against the oracle in tests/test_oracle_kat.py."""

    def __init__(self, orc):
        self.orc = orc  # (it reads the oracle's retained map for filters without wildcards)
        self.h = lib().orc_fast_msg_build(orc.h)

    def close(self):
        if self.h:
            lib().orc_fast_msg_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def digest_batch(self, bytes_, offs, nthreads=8):
        n = len(offs) - 1
        dig = np.zeros(n, np.uint64)
        cnt = np.zeros(n, np.uint32)
        lib().orc_fast_msg_digest_batch(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n, nthreads,
                                        _ptr(dig, _u64p), _ptr(cnt, _u32p))
        return dig, cnt

    def bench_messages(self, bytes_, offs, nthreads):
        n = len(offs) - 1
        sink = C.c_uint64()
        secs = lib().orc_fast_msg_bench(self.h, _ptr(bytes_, _u8p), _ptr(offs, _u64p), n, nthreads, C.byref(sink))
        return float(secs), int(sink.value)
