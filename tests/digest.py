"""Per-topic digests of the engine's result rows, computed exactly as the oracle computes them
from its Go-shaped maps (oracle/oracle_capi.cpp digest_subscribers): per row category the count
and the wrapping u64 sum of row hashes, folded together. Test infrastructure."""
import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
SEED = np.uint64(0x6D716D61)


def mix64(x):
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x


def fold(h, v):
    with np.errstate(over="ignore"):
        return mix64(np.asarray(h, np.uint64) ^ mix64(np.asarray(v, np.uint64) + GOLD))


def row_hash(cat, a, b, c, d):
    return fold(fold(fold(fold(np.uint64(cat), a), b), c), d)


def _ranges(starts, counts):
    """Concatenated index ranges [starts[i], starts[i]+counts[i])."""
    counts = counts.astype(np.int64)
    total = int(counts.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    rep = np.repeat(starts.astype(np.int64) - np.concatenate(([0], np.cumsum(counts)[:-1])), counts)
    return rep + np.arange(total, dtype=np.int64)


def _seg_sums(h, counts):
    c = np.concatenate(([np.uint64(0)], np.cumsum(h, dtype=np.uint64))).astype(np.uint64)
    ends = np.cumsum(counts.astype(np.int64))
    starts = ends - counts.astype(np.int64)
    with np.errstate(over="ignore"):
        return c[ends] - c[starts]


def engine_digests(res):
    """res: Engine.match_batch() dict -> (digests u64[n], counts u32[n,4])."""
    n = len(res["n_client"])
    rows = res["rows"].astype(np.uint64)
    base, cap = res["sub_base"].astype(np.int64), res["sub_cap"].astype(np.int64)
    nc, ni = res["n_client"].astype(np.int64), res["n_ident"].astype(np.int64)
    ci = _ranges(base, nc)
    ii = _ranges(base + cap - ni, ni)
    si = _ranges(res["shared_base"].astype(np.int64), res["n_shared"].astype(np.int64))
    li = _ranges(res["inline_base"].astype(np.int64), res["n_inline"].astype(np.int64))
    hc = row_hash(1, rows[ci, 0], rows[ci, 1], rows[ci, 2], rows[ci, 3])
    hi = row_hash(2, rows[ii, 0], rows[ii, 1], rows[ii, 2], 0)
    sh = res["shared"].astype(np.uint64)
    hs = row_hash(3, sh[si, 0], sh[si, 1], 0, 0)
    il = res["inline"].astype(np.uint64)
    hl = row_hash(4, il[li, 0], il[li, 1], 0, 0)
    d = np.full(n, SEED, np.uint64)
    counts = np.stack([nc, ni, res["n_shared"].astype(np.int64), res["n_inline"].astype(np.int64)], 1)
    for k, h in enumerate((hc, hi, hs, hl)):
        d = fold(fold(d, counts[:, k].astype(np.uint64)), _seg_sums(h, counts[:, k]))
    return d, counts.astype(np.uint32)
