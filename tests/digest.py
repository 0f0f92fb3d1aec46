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
    counts, sums = engine_digest_parts(res)
    return fold_parts(counts, sums), counts.astype(np.uint32)


def fold_parts(counts, sums):
    """Per-topic digest from per-category row counts and wrapping sums of row hashes (the parts
    of disjoint results, e.g. the shards of a sharded index, add up)."""
    d = np.full(len(counts), SEED, np.uint64)
    for k in range(4):
        d = fold(fold(d, counts[:, k].astype(np.uint64)), sums[:, k].astype(np.uint64))
    return d


def engine_digest_parts(res):
    """res: Engine.match_batch() dict -> (counts i64[n,4], sums u64[n,4]) per row category."""
    n = len(res["n_client"])
    rows = res["rows"].astype(np.uint64)
    base, cap = res["sub_base"].astype(np.int64), res["sub_cap"].astype(np.int64)
    nc, ni = res["n_client"].astype(np.int64), res["n_ident"].astype(np.int64)
    # every gathered record leaves one row in [base, base + cap): client rows (kind 0), ident
    # rows (MQ_ROW_IDENT) and dropped rows (MQ_ROW_DROP), in gather order
    ri = _ranges(base, cap)
    kind = rows[ri, 3] >> np.uint64(30)
    zero = np.uint64(0)
    hc = np.where(kind == 0, row_hash(1, rows[ri, 0], rows[ri, 1], rows[ri, 2], rows[ri, 3]), zero)
    hi = np.where(kind == 1, row_hash(2, rows[ri, 0], rows[ri, 1], rows[ri, 2], 0), zero)
    k_c = _seg_sums((kind == 0).astype(np.uint64), cap)
    k_i = _seg_sums((kind == 1).astype(np.uint64), cap)
    assert (k_c == nc.astype(np.uint64)).all() and (k_i == ni.astype(np.uint64)).all(), \
        "row kinds disagree with n_client / n_ident"
    si = _ranges(res["shared_base"].astype(np.int64), res["n_shared"].astype(np.int64))
    li = _ranges(res["inline_base"].astype(np.int64), res["n_inline"].astype(np.int64))
    sh = res["shared"].astype(np.uint64)
    hs = row_hash(3, sh[si, 0], sh[si, 1], 0, 0)
    il = res["inline"].astype(np.uint64)
    hl = row_hash(4, il[li, 0], il[li, 1], 0, 0)
    counts = np.stack([nc, ni, res["n_shared"].astype(np.int64), res["n_inline"].astype(np.int64)], 1)
    sums = np.stack([_seg_sums(hc, cap), _seg_sums(hi, cap), _seg_sums(hs, counts[:, 2]), _seg_sums(hl, counts[:, 3])],
                    1).astype(np.uint64)
    return counts, sums
