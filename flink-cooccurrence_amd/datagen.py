"""Seeded synthetic interaction logs for BASELINE.json's configs.

All generators use numpy PCG64 and return a CSR of per-user histories in arrival order:
``user_ptr`` int64[U+1], ``items`` int32[N] and, for streaming configs, ``ts`` int64[N] (event time
in ms, the `user,item,timestamp` schema of Configuration.java:59 / FlinkCooccurrences.java:207-217).
There is no network: these stand in for MovieLens / click logs of the same shape.
"""
from __future__ import annotations

import numpy as np


def _zipf_cdf(M: int, s: float) -> np.ndarray:
    w = 1.0 / np.power(np.arange(1, M + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    return c / c[-1]


def _draw(rng, cdf: np.ndarray, n: int) -> np.ndarray:
    return np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), len(cdf) - 1).astype(np.int32)


def ordered_pairs(user_ptr: np.ndarray) -> int:
    """P = sum_u n_u (n_u - 1): the reference's ObservedCooccurrences unit (NonSampled...java:153)."""
    n = np.diff(np.asarray(user_ptr, np.int64))
    return int(np.sum(n * (n - 1)))


def zipf_with_replacement(rng, lens: np.ndarray, M: int, s: float) -> np.ndarray:
    return _draw(rng, _zipf_cdf(M, s), int(lens.sum()))


def zipf_without_replacement(rng, lens: np.ndarray, M: int, s: float) -> np.ndarray:
    """Distinct items per user, drawn from Zipf(s) by rejection of duplicates (rating-log shape).

    Rounds only touch the users that still lack items; a user that overshoots keeps a random
    subset of its distinct draws."""
    cdf = _zipf_cdf(M, s)
    U = len(lens)
    lens = np.asarray(lens, np.int64)
    if np.any(lens > M):
        raise ValueError("a user cannot rate more distinct items than exist")
    done = []
    carry = np.zeros(0, np.int64)          # sorted keys (user * M + item) of unfinished users
    act = np.arange(U, dtype=np.int64)     # unfinished users
    have = np.zeros(U, np.int64)
    rnd = 0
    while len(act):
        need = lens[act] - have[act]
        draw = (need * (1.3 + 0.7 * rnd) + 8).astype(np.int64)
        users = np.repeat(act, draw)
        keys = np.unique(np.concatenate([carry, users * M + _draw(rng, cdf, len(users))]))
        owner = keys // M
        # trim overshoot: a user with more distinct draws than lens[u] keeps a random subset
        cnt = np.bincount(owner, minlength=U)
        over = cnt[owner] > lens[owner]
        if over.any():
            ok, ko = keys[~over], keys[over]
            oo = ko // M
            order = np.argsort((oo << 24) | rng.integers(0, 1 << 24, len(ko)), kind="stable")
            ko, oo = ko[order], oo[order]
            first = np.searchsorted(oo, oo, side="left")
            ko = ko[(np.arange(len(ko)) - first) < lens[oo]]
            keys = np.sort(np.concatenate([ok, ko]))
            owner = keys // M
        cnt = np.bincount(owner, minlength=U)
        have[act] = cnt[act]
        complete = cnt[owner] >= lens[owner]
        done.append(keys[complete])
        carry = np.sort(keys[~complete])
        act = act[have[act] < lens[act]]
        rnd += 1
    keys = np.concatenate(done) if done else np.zeros(0, np.int64)
    owner = keys // M
    # arrival order inside each user: random permutation
    order = np.argsort((owner << 24) | rng.integers(0, 1 << 24, len(keys)))
    return (keys[order] % M).astype(np.int32)


def config_c1(seed: int = 1, U: int = 10_000, M: int = 1_000, mean: float = 20.0, window_ms: int = 1000):
    """C1, the reference MiniCluster config: click log, Poisson(20) items/user, Zipf(1.0) with
    replacement, strictly ascending ms timestamps over a random interleave of users, 1 s windows."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.maximum(rng.poisson(mean, U), 1).astype(np.int64)
    items = zipf_with_replacement(rng, lens, M, 1.0)
    user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    # arrival: a random interleave of the users' streams, one interaction per ms.  Slot k of the
    # arrival sequence belongs to user seq_owner[k]; user u's i-th interaction (CSR order) takes u's
    # i-th slot, so grouping the slots by user (stable) lists the CSR timestamps in order.
    owner = np.repeat(np.arange(U, dtype=np.int64), lens)
    seq_owner = owner[rng.permutation(len(owner))]
    ts_csr = np.argsort(seq_owner, kind="stable").astype(np.int64)
    return dict(user_ptr=user_ptr, items=items, ts=ts_csr, n_items=M, window_ms=window_ms,
                name="C1 click log 10k users x 1k items", seed=seed)


def lognormal_lengths(rng, U: int, N: int, floor: int, cap: int, sigma: float = 1.0) -> np.ndarray:
    """n_u = max(floor, lognormal) rescaled so that sum n_u == N exactly, each in [floor, cap]."""
    x = rng.lognormal(0.0, sigma, U)
    lens = np.maximum(floor, np.round(x * (N / x.sum()))).astype(np.int64)
    for _ in range(64):
        lens = np.clip(np.round(floor + (lens - floor) * ((N - floor * U) / max(1, (lens - floor).sum()))), floor,
                       cap).astype(np.int64)
        if abs(int(lens.sum()) - N) < U:
            break
    diff = N - int(lens.sum())
    while diff != 0:
        step = 1 if diff > 0 else -1
        ok = np.nonzero((lens + step >= floor) & (lens + step <= cap))[0]
        pick = rng.choice(ok, size=min(abs(diff), len(ok)), replace=False)
        lens[pick] += step
        diff = N - int(lens.sum())
    return lens


def config_c2(seed: int = 2, U: int = 138_493, M: int = 26_744, N: int = 20_000_263, s: float = 0.9,
              floor: int = 20, cap: int = 5_000):
    """C2, MovieLens-20M-shaped: n_u = max(20, lognormal) rescaled to exactly N; Zipf(0.9) items
    without replacement per user (ratings are unique); one window."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = lognormal_lengths(rng, U, N, floor, min(cap, M))
    items = zipf_without_replacement(rng, lens, M, s)
    user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return dict(user_ptr=user_ptr, items=items, ts=None, n_items=M, window_ms=None,
                name="C2 MovieLens-20M-shaped 138,493 users x 26,744 items, 20,000,263 interactions", seed=seed)


def config_c3(seed: int = 3, U: int = 10_000_000, M: int = 1_000_000, N: int = 1_000_000_000, shard: int = 0,
              n_shards: int = 1, cap: int = 10_000):
    """C3, Zipf-skewed 1B log: n_u ~ lognormal(sigma=1) scaled to mean N/U and capped at 10,000; items
    Zipf(1.0) with replacement.  `shard`/`n_shards` generate one contiguous user shard (seed 3 +
    shard) so that each rank of a multi-GPU run materialises only its own users."""
    rng = np.random.Generator(np.random.PCG64(seed + shard))
    Us = U // n_shards + (1 if shard < U % n_shards else 0)
    Ns = int(round(N * Us / U))
    lens = lognormal_lengths(rng, Us, Ns, 1, cap)
    items = zipf_with_replacement(rng, lens, M, 1.0)
    user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return dict(user_ptr=user_ptr, items=items, ts=None, n_items=M, window_ms=None,
                name=f"C3 Zipf 1B: shard {shard}/{n_shards} ({Us} users, {Ns} interactions, 1e6 items)", seed=seed + shard)


# ---- C3, shard-invariant: every user's list is a pure function of (seed, user id) -----------------
# The generator above draws users sequentially from one PCG64 stream, so a 1-GPU run and an 8-GPU
# run would process different logs.  c3_users(u0, u1) instead derives user u's length and items from
# a counter-based hash (splitmix64 of (seed, u) and of (seed, u, j)), so any user range of the same
# 1B log can be materialised on its own, on the host (numpy) or on a GPU (torch), bit-identically.
#   n_u   = LEN_TABLE[top 16 bits of h(seed, u)]: 65,536 quantiles of lognormal(sigma = 1) scaled to a
#           mean of 100, capped at 10,000;
#   x_uj  = the item of rank searchsorted(Zipf(1.0) CDF over 1e6 items, uniform53(h(seed, u, j))).
C3_USERS, C3_ITEMS, C3_SEED = 10_000_000, 1_000_000, 3
_M64 = (1 << 64) - 1
_GOLD, _MIX1, _MIX2 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
_c3_cache: dict = {}


def _c3_tables(M: int = C3_ITEMS, mean: float = 100.0, cap: int = 10_000, sigma: float = 1.0):
    key = (M, mean, cap, sigma)
    if key not in _c3_cache:
        from scipy.special import ndtri

        q = (np.arange(65536, dtype=np.float64) + 0.5) / 65536.0
        lens = np.clip(np.round(np.exp(sigma * ndtri(q)) * (mean / np.exp(0.5 * sigma * sigma))), 1, cap)
        _c3_cache[key] = (lens.astype(np.int64), _zipf_cdf(M, 1.0))
    return _c3_cache[key]


def _splitmix_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(_GOLD)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_MIX1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_MIX2)
        return z ^ (z >> np.uint64(31))


def _i64(c: int) -> int:  # a uint64 constant as the int64 with the same bits
    return c - (1 << 64) if c >= 1 << 63 else c


def _splitmix_torch(x):
    import torch

    def srl(z, k):  # logical shift right of an int64 tensor
        return (z >> k) & ((1 << (64 - k)) - 1)

    z = x + _i64(_GOLD)
    z = (z ^ srl(z, 30)) * _i64(_MIX1)
    z = (z ^ srl(z, 27)) * _i64(_MIX2)
    return z ^ srl(z, 31)


def c3_lengths(u0: int, u1: int, seed: int = C3_SEED, device=None):
    """History lengths of users [u0, u1) of the shard-invariant C3 log."""
    lens_t, _ = _c3_tables()
    if device is None:
        h = _splitmix_np((np.arange(u0, u1, dtype=np.uint64) ^ np.uint64(seed << 40)))
        return lens_t[(h >> np.uint64(48)).astype(np.int64)]
    import torch

    h = _splitmix_torch(torch.arange(u0, u1, dtype=torch.int64, device=device) ^ (seed << 40))
    return torch.as_tensor(lens_t, device=device)[(h >> 48) & 0xFFFF]


C3_PERM_SEED = 0xC3B1  # the item-id bijection of the permuted C3 log (c3_item_perm)


def c3_item_perm(M: int = C3_ITEMS, seed: int = C3_PERM_SEED) -> np.ndarray:
    """A fixed bijection of [0, M) (numpy PCG64(seed).permutation): the permuted C3 log names the item
    of Zipf rank r as perm[r], so item ids carry no popularity order (MovieLens / hashed ids)."""
    key = ("perm", M, seed)
    if key not in _c3_cache:
        _c3_cache[key] = np.random.Generator(np.random.PCG64(seed)).permutation(M).astype(np.int32)
    return _c3_cache[key]


def c3_users(u0: int, u1: int, seed: int = C3_SEED, device=None, permute: bool = False):
    """CSR (user_ptr int64[U+1], items int32[N]) of users [u0, u1) of the shard-invariant C3 log:
    numpy arrays when device is None, else torch tensors built on that device.  permute: every item id
    x becomes c3_item_perm()[x] (same log, ids not in popularity order)."""
    lens = c3_lengths(u0, u1, seed, device)
    _, cdf = _c3_tables()
    if device is None:
        user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        owner = np.repeat(np.arange(u0, u1, dtype=np.uint64), lens)
        j = np.arange(int(user_ptr[-1]), dtype=np.int64) - np.repeat(user_ptr[:-1], lens)
        h = _splitmix_np(((owner << np.uint64(14)) | j.astype(np.uint64)) ^ np.uint64((seed << 58) | 0x5A5A))
        x = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        items = np.minimum(np.searchsorted(cdf, x, side="right"), len(cdf) - 1).astype(np.int32)
        if permute:
            items = c3_item_perm(len(cdf))[items]
        return user_ptr, items
    import torch

    user_ptr = torch.zeros(u1 - u0 + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=user_ptr[1:])
    n = int(user_ptr[-1].item())
    owner = torch.repeat_interleave(torch.arange(u0, u1, dtype=torch.int64, device=device), lens, output_size=n)
    j = torch.arange(n, dtype=torch.int64, device=device) - torch.repeat_interleave(user_ptr[:-1], lens, output_size=n)
    h = _splitmix_torch(((owner << 14) | j) ^ ((seed << 58) | 0x5A5A))
    del owner, j
    x = ((h >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / 9007199254740992.0)
    del h
    cdf_t = torch.as_tensor(cdf, device=device)
    items = torch.clamp(torch.searchsorted(cdf_t, x, right=True), max=len(cdf) - 1)
    if permute:
        items = torch.as_tensor(c3_item_perm(len(cdf)), device=device)[items]
    return user_ptr, items.to(torch.int32)


def c3_log_device(device, u1: int = C3_USERS, shard: int = C3_USERS // 8, seed: int = C3_SEED, permute: bool = False):
    """Users [0, u1) of the C3 log as one device CSR, generated shard by shard (bounded temporaries): the state of
    every rank of an N-GPU run after the histories' all-gather (u1 = C3_USERS: the whole 1B log, 4 GB of ids)."""
    import torch

    ups, its, base = [], [], 0
    for a in range(0, u1, shard):
        up, it = c3_users(a, min(u1, a + shard), seed, device=device, permute=permute)
        ups.append(up[:-1] + base)
        its.append(it)
        base += int(up[-1].item())
        del up
    user_ptr = torch.cat(ups + [torch.tensor([base], dtype=torch.int64, device=device)])
    del ups
    items = torch.cat(its)
    return user_ptr, items


def closed_form_rowsums_device(user_ptr, items, n_items: int):
    """rowsum[a] = sum_u m_ua (n_u - 1) over a device CSR, exact int64: what the N-GPU run's owners
    hold for their rows after the row-sum all-reduce (the broadcast of FlinkCooccurrences.java:163)."""
    import torch

    lens = user_ptr[1:] - user_ptr[:-1]
    w = torch.repeat_interleave(lens - 1, lens, output_size=int(items.numel()))
    rs = torch.zeros(n_items, dtype=torch.int64, device=items.device)
    rs.index_add_(0, items.long(), w)
    return rs


def c3_ordered_pairs(u0: int, u1: int, seed: int = C3_SEED) -> int:
    n = c3_lengths(u0, u1, seed).astype(np.int64)
    return int(np.sum(n * (n - 1)))


def spread_over_windows(rng, user_ptr: np.ndarray, n_windows: int, window_ms: int) -> np.ndarray:
    """C4: event times spread over n_windows tumbling windows, ascending within each user."""
    n = int(user_ptr[-1])
    ts = rng.integers(0, n_windows * window_ms, n).astype(np.int64)
    lens = np.diff(user_ptr)
    owner = np.repeat(np.arange(len(lens)), lens)
    order = np.lexsort((ts, owner))
    return ts[order]


def config_c4(seed: int = 4, n_windows: int = 100, window_ms: int = 1000, **c2_kwargs):
    """C4, streaming: the C2 log with timestamps spread over 100 tumbling 1 s windows."""
    d = config_c2(**c2_kwargs)
    rng = np.random.Generator(np.random.PCG64(seed))
    d["ts"] = spread_over_windows(rng, d["user_ptr"], n_windows, window_ms)
    d["window_ms"] = window_ms
    d["name"] = f"C4 streaming: C2 over {n_windows} x {window_ms} ms windows"
    return d


def small_log(seed: int, U: int, M: int, mean_len: float, s: float = 1.0, replacement: bool = True):
    """Small seeded logs for parity tests."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.maximum(rng.poisson(mean_len, U), 1).astype(np.int64)
    if replacement:
        items = zipf_with_replacement(rng, lens, M, s)
    else:
        lens = np.minimum(lens, M)
        items = zipf_without_replacement(rng, lens, M, s)
    user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return user_ptr, items


def to_records(user_ptr: np.ndarray, items: np.ndarray, ts: np.ndarray, user_ids: np.ndarray | None = None):
    """CSR + per-interaction timestamps -> arrival-ordered (user, item, ts) records."""
    lens = np.diff(user_ptr)
    users = np.repeat(np.arange(len(lens), dtype=np.int32) if user_ids is None else user_ids, lens)
    order = np.argsort(ts, kind="stable")
    return users[order].astype(np.int32), items[order].astype(np.int32), ts[order].astype(np.int64)
