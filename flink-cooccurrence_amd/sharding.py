"""Multi-GPU sharding layer: users sharded over ranks, rows owned by one rank each.

Three exchanges are implemented, all keyed by a row owner (the reference's
keyBy(ItemCooccurrences::getItem), FlinkCooccurrences.java:152): ``count_owned`` (C3 / C5 universes,
owner = the frequency-snake map), ``count_records`` and ``count_sharded`` (owner(a) = a mod world):

* ``count_records`` (default) routes the pair RECORDS: every rank all-gathers the users' u16
  histories once (input sized) and all-to-alls one 8-B descriptor per (row, user) record to the
  row's owner, which then reduces complete rows.  Exchanged bytes ~ 2 N + 8 N per rank.
* ``count_sharded`` routes PARTIAL COUNTS: every rank reduces its own users, packs its partial
  rows by owner and the owner merges them.  Exchanged bytes ~ 8 D per rank (D = distinct keys of
  a rank's partial result, up to n_items^2), which dominates on dense co-occurrence data.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Mirrors the
reference's keyed data-parallelism:

* keyBy(user) (FlinkCooccurrences.java:70)  -> every rank expands only its own users' histories;
* keyBy(ItemCooccurrences::getItem) (:152)    -> an all-to-all of each rank's partial rows to the
                                                 row's owner, then an owner-side merge;
* rowSumStream.broadcast() (:163)             -> one all-reduce of the int64 row-sum vector.

* ``count_owned`` (n_items >= 40,320: the C3 / C5 universes) routes the INPUT: every rank
  all-gathers the users' histories (input sized, 4 B per interaction), and counts the rows it owns
  over all of them.  Ownership balances the row work: rows sorted by global item frequency are dealt
  to the ranks in snake order (Zipf-hot rows spread over every rank).  Nothing is merged.

Every library call runs on torch's current stream (cooc.h stream contract), so collectives and
kernels are ordered by the stream itself; no device-wide synchronisation is needed.
The compute (local reduce, pack, merge) runs in libcooc_hip.so.  ``count_owned`` / ``topk_owned`` run
WHOLE inside the library once the context has a communicator (``init_comm``: RCCL over xGMI, the
product path; ``init_comm_torch_ops``: the same library exchange over torch.distributed collectives,
e.g. gloo in the 2-process tests); without one this module moves the buffers itself.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch
import torch.distributed as dist


def balanced_user_ranges(user_ptr, world: int) -> list:
    """Contiguous user ranges [u0, u1) of about equal pair work sum n_u (n_u - 1), one per rank: the
    keyBy(user) of FlinkCooccurrences.java:70 balanced on sum n_u^2, since hashing users
    to ranks is unbalanced under skew.  user_ptr: int64 numpy array or tensor [U+1]; deterministic, so
    every rank computes the same split from the same offsets."""
    import numpy as np

    up = user_ptr.cpu().numpy() if isinstance(user_ptr, torch.Tensor) else np.asarray(user_ptr, np.int64)
    n = np.diff(up).astype(np.int64)
    cum = np.cumsum(n * (n - 1))
    total = int(cum[-1]) if len(cum) else 0
    cuts = [0]
    for r in range(1, world):
        # first user whose prefix reaches r/world of the work (ties: ranges stay non-decreasing)
        cuts.append(max(cuts[-1], int(np.searchsorted(cum, total * r / world, side="left")) + 1 if total else 0))
    cuts.append(len(n))
    cuts = [min(c, len(n)) for c in cuts]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_users(user_ptr, items, world: int, rank: int):
    """This rank's users of a whole log (CSR) under balanced_user_ranges: (user_ptr, items, u0) with
    user_ptr rebased to 0."""
    u0, u1 = balanced_user_ranges(user_ptr, world)[rank]
    s, e = int(user_ptr[u0]), int(user_ptr[u1])
    return user_ptr[u0:u1 + 1] - s, items[s:e], u0


def rows_owned(n_items: int, n_parts: int, part: int) -> int:
    return (n_items - part + n_parts - 1) // n_parts if part < n_items else 0


@dataclass
class ShardResult:
    part: int
    n_parts: int
    merged: object          # CoocDeviceResult of the owned rows (rows r -> items part + r * n_parts)
    rowsum: torch.Tensor    # all-reduced exact row sums, int64 [n_items] (device)
    observed: int           # global ordered pairs (sum over ranks)
    local_observed: int
    sent_entries: int
    recv_entries: int


def count_sharded(core, user_ptr, items, group=None, stream=None) -> ShardResult:
    """One window over this rank's users, exchanged and merged by row owner."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = items.device
    M = core.n_items
    res = core.count_device(user_ptr, items, stream)
    # row sums: all-reduce (the broadcast of the reference's row-sum stream)
    rowsum = torch.empty(M, dtype=torch.int64, device=dev)
    core.copy_rowsum_device(rowsum, stream)
    work = dist.all_reduce(rowsum, group=group, async_op=True)
    # partial rows -> owners
    send_counts = core.partition_plan(world)
    row_nnz = torch.empty(M, dtype=torch.int32, device=dev)
    entries = torch.empty(int(send_counts.sum()), dtype=torch.int64, device=dev)
    core.partition_pack(world, row_nnz, entries, stream)
    counts = torch.as_tensor(send_counts, dtype=torch.int64, device=dev)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    recv_counts_h = recv_counts.cpu().tolist()
    R = rows_owned(M, world, rank)
    recv_nnz = torch.empty(R * world, dtype=torch.int32, device=dev)
    dist.all_to_all_single(recv_nnz, row_nnz, [R] * world, [rows_owned(M, world, o) for o in range(world)],
                           group=group)
    recv_entries = torch.empty(int(sum(recv_counts_h)), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_entries, entries, recv_counts_h, send_counts.tolist(), group=group)
    work.wait()
    obs = torch.tensor([res.observed], dtype=torch.int64, device=dev)
    dist.all_reduce(obs, group=group)
    merged = core.merge_partitions(world, rank, recv_nnz, recv_entries, rowsum, stream)
    return ShardResult(rank, world, merged, rowsum, int(obs.item()), int(res.observed), int(send_counts.sum()),
                       int(sum(recv_counts_h)))




@dataclass
class RecordsResult:
    part: int
    n_parts: int
    owned: object           # CoocDeviceResult of the owned rows (rows r -> items part + r * n_parts), complete
    observed: int           # global ordered pairs (sum over ranks)
    local_observed: int     # this rank's users' ordered pairs
    sent_records: int
    recv_records: int
    arena_stride: int


def count_records(core, user_ptr, items, group=None, stream=None) -> RecordsResult:
    """One window over this rank's users; pair records routed to owner(a) and reduced there."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = items.device
    M = core.n_items
    n_users, n = int(user_ptr.numel()) - 1, int(items.numel())
    # every rank's arena slot has the same size (all_gather_into_tensor): the largest part's need
    cap = torch.tensor([core.shard_arena_cap(n_users, n)], dtype=torch.int64, device=dev)
    dist.all_reduce(cap, op=dist.ReduceOp.MAX, group=group)
    stride = int(cap.item())
    arena = torch.empty(stride, dtype=torch.int16, device=dev)
    desc = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    row_counts = torch.empty(M, dtype=torch.int32, device=dev)
    send, _arena_ids, local_obs = core.shard_plan(user_ptr, items, world, desc, row_counts, arena, stream)
    arena_all = torch.empty(world * stride, dtype=torch.int16, device=dev)
    # u16 ids travel as int32 pairs (RCCL has no 16-bit integer type; the stride is a multiple of 8 ids)
    work = dist.all_gather_into_tensor(arena_all.view(torch.int32), arena.view(torch.int32), group=group,
                                       async_op=True)
    counts = torch.as_tensor(send, dtype=torch.int64, device=dev)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    R = rows_owned(M, world, rank)
    recv_rc = torch.empty(world * R, dtype=torch.int32, device=dev)
    dist.all_to_all_single(recv_rc, row_counts, [R] * world, [rows_owned(M, world, o) for o in range(world)],
                           group=group)
    recv_h = recv_counts.cpu().tolist()
    recv_desc = torch.empty(sum(recv_h), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_desc, desc, recv_h, send.tolist(), group=group)
    obs = torch.tensor([local_obs], dtype=torch.int64, device=dev)
    dist.all_reduce(obs, group=group)
    work.wait()
    owned = core.shard_count(world, rank, recv_rc, recv_desc, arena_all, stride, stream)
    return RecordsResult(rank, world, owned, int(obs.item()), int(local_obs), n, int(sum(recv_h)), stride)


def snake_owner(item_counts: torch.Tensor, world: int, head: int = 4096) -> torch.Tensor:
    """Row owner map balancing the row work (~ the item's frequency): the `head` most frequent rows
    are placed greedily on the least loaded rank (largest first), the rest are dealt in snake order
    (0..W-1, W-1..0, ...).  Deterministic (stable sort, fixed tie order), so every rank computes the
    same map from the same all-reduced counts."""
    import heapq

    M = item_counts.numel()
    order = torch.argsort(-item_counts, stable=True)
    owner = torch.empty(M, dtype=torch.int32, device=item_counts.device)
    h = min(head, M)
    top = item_counts[order[:h]].cpu().tolist()
    load = [(0, r) for r in range(world)]
    heapq.heapify(load)
    head_own = []
    for wgt in top:
        l, r = heapq.heappop(load)
        head_own.append(r)
        heapq.heappush(load, (l + int(wgt), r))
    owner[order[:h]] = torch.tensor(head_own, dtype=torch.int32, device=item_counts.device)
    # the tail: snake order, starting from the least loaded rank's side
    pos = torch.arange(M - h, device=item_counts.device)
    lap, r = pos // world, pos % world
    rank_by_load = torch.tensor([r_ for _, r_ in sorted(load)], dtype=torch.int64, device=item_counts.device)
    slot = torch.where(lap % 2 == 0, r, world - 1 - r)
    owner[order[h:]] = rank_by_load[slot].to(torch.int32)
    return owner


@dataclass
class OwnedResult:
    part: int
    n_parts: int
    owned: object           # CoocDeviceResult over all n_items rows; rows of other ranks are empty
    owner: torch.Tensor     # int32 [n_items] row owner map
    observed: int           # global ordered pairs (sum over ranks of the owned rows' pairs)
    local_observed: int     # ordered pairs of this rank's owned rows
    n_users_all: int
    n_interactions_all: int
    gathered_bytes: int     # history bytes this rank received


def _gather_parts(out, part, sizes, group=None):
    """out = the ranks' parts concatenated in rank order (sizes[r] elements from rank r): an uneven
    all-to-all with this rank's part as the input of every destination -- over RCCL without a world-fold
    copy of it (the list form); gloo has only the single-tensor form, which gets a repeated copy, freed at
    once."""
    world = len(sizes)
    if world == 1:
        out.copy_(part)
        return
    if dist.get_backend(group) == "nccl":
        dist.all_to_all(list(out.split(list(sizes))), [part] * world, group=group)
        return
    n = int(part.numel())
    rep = part.repeat(world) if n else part
    dist.all_to_all_single(out, rep, output_split_sizes=list(sizes), input_split_sizes=[n] * world, group=group)
    del rep


# ---- the library's communicator ---------------------------------------------------------------------
def init_comm(core, group=None) -> None:
    """Give `core` the library's RCCL communicator over the ranks of `group` (one context per GPU
    process): rank 0 creates the id (cooc_comm_unique_id), torch.distributed broadcasts it, every rank
    joins (cooc_comm_init).  cooc_count_owned / cooc_topk_owned then run their exchanges inside the
    library over RCCL (xGMI), on the caller's stream."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    buf = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        buf.copy_(torch.frombuffer(bytearray(core.comm_unique_id()), dtype=torch.uint8))
    dist.broadcast(buf, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    core.comm_init(bytes(buf.cpu().numpy().tobytes()), rank, world)


def init_comm_torch_ops(core, group=None) -> None:
    """The library's exchange (cooc_count_owned / cooc_topk_owned) over torch.distributed collectives
    through cooc_comm_ops callbacks (any backend; gloo in the tests): every callback drains the stream,
    copies its device buffers to the host, runs the collective, and copies the result back."""
    import numpy as np

    from . import _lib

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    D2H, H2D = 2, 1

    def d2h(ptr, nbytes):
        a = np.empty(nbytes, np.uint8)
        if nbytes:
            assert hip.hipMemcpy(a.ctypes.data, ptr, nbytes, D2H) == 0
        return a

    def h2d(ptr, a):
        if a.nbytes:
            assert hip.hipMemcpy(ptr, a.ctypes.data, a.nbytes, H2D) == 0

    def guard(fn):
        def wrapped(*args):
            try:
                fn(*args)
                return 0
            except Exception:  # (a callback cannot raise through the C-ABI)
                import traceback

                traceback.print_exc()
                return 1
        return wrapped

    @guard
    def allreduce(_user, d_buf, n, stream):
        assert hip.hipStreamSynchronize(stream) == 0
        t = torch.from_numpy(d2h(d_buf, 8 * n).view(np.int64).copy())
        dist.all_reduce(t, group=group)
        h2d(d_buf, t.numpy().view(np.uint8))

    @guard
    def allgather(_user, d_send, d_recv, nbytes, stream):
        assert hip.hipStreamSynchronize(stream) == 0
        world = dist.get_world_size(group)
        mine = torch.from_numpy(d2h(d_send, nbytes))
        out = torch.empty(world * nbytes, dtype=torch.uint8)
        dist.all_gather(list(out.split(nbytes)), mine, group=group)
        h2d(d_recv, out.numpy())

    @guard
    def alltoallv(_user, d_send, send_off, send_bytes, d_recv, recv_off, recv_bytes, stream):
        assert hip.hipStreamSynchronize(stream) == 0
        world = dist.get_world_size(group)
        sb = [int(send_bytes[p]) for p in range(world)]
        rb = [int(recv_bytes[p]) for p in range(world)]
        ins = torch.from_numpy(np.concatenate([d2h((d_send or 0) + int(send_off[p]), sb[p]) for p in range(world)]))
        out = torch.empty(sum(rb), dtype=torch.uint8)
        dist.all_to_all_single(out, ins, output_split_sizes=rb, input_split_sizes=sb, group=group)
        pos = 0
        for p in range(world):
            h2d((d_recv or 0) + int(recv_off[p]), out[pos:pos + rb[p]].numpy())
            pos += rb[p]

    ops = _lib.CoocCommOps(_lib.ALLREDUCE_FN(allreduce), _lib.ALLGATHER_FN(allgather), _lib.ALLTOALLV_FN(alltoallv))
    core.comm_init_ops(dist.get_rank(group), dist.get_world_size(group), ops)


def _device_array(ptr: int, n: int, dtype, dev):
    """A device tensor copy of n elements at a library-owned device pointer (borrowed view)."""
    out = torch.empty(n, dtype=dtype, device=dev)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_void_p]
        assert hip.hipMemcpyAsync(out.data_ptr(), ptr, out.element_size() * n, 3,
                                  torch.cuda.current_stream(dev).cuda_stream) == 0
    return out


def count_owned(core, user_ptr, items, group=None, stream=None) -> OwnedResult:
    """One window over this rank's users; histories all-gathered, owned rows counted here.  With a
    library communicator (init_comm / init_comm_torch_ops) the whole step is cooc_count_owned."""
    if getattr(core, "comm_world", 0) > 0:
        res, info = core.count_owned(user_ptr, items, stream=stream)
        owner = _device_array(info.owner, core.n_items, torch.int32, items.device)
        return OwnedResult(info.part, info.n_parts, res, owner, int(info.observed), int(info.local_observed),
                           int(info.n_users_all), int(info.n_interactions_all), int(info.gathered_bytes))
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = items.device
    M = core.n_items
    n_users, n = int(user_ptr.numel()) - 1, int(items.numel())
    # global item frequencies (the planner's column estimate) and the row owner map
    counts = core.item_counts(items, stream=stream)  # (torch.bincount: global atomics on Zipf-hot bins)
    dist.all_reduce(counts, group=group)
    owner = snake_owner(counts, world)
    # all-gather the histories straight into one compact CSR: one uneven all-to-all per array, every
    # rank sending its whole part to every rank, so that the parts land at their exact places (no
    # padding, no compacting copy) and all the transfers of a collective run at once -- on xGMI's
    # point-to-point links every peer pair moves its part over its own link
    sizes = torch.tensor([n_users, n], dtype=torch.int64, device=dev)
    all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_sizes, sizes, group=group)
    sz = all_sizes.view(world, 2).cpu().tolist()
    n_users_all = sum(s_[0] for s_ in sz)
    n_all = sum(s_[1] for s_ in sz)
    up_all = torch.zeros(n_users_all + 1, dtype=torch.int64, device=dev)
    it_all = torch.empty(max(n_all, 1), dtype=torch.int32, device=dev)
    lens_all = up_all[1:]
    _gather_parts(lens_all, torch.sub(user_ptr[1:], user_ptr[:-1]), [s_[0] for s_ in sz], group)
    _gather_parts(it_all[:n_all], items, [s_[1] for s_ in sz], group)
    lens_all.cumsum_(0)  # lengths -> offsets, in place (up_all[0] == 0)
    res = core.count_device_owned(up_all, it_all, owner, rank, counts, n_all, stream)
    obs = torch.tensor([res.observed], dtype=torch.int64, device=dev)
    dist.all_reduce(obs, group=group)
    return OwnedResult(rank, world, res, owner, int(obs.item()), int(res.observed), n_users_all, n_all,
                       4 * (n_all - n) + 8 * (n_users_all - n_users))


@dataclass
class TopkResult:
    sizes: torch.Tensor     # int32 [n_items]: heap sizes (0 for rows owned elsewhere)
    values: torch.Tensor    # int32 [n_items, k]: IntDoublePriorityQueue heap positions 1..size
    scores: torch.Tensor    # float64 [n_items, k]
    rowsum: torch.Tensor    # int64 [n_items]: the all-reduced row sums the scores used


def topk_owned(core, owned: OwnedResult, topk: int, group=None, exact_scores: bool = False,
               stream=None) -> TopkResult:
    """C5 after count_owned: the rows' LLR top-k on their owner (ItemRowRescorer...java:195-241).
    The owned results' row sums are all-reduced first -- the reference broadcasts its row-sum stream to
    every rescorer (FlinkCooccurrences.java:163) -- so that k21 = rowSum(b) - k11 and the observed total
    are the whole log's; each rank then scores only the rows it owns."""
    M = core.n_items
    dev = owned.owner.device
    rowsum = torch.empty(M, dtype=torch.int64, device=dev)
    sizes = torch.empty(M, dtype=torch.int32, device=dev)
    values = torch.empty((M, topk), dtype=torch.int32, device=dev)
    scores = torch.empty((M, topk), dtype=torch.float64, device=dev)
    if getattr(core, "comm_world", 0) > 0:  # the all-reduce and the scoring inside the library
        core.topk_owned(topk, sizes, values, scores, rowsum_global=rowsum, exact_scores=exact_scores, stream=stream)
        return TopkResult(sizes, values, scores, rowsum)
    core.copy_rowsum_device(rowsum, stream)
    dist.all_reduce(rowsum, group=group)
    core.topk_batch_device(topk, sizes, values, scores, rowsum_global=rowsum, exact_scores=exact_scores, stream=stream)
    return TopkResult(sizes, values, scores, rowsum)
