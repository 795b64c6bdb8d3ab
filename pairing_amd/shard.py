"""Multi-GPU sharding of the path's batches.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Pairings are independent, so a global batch is split into contiguous shards,
one per rank, with no collective on the data path; the only exchange is a
single gather of the Fq12 results to the root.  For the trait's multi-pair
semantics (Engine::miller_loop over all pairs = the product of per-pair
Miller values, mod.rs:40-102) each rank reduces its shard to one Fq12 and
the root gathers 576 B per rank.

The other batch shapes shard the same way: an Fq / Fr multiply batch, a
point-decoding batch and a fixed-base scalar batch (`Wnaf::base(g, n)
.scalar(s_i)` with the scalars split and every rank holding its own table --
what `Wnaf::shared()`, wnaf.rs:131-154, exists for) are `sharded_batch_from`
with a gather of their rows; a multi-scalar multiplication is
`sharded_reduce`: each rank sums its terms, the root adds one point per rank.

The functions are backend-agnostic (they take the local compute as a
callable and use torch.distributed collectives), so the same code path runs
with RCCL on MI355X and with gloo on CPU in tests/test_distributed.py.
"""
import torch
import torch.distributed as dist


def shard_range(n, world, rank):
    """Contiguous [start, stop) of rank's shard: sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank %d/%d" % (world, rank))
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_rows_to_root(local, n_global, root=0, group=None):
    """Gather every rank's (n_r, w) row block to `root` in rank order.
    Ragged shards are padded to the largest shard for the collective.
    Returns the (n_global, w) tensor on root, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [b - a for a, b in (shard_range(n_global, world, r) for r in range(world))]
    width = local.shape[1]
    cap = max(sizes)
    if local.shape[0] != sizes[rank]:
        raise ValueError("rank %d holds %d rows, shard is %d" % (rank, local.shape[0], sizes[rank]))
    send = local
    if local.shape[0] < cap:
        send = torch.zeros((cap, width), dtype=local.dtype, device=local.device)
        send[:local.shape[0]] = local
    bufs = [torch.empty((cap, width), dtype=local.dtype, device=local.device) for _ in range(world)] \
        if rank == root else None
    dist.gather(send.contiguous(), bufs, dst=root, group=group)
    if rank != root:
        return None
    return torch.cat([bufs[r][:sizes[r]] for r in range(world)], dim=0)


class RowGatherer:
    """gather_rows_to_root with preallocated buffers in `slots` rotating sets,
    so that the gather of one batch can run asynchronously (RCCL's stream, or
    gloo's thread) while the next batch computes into another output buffer.
    gather(local, slot) returns the collective's work handle; the caller
    waits on it before it writes `local` again."""

    def __init__(self, n_global, width, like, root=0, group=None, slots=2):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.root, self.group = root, group
        self.sizes = [b - a for a, b in (shard_range(n_global, self.world, r) for r in range(self.world))]
        self.cap = max(self.sizes)
        mk = lambda: torch.empty((self.cap, width), dtype=like.dtype, device=like.device)  # noqa: E731
        self.send = [mk() for _ in range(slots)] if self.sizes[self.rank] < self.cap else None
        self.recv = [[mk() for _ in range(self.world)] for _ in range(slots)] if self.rank == root else None

    def gather(self, local, slot=0, async_op=True):
        if local.shape[0] != self.sizes[self.rank]:
            raise ValueError("rank %d holds %d rows, shard is %d" % (self.rank, local.shape[0], self.sizes[self.rank]))
        send = local
        if self.send is not None:
            send = self.send[slot]
            send[:local.shape[0]].copy_(local)
        bufs = self.recv[slot] if self.recv is not None else None
        return dist.gather(send.contiguous(), bufs, dst=self.root, group=self.group, async_op=async_op)

    def result(self, slot=0):
        """the (n_global, w) rows of a finished gather, on root (None elsewhere)"""
        if self.recv is None:
            return None
        return torch.cat([self.recv[slot][r][:self.sizes[r]] for r in range(self.world)], dim=0)


def sharded_batch_from(load, n, compute, root=0, group=None):
    """out[i] over a global batch of n pairings, sharded across ranks, where
    each rank stages ONLY its own shard: load(start, stop) -> (p_shard,
    q_shard) (from a file, a memmap or a generator), compute: (p_shard,
    q_shard) -> (n_shard, w) tensor on this rank's device.  Returns the (n, w)
    result on root, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(n, world, rank)
    local = compute(*load(a, b))
    return gather_rows_to_root(local, n, root=root, group=group)


def sharded_batch(p, q, compute, root=0, group=None):
    """sharded_batch_from over indexable p, q (arrays, memmaps, tensors): each
    rank slices its own rows, so a memmap'd global batch is read only shard by
    shard."""
    return sharded_batch_from(lambda a, b: (p[a:b], q[a:b]), p.shape[0], compute, root=root, group=group)


def sharded_reduce(load, n, local_reduce, combine, root=0, group=None):
    """A reduction over a global batch of n items sharded across ranks: each
    rank stages only its rows, load(start, stop) -> operands, and reduces them
    to one row, local_reduce(*operands) -> (1, w) tensor; the root gathers one
    row per rank and folds them, combine((world, w)) -> result.  Returns the
    result on root, None elsewhere.  Used for the multi-pair Miller loop
    (sharded_product) and the multi-scalar multiplication (sum of per-rank
    partial sums)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(n, world, rank)
    local = local_reduce(*load(a, b))
    rows = [torch.empty_like(local) for _ in range(world)] if rank == root else None
    dist.gather(local.contiguous(), rows, dst=root, group=group)
    if rank != root:
        return None
    return combine(torch.cat(rows, dim=0))


def sharded_product(p, q, local_product, combine, root=0, group=None):
    """The multi-pair Miller loop across ranks: each rank reduces its shard to
    one Fq12 with `local_product(p_shard, q_shard) -> (1, 72)`, the root
    gathers one row per rank and folds them with `combine((world, 72)) -> (1, 72)`."""
    return sharded_reduce(lambda a, b: (p[a:b], q[a:b]), p.shape[0], local_product, combine, root=root,
                          group=group)
