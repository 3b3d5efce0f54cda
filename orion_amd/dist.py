"""Multi-GPU control path: one process per GPU, independent image shards,
evaluation keys broadcast once over RCCL (xGMI) -- SURVEY.md §8e.

The reference has no distributed code at all.  Images are
independent ciphertexts (orion/backend/python/tensors.py:143-157), so the
forward pass needs no collective; the only exchange is the one-off broadcast
of the key bundle (public + relinearisation + Galois keys) from the keygen
rank.  Everything here is backend-agnostic so the same code runs over RCCL
("nccl") on the GPU box and over gloo in the CPU tests.
"""
import os

import torch


def env_ranks():
    """(world, rank, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_total, world, rank):
    """Contiguous [lo, hi) slice of n_total images owned by rank (sizes differ
    by at most one)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def broadcast_bundle(dist, nbytes_fn, export_fn, import_fn, device, src=0):
    """Broadcast one opaque byte bundle from rank `src` to every rank.

    nbytes_fn() -> int and export_fn(buf) run on src only (export_fn fills the
    uint8 tensor `buf`); import_fn(buf) runs on every other rank.  Returns the
    bundle size in bytes.  One size broadcast + one payload broadcast: RCCL
    splits the payload over the 7 xGMI links of an MI355X node itself.
    """
    rank = dist.get_rank()
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = int(nbytes_fn())
    dist.broadcast(n, src)
    nbytes = int(n.item())
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if rank == src:
        export_fn(buf)
    if buf.is_cuda:
        torch.cuda.synchronize(device)
    dist.broadcast(buf, src)
    if buf.is_cuda:
        torch.cuda.synchronize(device)
    if rank != src:
        import_fn(buf)
    del buf
    return nbytes


def max_over_ranks(dist, seconds, device):
    """Slowest rank's time (the timed region ends when every shard is done)."""
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, value, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
