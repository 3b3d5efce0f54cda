"""World-size-2 gloo tests of the multi-GPU control path (orion_amd/dist.py)
on the CPU: key-bundle broadcast, image sharding and max-over-ranks timing,
the same calls bench.py makes over RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from orion_amd import dist as odist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bundle(nbytes):
    return np.random.default_rng(99).integers(0, 256, nbytes, dtype=np.uint8)


def _worker(rank, world, port, nbytes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = {}
        exp = _bundle(nbytes)

        def export(buf):
            buf.copy_(torch.from_numpy(exp))

        def load(buf):
            got["bytes"] = buf.numpy().copy()

        n = odist.broadcast_bundle(dist, lambda: nbytes, export, load, torch.device("cpu"))
        ok_bundle = n == nbytes and (rank == 0 or np.array_equal(got["bytes"], exp))
        slowest = odist.max_over_ranks(dist, 1.0 + rank, torch.device("cpu"))
        lo, hi = odist.shard(130, world, rank)
        total = odist.sum_over_ranks(dist, hi - lo, torch.device("cpu"))
        q.put((rank, ok_bundle, slowest, (lo, hi), total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nbytes", [1, 3 << 20])
def test_key_bundle_broadcast_world2(nbytes):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nbytes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), "bundle differs on a non-root rank"
    assert all(r[2] == 2.0 for r in res), "max over ranks"
    assert [r[3] for r in res] == [(0, 65), (65, 130)]
    assert all(r[4] == 130 for r in res)


def test_shard_covers_every_image():
    for n in (0, 1, 7, 64, 512):
        for world in (1, 2, 3, 8):
            spans = [odist.shard(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _run_bench(args, extra_env=None, timeout=240):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(ORION_BENCH_DRYRUN="1", **(extra_env or {}))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=root)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


def test_bench_launches_n_ranks_itself():
    """`bench.py --gpus 2` with no torch.distributed.run environment starts two
    rank processes itself (--gpus was ignored); rank 0 prints one
    line with n_gpus 2, gathered from two distinct processes, after the key
    bundle broadcast over gloo reached the other rank."""
    r, lines = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["dryrun"] is True and ln["value"] is None
    assert len(set(ln["rank_pids"])) == 2
    assert ln["bundle_broadcast_ok"] is True


def test_bench_refuses_world_mismatch():
    """Under an external launcher, WORLD_SIZE must equal --gpus."""
    r, lines = _run_bench(["--gpus", "2"], extra_env=dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and not lines
    assert "--gpus 2" in r.stderr
