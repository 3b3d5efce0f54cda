"""Encrypted-inference throughput of Orion's LoLA on the MI355X HIP backend.

Metric (BASELINE.json): encrypted images/sec (LoLA, N=2^15) + NTT achieved
HBM GB/s vs peak.  A "step" is one FHE forward pass `net(ct)` of the LoLA op
stream (the exact backend-call sequence the reference frontend emits, see
orion_amd/replay.py) over one batch of B images per GPU, every ciphertext
already resident in HBM, run as --pipelines frontend threads of B/P images
(each on a pipeline context of its own); the same steps on one context are
timed right after (value_single_pipeline, and the roofline).  Multi-GPU: one process per GPU, independent image
shards (weak scaling), evaluation keys generated on rank 0 and broadcast over
RCCL/xGMI once before timing; no collective inside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--pipelines P]

--gpus N without a torch.distributed.run environment starts N rank processes
itself (one per GPU, fresh interpreters, before anything touches the GPU);
under torch.distributed.run, WORLD_SIZE must equal N.
ORION_BENCH_REHEARSE=1 rehearses the N-rank flow on fewer GPUs (ranks share
devices, gloo carries the broadcast); ORION_BENCH_DRYRUN=1 runs only the
launcher and the collective flow on the CPU (no GPU, no number reported as a
measurement) -- both are for tests, never for a reported value.
"""
import argparse
import faulthandler
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "encrypted images/sec (LoLa N=2^15) + NTT HBM GB/s vs peak"


def host_cpu():
    """CPUs this process may use on this host, and the host's physical layout."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    cores, sockets, model = set(), set(), ""
    try:
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and not model:
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None:
                    cores.add((phys, core))
                    sockets.add(phys)
                    phys = core = None
    except OSError:
        pass
    info["physical_cores"] = len(cores) or info["nproc"]
    info["sockets"] = len(sockets) or 1
    info["model"] = model
    usable = min(info["affinity"], int(quota) if quota else info["affinity"])
    info["usable"] = max(1, usable)
    return info


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("ORION_BENCH_BATCH", 64)))
    # the GPU's batch as P frontend threads of batch/P images each, every
    # thread on a pipeline context of its own (the scheme's keys and compiled
    # transforms, its own HIP stream): their kernels run concurrently
    ap.add_argument("--pipelines", type=int, default=int(os.environ.get("ORION_BENCH_PIPELINES", 2)))
    ap.add_argument("--workload", default="lola_n15")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # profiler passes: skip the client-side, batch-1 and hipGraph measurements
    # beside the line (rocprofv3's PMC collection does not survive graph replay)
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--cpu-images", type=int, default=8)
    # default: one worker per physical core this process may run on (the
    # host's physical cores, capped by the cgroup CPU quota / affinity mask)
    ap.add_argument("--cpu-workers", type=int, default=0)
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Start n rank processes of this script (fresh interpreters, nothing in
    this parent has touched the GPU), each with the torch.distributed.run
    environment for one local GPU; wait for all, stop the rest if one fails,
    exit with the worst status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0:
                rc = rc or r
                for q in alive:  # a dead rank would leave the others waiting in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc if rc > 0 else (1 if rc else 0)


def _cpu_worker(args):
    """One CPU-baseline worker (a spawned process, no GPU): the oracle's own
    keygen/compile, then `n` timed forward passes of the op stream."""
    name, n = args
    from oracle.replay_cpu import CpuStream
    s = CpuStream(name)
    s.keygen()
    s.compile()
    cts = [s.encrypt(s.arrays["input"]) for _ in range(n)]
    t0 = time.perf_counter()
    for ct in cts:
        s.forward(ct)
    return time.perf_counter() - t0


def cpu_baseline(name, n_images, workers):
    """The CPU parity oracle (single-threaded C restatement of the Lattigo
    algorithms, oracle/ckks_oracle.c -- the builder's Lattigo stand-in, not
    Lattigo) running the same op stream on this host: (a) one core, n_images
    images timed in this process; (b) all-core throughput, `workers` spawned
    processes with one independent image stream each."""
    cpu = host_cpu()
    workers = workers or min(cpu["physical_cores"], cpu["usable"])
    single_dt = _cpu_worker((name, n_images))
    single = n_images / single_dt
    import multiprocessing as mp
    per = 2
    with mp.get_context("spawn").Pool(workers) as pool:
        dts = pool.map(_cpu_worker, [(name, per)] * workers)
    allcore = workers * per / max(dts)
    # the GPU box's cgroup grants fewer CPUs than the host has cores: the
    # measured value uses what this process may run on; the linear scaling to
    # every physical core is reported beside it as an estimate, never as value
    est = allcore / workers * cpu["physical_cores"] if workers < cpu["physical_cores"] else None
    return dict(value=allcore, unit="images/s", cores=workers, kind="port",
                all_physical_cores_linear_estimate=est,
                label="builder C oracle (Lattigo stand-in), single-threaded per op",
                single_core_images_per_s=single,
                host={k: cpu[k] for k in ("model", "nproc", "physical_cores", "sockets", "affinity",
                                          "cgroup_cpus", "usable")},
                sample=f"{name}: all-core = {workers} processes x {per} images (slowest {max(dts):.1f} s); "
                       f"single core = {n_images} images in {single_dt:.1f} s")


def dryrun(args, world, rank):
    """Launcher + collective flow on the CPU (tests): gloo process group,
    bundle broadcast, barrier-bracketed stub step, max over ranks, one line."""
    import torch
    import torch.distributed as dist
    from orion_amd import dist as odist
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group("gloo")
    payload = bytes(range(256)) * 64
    got = {}
    if world > 1:
        def export(buf):
            buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
        odist.broadcast_bundle(dist, lambda: len(payload), export,
                               lambda buf: got.setdefault("ok", bytes(buf.numpy()) == payload), dev)
    ok = got.get("ok", True) if rank else True
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * args.steps)
    dt = time.perf_counter() - t0
    pids = [os.getpid()]
    if world > 1:
        dt = odist.max_over_ranks(dist, dt, dev)
        ok = odist.sum_over_ranks(dist, 0.0 if ok else 1.0, dev) == 0
        allp = [None] * world
        dist.all_gather_object(allp, os.getpid())
        pids = allp
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dryrun": True, "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(dt / max(args.steps, 1) * 1e3, 3),
                          "rank_pids": pids, "bundle_broadcast_ok": ok}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def dump_maps(tag):
    """ORION_DUMP_MAPS=<prefix>: write /proc/self/maps to <prefix>_<tag>.txt, so
    that the PCs of a native crash report (e.g. a profiler's signal handler)
    can be resolved to library + offset afterwards."""
    prefix = os.environ.get("ORION_DUMP_MAPS")
    if prefix:
        with open("/proc/self/maps") as f, open(f"{prefix}_{tag}.txt", "w") as o:
            o.write(f.read())


def stage(name):
    """ORION_BENCH_STAGES=1: name each phase on stderr (locates a crash)"""
    if os.environ.get("ORION_BENCH_STAGES") == "1":
        print(f"bench stage: {name} t={time.perf_counter():.3f}", file=sys.stderr, flush=True)


def main():
    faulthandler.enable()  # a native crash prints the Python frames of every thread
    args = parse()
    from orion_amd import dist as odist
    world, rank, local = odist.env_ranks()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("ORION_BENCH_DRYRUN") == "1":
        return dryrun(args, world, rank)

    import torch
    # ORION_BENCH_REHEARSE=1: rehearse the N-rank flow on a box with fewer GPUs
    # (ranks share devices round-robin, gloo carries the broadcast and the
    # max-reduce); never used for a reported number
    rehearse = os.environ.get("ORION_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from orion_amd.replay import OrionStream, Pipelines
    lib_seed = 2024
    P = max(1, min(args.pipelines, args.batch))  # (a batch of one image runs on one pipeline)
    if args.batch % P:
        print(f"bench.py: --batch {args.batch} is not a multiple of --pipelines {P}", file=sys.stderr)
        sys.exit(2)
    st = OrionStream(args.workload, seed=lib_seed + rank, device=local)
    lib = st.lib
    torch_stream = torch.cuda.Stream()
    lib.OrionHipSetStream(torch_stream.cuda_stream)

    t_setup = time.perf_counter()
    if rank == 0:
        st.keygen(with_po2=True)
        st.compile(gen_keys=True)
    else:
        st.compile(gen_keys=False)
    bundle_bytes = 0
    if world > 1:
        # RCCL broadcast of the public + evaluation keys; the secret key stays
        # on rank 0 (outputs are gathered there for the check)
        def export(buf):
            lib.OrionHipSynchronize()
            if lib.lib.ExportKeyBundle(buf.data_ptr(), 0) != 0:
                raise RuntimeError(lib.lib.OrionHipLastError().decode())
            lib.OrionHipSynchronize()

        def load(buf):
            if lib.lib.ImportKeyBundle(buf.data_ptr(), buf.numel()) != 0:
                raise RuntimeError(lib.lib.OrionHipLastError().decode())
            lib.OrionHipSynchronize()

        bundle_bytes = odist.broadcast_bundle(dist, lambda: lib.KeyBundleBytes(0), export, load, device)
    t_setup = time.perf_counter() - t_setup

    # this rank's shard of synthetic images (MNIST-shaped, N(0,1), seed 42 + rank)
    g = torch.Generator().manual_seed(42 + rank)
    imgs = torch.randn(args.batch, 1, 28, 28, generator=g).numpy()
    imgs[0] = st.reference_input().reshape(1, 28, 28)
    bp = args.batch // P
    # P pipelines = P frontend threads, each running the unchanged op stream
    # (forward() of the one compiled stream) on the batch/P images it encrypted
    # itself; the library binds each thread to a context of its own (the
    # scheme's keys and compiled transforms, its own HIP stream, pool and
    # handles: OrionHipThreadPipelines), so their kernels overlap on the GPU
    pipes = Pipelines(lib, P, device=local) if P > 1 else None
    if pipes:
        cts = pipes.run([(lambda i=i: st.encrypt_batch(imgs[i * bp:(i + 1) * bp])) for i in range(P)])
    else:
        cts = [st.encrypt_batch(imgs)]
    # the whole batch on the scheme's own context (main thread): the
    # single-pipeline timing and the per-kernel breakdown
    ct_all = st.encrypt_batch(imgs) if P > 1 else cts[0]
    lib.OrionHipSynchronize()

    def step():
        """one pass of the op stream over the GPU's batch: P threads, one pipeline each"""
        if P == 1:
            return [st.forward(cts[0])]
        return pipes.run([(lambda c=c: st.forward(c)) for c in cts])

    def delete(outs):
        for o in outs:
            lib.DeleteCiphertext(o)  # (a handle is deleted on its own context)

    def timed(fn, steps):
        """K steps of fn bracketed by barrier + synchronize; returns (seconds, outputs)"""
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        lib.OrionHipSynchronize()
        t0 = time.perf_counter()
        outs = [fn() for _ in range(steps)]
        lib.OrionHipSynchronize()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, outs

    dump_maps("setup")
    stage("warmup")
    for _ in range(args.warmup):
        delete(step())
    lib.OrionHipSynchronize()

    stage("timed")
    lib.OrionHipProfileReset()
    lib.OrionHipProfileClock()
    lib.OrionHipProfile(0b11)  # HIP events around the NTT launches only (the roofline kernel)
    lib.OrionHipLogMark("timed begin")  # (ORION_NTT_LOG: tools/pmc_summary.py cuts the trace to the timed steps)
    dt, outs = timed(step, args.steps)
    lib.OrionHipLogMark("timed end")
    lib.OrionHipProfile(0)
    prof = lib.profile_read()
    ntt_union_ms = lib.profile_union(0b11)  # wall clock with an NTT (forward or inverse) of any pipeline running
    if dist:
        dt = odist.max_over_ranks(dist, dt, device)

    # correctness of the timed output: image 0 of every shard is the fixture's
    # reference input; each rank's output ciphertext for it is gathered to
    # rank 0, which holds the only secret key, and decrypted there
    exp = st.arrays["expected_output"].reshape(-1)
    out0 = lib.export_ciphertext(outs[-1][0])[0]
    level0 = lib.GetCiphertextLevel(outs[-1][0])
    scale0 = lib.GetCiphertextScaleF(outs[-1][0])
    shards = [out0]
    if dist:
        t = torch.from_numpy(out0.view(np.int64).copy()).to(device if not rehearse else "cpu")
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        shards = [a.cpu().numpy().view(np.uint64) for a in allt]
    mae = None
    if rank == 0:
        maes = []
        n_out = int(np.prod(st.meta["output_shape"]))
        for sh in shards:
            h = lib.import_ciphertext(sh[None], scale0)
            assert lib.GetCiphertextLevel(h) == level0
            pt = lib.Decrypt(h)
            vals = np.array(lib.Decode(pt), dtype=np.float64)[:n_out]
            lib.DeletePlaintext(pt)
            lib.DeleteCiphertext(h)
            maes.append(float(np.abs(vals - exp).mean()))
        mae = max(maes)
    for o in outs:
        delete(o)

    # the same K steps with the whole batch on ONE pipeline (the scheme's
    # context, main thread): value_single_pipeline, and the roofline -- every
    # NTT launch timed there has the GPU to itself (with P pipelines the
    # launches of one overlap the other's kernels)
    stage("timed single pipeline")
    if P > 1:
        lib.DeleteCiphertext(st.forward(ct_all))  # warm: this batch size's buffers
    lib.OrionHipSynchronize()
    lib.OrionHipProfileReset()
    lib.OrionHipProfile(0b11)
    lib.OrionHipLogMark("single begin")
    dt1, outs1 = timed(lambda: st.forward(ct_all), args.steps)
    lib.OrionHipLogMark("single end")
    lib.OrionHipProfile(0)
    prof1 = lib.profile_read()
    if dist:
        dt1 = odist.max_over_ranks(dist, dt1, device)
    for o in outs1:
        lib.DeleteCiphertext(o)
    # one extra, fully profiled single-pipeline step (outside the timed
    # regions) for the per-kernel breakdown
    lib.OrionHipProfileReset()
    lib.OrionHipProfile(1)
    lib.OrionHipLogMark("solo begin")
    lib.DeleteCiphertext(st.forward(ct_all))
    lib.OrionHipSynchronize()
    lib.OrionHipLogMark("solo end")
    lib.OrionHipProfile(0)
    breakdown = lib.profile_read()

    client_ms, b1_ms, graph_step = None, None, None
    dump_maps("extras")
    stage("extras: client")
    if rank == 0 and not args.no_extras:
        # client side on the GPU (outside the timed region): encode + encrypt of
        # the batch from HBM-resident slots, and decrypt + decode of the output
        enc_ev = [e for e in st.input_events() if e["op"] == "Encode"][0]
        dvals = torch.zeros(args.batch, st.slots, dtype=torch.float32, device=device)
        dvals[:, :imgs[0].size] = torch.from_numpy(imgs.reshape(args.batch, -1)).to(device)
        torch.cuda.synchronize()
        ct_full = st.encrypt_batch(imgs)
        out_ct = st.forward(ct_full)  # the whole batch's output, on one context
        lib.DeleteCiphertext(ct_full)
        dout = torch.empty(args.batch, lib.slots, dtype=torch.float64, device=device)  # DecodeDevice: [B][slots]

        def client(fn, reps=5):
            fn()
            lib.OrionHipSynchronize()
            t = time.perf_counter()
            for _ in range(reps):
                fn()
            lib.OrionHipSynchronize()
            return (time.perf_counter() - t) / reps * 1e3

        def enc_once():
            pt = lib.encode_batch_device(dvals, enc_ev["args"][1], enc_ev["args"][2])
            lib.DeleteCiphertext(lib.Encrypt(pt))
            lib.DeletePlaintext(pt)

        def dec_once():
            pt = lib.Decrypt(out_ct)
            lib.decode_device(pt, dout)
            lib.DeletePlaintext(pt)

        client_ms = {"encode_encrypt_ms_per_batch": round(client(enc_once), 3),
                     "decrypt_decode_ms_per_batch": round(client(dec_once), 3)}
        lib.DeleteCiphertext(out_ct)

        # BASELINE configs[2] (LoLA N=2^15, batch=1): single-image latency of the
        # same op stream, outside the timed region (one image per launch leaves
        # most CUs idle; the throughput line above is the batched shard)
        stage("extras: batch-1 stream")
        ct1 = st.encrypt_batch(imgs[:1])
        lib.DeleteCiphertext(st.forward(ct1))
        lib.OrionHipSynchronize()
        reps1 = 10
        t1 = time.perf_counter()
        for _ in range(reps1):
            lib.DeleteCiphertext(st.forward(ct1))
        lib.OrionHipSynchronize()
        b1_stream_ms = (time.perf_counter() - t1) / reps1 * 1e3
        # the same pass captured once into a hipGraph and replayed: one launch
        # per image instead of ~900 (launch-bound at one image per launch)
        stage("extras: batch-1 graph capture + replay")
        gid, g_out = st.capture(ct1)
        lib.OrionHipGraphLaunch(gid)
        lib.OrionHipSynchronize()
        b1_check = float(np.abs(st.decrypt_output(g_out)[0] - st.arrays["expected_output"].reshape(-1)).mean())
        t1 = time.perf_counter()
        for _ in range(reps1 * 5):
            lib.OrionHipGraphLaunch(gid)
        lib.OrionHipSynchronize()
        b1_ms = (time.perf_counter() - t1) / (reps1 * 5) * 1e3
        lib.OrionHipGraphDestroy(gid)
        lib.DeleteCiphertext(g_out)
        lib.DeleteCiphertext(ct1)
        # the batched step as a hipGraph replay (reported beside the line; the
        # value above is the stream-launched step the NTT events are timed on)
        stage("extras: batched graph capture + replay")
        # one graph per pipeline, captured by its thread on its stream (one
        # capture at a time); a launch runs on the stream of the context that
        # captured the graph, whichever thread issues it
        gids = ([pipes.run_one(i, lambda c=c: st.capture(c)) for i, c in enumerate(cts)] if pipes
                else [st.capture(cts[0])])

        def launch_all():
            for gid, _ in gids:
                lib.OrionHipGraphLaunch(gid)

        launch_all()
        lib.OrionHipSynchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            launch_all()
        lib.OrionHipSynchronize()
        g_ms = (time.perf_counter() - t1) / args.steps * 1e3
        graph_step = {"ms_per_step": round(g_ms, 3), "images_per_s": round(args.batch / g_ms * 1e3, 3),
                      "graphs": P}
        for gid, g_out in gids:
            lib.OrionHipGraphDestroy(gid)
            lib.DeleteCiphertext(g_out)
    if pipes:
        pipes.close()

    stage("report")
    images = args.batch * world * args.steps
    value = images / dt
    value_single = args.batch * world * args.steps / dt1

    def ntt_sums(pr):
        ntt = [pr.get("ntt_fwd", {}), pr.get("ntt_inv", {})]
        return (sum(p.get("launches", 0) for p in ntt), sum(p.get("ms", 0.0) for p in ntt),
                sum(p.get("bytes", 0.0) for p in ntt),  # fused model (epilogue operands/addends counted)
                sum(p.get("strict_bytes", 0.0) for p in ntt))  # 16 N per limb-transform
    # the roofline: the single-pipeline timed region (every NTT launch with
    # the GPU to itself; HIP events on the library stream the NTTs run on)
    n_launch, n_ms, n_bytes, n_strict = ntt_sums(prof1)
    concurrent = None
    if P > 1:
        # with P pipelines an NTT launch shares the GPU with the other
        # pipelines' kernels, so its duration describes the mix, not the
        # kernel: the P-pipeline timed region's own figures, beside the line.
        # frac_union: the bytes over the wall-clock time at least one NTT ran
        c_launch, c_ms, _, c_strict = ntt_sums(prof)
        concurrent = {"definition": "timed region, P pipelines: 16 N per limb-transform / the wall-clock union "
                                    "of the NTT launch intervals (frac_union), / the summed launch durations "
                                    "(frac_summed); NTTs overlap the other pipelines' kernels",
                      "frac_union": round(c_strict / (ntt_union_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                      if ntt_union_ms > 0 else None,
                      "frac_summed": round(c_strict / (c_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if c_ms > 0 else None,
                      "ntt_union_ms_per_step": round(ntt_union_ms / args.steps, 3),
                      "ntt_summed_launch_ms_per_step": round(c_ms / args.steps, 3),
                      "launches": c_launch}
    achieved = (n_strict / (n_ms / 1e3)) / 1e9 if n_ms > 0 else 0.0
    achieved_fused = (n_bytes / (n_ms / 1e3)) / 1e9 if n_ms > 0 else 0.0
    total_prof_ms = sum(p["ms"] for p in breakdown.values())
    bd_ntt_ms = breakdown.get("ntt_fwd", {}).get("ms", 0) + breakdown.get("ntt_inv", {}).get("ms", 0)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "ntt_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        # HBM bytes per algorithmic byte of the NTT launches, from the committed
        # rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/pmc_summary.py)
        # (the solo window's ratio when the profile has one: the roofline's own step)
        if tj.get("workload") == args.workload and tj.get("batch") == args.batch and n_launch:
            r = tj.get("hbm_bytes_per_algorithmic_byte_solo") or tj["hbm_bytes_per_algorithmic_byte"]
            traffic = round(r * n_bytes / n_launch)

    valu = None
    vfile = os.path.join(ROOT, "profiles", "valu_roofline.json")
    if os.path.exists(vfile):
        with open(vfile) as f:
            vj = json.load(f)
        # VALU roofline of the VALU-bound kernels, from the committed rocprofv3
        # SQ/GRBM pass over this same workload (tools/pmc_summary.py)
        if vj.get("workload") == args.workload and vj.get("batch") == args.batch:
            valu = {"profile": vj["tag"], "definition": vj["definition"],
                    "valu_busy": {k: round(v["valu_busy"], 3) for k, v in vj["kernels"].items()}}

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(args.workload, args.cpu_images, args.cpu_workers)
            except Exception as e:  # the baseline must never break the GPU line
                cpu = dict(value=None, unit="images/s", cores=1, kind="port", sample=f"failed: {e}")
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "value_single_pipeline": round(value_single, 3),
            "ms_per_step_single_pipeline": round(dt1 / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: N(0,1) 1x28x28 images (image 0 = fixture input), LoLA diagonals from the "
                    "reference frontend's compile of seeded random-init weights",
            "config": {"workload": f"LoLA (models/lola.py) {args.workload}: N=2^15, LogQ=[60]+[40]x11, "
                                   f"LogP=[60,60], input level {st.input_level}, Standard ring",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "parallelism": f"replicas x{world} (image shards), keys RCCL-broadcast"
                                      + (" (rehearsal: gloo, shared GPUs)" if rehearse else "")
                                      + (f"; per GPU {P} frontend threads of {args.batch // P} images each, "
                                         "each thread on a pipeline context of its own (the scheme's keys and "
                                         "compiled transforms, its own HIP stream), kernels concurrent"
                                         if P > 1 else "")},
            "roofline": {"bound": "hbm", "kernel": "ntt (fwd+inv: one-pass, 1 limb per workgroup; two-pass for partial-round launches)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "definition": "strict (SURVEY 8d): 16 N bytes per limb-transform / the NTT launches' "
                                       "HIP-event durations over the single-pipeline timed region (the whole "
                                       "batch on one context: value_single_pipeline; log window 'single')",
                         "pipelines": P,
                         "concurrent": concurrent,
                         "achieved_fused": round(achieved_fused, 1),
                         "frac_fused": round(achieved_fused / HBM_PEAK_GBS, 4),
                         "definition_fused": "16 N per limb-transform + 8 N per epilogue operand or addend read "
                                             "(scatter index excluded like the twiddles)",
                         "launches": n_launch, "avg_launch_us": round(n_ms / max(n_launch, 1) * 1e3, 2),
                         "algorithmic_bytes_per_launch": round(n_strict / max(n_launch, 1)),
                         "fused_bytes_per_launch": round(n_bytes / max(n_launch, 1)),
                         "ntt_share_of_kernel_time": round(bd_ntt_ms / total_prof_ms, 3) if total_prof_ms else None},
            "valu_roofline": valu,
            "cpu_baseline": cpu,
            "check": {"mae_image0_vs_cleartext": mae, "mae_over_ranks": "max (outputs gathered to rank 0)",
                      "setup_s": round(t_setup, 1), "key_bundle_bytes": bundle_bytes},
            "client_gpu": dict(client_ms, end_to_end_images_per_s=round(
                args.batch / ((dt / args.steps) + (client_ms["encode_encrypt_ms_per_batch"]
                                                   + client_ms["decrypt_decode_ms_per_batch"]) / 1e3) * world, 3))
            if client_ms else None,
            "batch1": {"ms_per_image": round(b1_ms, 3), "images_per_s": round(1e3 / b1_ms, 1), "launch": "hipGraph",
                       "stream_ms_per_image": round(b1_stream_ms, 3), "mae_vs_cleartext": round(b1_check, 7)}
            if b1_ms else None,
            "graph_replay": graph_step,
            "kernel_ms_per_step": {k: round(v["ms"], 3) for k, v in breakdown.items()},
            "kernel_algorithmic_gbs": {k: round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1)
                                       for k, v in breakdown.items() if v["ms"] > 0},
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
