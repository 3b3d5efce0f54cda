"""Encrypted-inference throughput of Orion's LoLA on the MI355X HIP backend.

Metric (BASELINE.json): encrypted images/sec (LoLA, N=2^15) + NTT achieved
HBM GB/s vs peak.  A "step" is one FHE forward pass `net(ct)` of the LoLA op
stream (the exact backend-call sequence the reference frontend emits, see
orion_amd/replay.py) over one batch of B images per GPU, every ciphertext
already resident in HBM.  Multi-GPU: one process per GPU, independent image
shards (weak scaling), evaluation keys generated on rank 0 and broadcast over
RCCL/xGMI once before timing; no collective inside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("ORION_BENCH_BATCH", 64)))
    ap.add_argument("--workload", default="lola_n15")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-images", type=int, default=8)
    ap.add_argument("--cpu-workers", type=int, default=min(16, os.cpu_count() or 1))
    return ap.parse_args()


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
    algorithms, oracle/ckks_oracle.c) running the same op stream on this host:
    (a) one core, n_images images timed in this process; (b) all-core
    throughput, `workers` spawned processes with one independent image
    stream each, 2 images per worker."""
    single_dt = _cpu_worker((name, n_images))
    single = n_images / single_dt
    import multiprocessing as mp
    per = 2
    with mp.get_context("spawn").Pool(workers) as pool:
        dts = pool.map(_cpu_worker, [(name, per)] * workers)
    allcore = workers * per / max(dts)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return dict(value=allcore, unit="images/s", cores=workers, kind="port",
                single_core_images_per_s=single,
                sample=f"{name}: oracle/ckks_oracle.c (single-threaded per op, like Lattigo); all-core = "
                       f"{workers} processes x {per} images (slowest {max(dts):.1f} s); single core = "
                       f"{n_images} images in {single_dt:.1f} s; host '{model}', nproc={os.cpu_count()}")


def main():
    args = parse()
    import torch
    from orion_amd import dist as odist
    world, rank, local = odist.env_ranks()
    # ORION_BENCH_REHEARSE=1: rehearse the N-rank flow on a box with fewer GPUs
    # (ranks share devices round-robin, gloo carries the broadcast and the
    # max-reduce); never used for a reported number
    rehearse = os.environ.get("ORION_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from orion_amd.replay import OrionStream
    lib_seed = 2024
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
    if world > 1:
        # RCCL broadcast of public + evaluation keys (+ secret for output checks)
        def export(buf):
            lib.OrionHipSynchronize()
            if lib.lib.ExportKeyBundle(buf.data_ptr(), 1) != 0:
                raise RuntimeError(lib.lib.OrionHipLastError().decode())
            lib.OrionHipSynchronize()

        def load(buf):
            if lib.lib.ImportKeyBundle(buf.data_ptr(), buf.numel()) != 0:
                raise RuntimeError(lib.lib.OrionHipLastError().decode())
            lib.OrionHipSynchronize()

        odist.broadcast_bundle(dist, lambda: lib.KeyBundleBytes(1), export, load, torch.device("cuda", local))
    t_setup = time.perf_counter() - t_setup

    # this rank's shard of synthetic images (MNIST-shaped, N(0,1), seed 42 + rank)
    g = torch.Generator().manual_seed(42 + rank)
    imgs = torch.randn(args.batch, 1, 28, 28, generator=g).numpy()
    imgs[0] = st.reference_input().reshape(1, 28, 28)
    ct = st.encrypt_batch(imgs)
    lib.OrionHipSynchronize()

    def step():
        out = st.forward(ct)
        return out

    for _ in range(args.warmup):
        lib.DeleteCiphertext(step())
    lib.OrionHipSynchronize()

    lib.OrionHipProfileReset()
    lib.OrionHipProfile(0b11)  # HIP events around the NTT launches only (the roofline kernel)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    lib.OrionHipSynchronize()
    t0 = time.perf_counter()
    outs = []
    for _ in range(args.steps):
        outs.append(step())
    lib.OrionHipSynchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lib.OrionHipProfile(0)
    prof = lib.profile_read()
    if dist:
        dist.barrier()
        dt = odist.max_over_ranks(dist, dt, torch.device("cuda", local))

    # correctness of the timed output (image 0 is the fixture's reference input)
    res = st.decrypt_output(outs[-1])
    exp = st.arrays["expected_output"].reshape(-1)
    mae = float(np.abs(res[0] - exp).mean())
    if dist:  # every rank decrypts with the key bundle it received: report the worst rank
        mae = odist.max_over_ranks(dist, mae, torch.device("cuda", local))
    for o in outs:
        lib.DeleteCiphertext(o)
    # one extra, fully profiled step (outside the timed region) for the per-kernel breakdown
    lib.OrionHipProfileReset()
    lib.OrionHipProfile(1)
    lib.DeleteCiphertext(step())
    lib.OrionHipProfile(0)
    breakdown = lib.profile_read()

    # client side on the GPU (outside the timed region): encode + encrypt of
    # the batch from HBM-resident slots, and decrypt + decode of the output
    enc_ev = [e for e in st.input_events() if e["op"] == "Encode"][0]
    dvals = torch.zeros(args.batch, st.slots, dtype=torch.float32, device=torch.device("cuda", local))
    dvals[:, :imgs[0].size] = torch.from_numpy(imgs.reshape(args.batch, -1)).to(dvals.device)
    torch.cuda.synchronize()
    out_ct = step()
    dout = torch.empty(args.batch, lib.N // 2, dtype=torch.float64, device=dvals.device)  # DecodeDevice: [B][N/2]

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
        lib.DecodeDevice(pt, dout.data_ptr())
        lib.DeletePlaintext(pt)

    client_ms = {"encode_encrypt_ms_per_batch": round(client(enc_once), 3),
                 "decrypt_decode_ms_per_batch": round(client(dec_once), 3)}
    lib.DeleteCiphertext(out_ct)

    # BASELINE configs[2] (LoLA N=2^15, batch=1): single-image latency of the
    # same op stream, outside the timed region (one image per launch leaves
    # most CUs idle; the throughput line above is the batched shard)
    ct1 = st.encrypt_batch(imgs[:1])
    lib.DeleteCiphertext(st.forward(ct1))
    lib.OrionHipSynchronize()
    reps1 = 10
    t1 = time.perf_counter()
    for _ in range(reps1):
        lib.DeleteCiphertext(st.forward(ct1))
    lib.OrionHipSynchronize()
    b1_ms = (time.perf_counter() - t1) / reps1 * 1e3
    lib.DeleteCiphertext(ct1)

    images = args.batch * world * args.steps
    value = images / dt
    ntt = [prof.get("ntt_fwd", {}), prof.get("ntt_inv", {})]
    n_launch = sum(p.get("launches", 0) for p in ntt)
    n_ms = sum(p.get("ms", 0.0) for p in ntt)
    n_bytes = sum(p.get("bytes", 0.0) for p in ntt)
    achieved = (n_bytes / (n_ms / 1e3)) / 1e9 if n_ms > 0 else 0.0
    total_prof_ms = sum(p["ms"] for p in breakdown.values())
    bd_ntt_ms = breakdown.get("ntt_fwd", {}).get("ms", 0) + breakdown.get("ntt_inv", {}).get("ms", 0)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "ntt_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        # HBM bytes per algorithmic byte of the NTT launches, from the committed
        # rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/pmc_summary.py)
        if tj.get("workload") == args.workload and tj.get("batch") == args.batch and n_launch:
            traffic = round(tj["hbm_bytes_per_algorithmic_byte"] * n_bytes / n_launch)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(args.workload, args.cpu_images, args.cpu_workers)
            except Exception as e:  # the baseline must never break the GPU line
                cpu = dict(value=None, unit="images/s", cores=1, kind="port", sample=f"failed: {e}")
        line = {
            "metric": "encrypted images/sec (LoLa N=2^15) + NTT HBM GB/s vs peak",
            "value": round(value, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: N(0,1) 1x28x28 images (image 0 = fixture input), LoLA diagonals from the "
                    "reference frontend's compile of seeded random-init weights",
            "config": {"workload": f"LoLA (models/lola.py) {args.workload}: N=2^15, LogQ=[60]+[40]x11, "
                                   f"LogP=[60,60], input level {st.input_level}, Standard ring",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "parallelism": f"replicas x{world} (image shards), keys RCCL-broadcast"},
            "roofline": {"bound": "hbm", "kernel": "ntt (fwd+inv: one-pass, 1 limb per workgroup; two-pass for partial-round launches)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "launches": n_launch, "avg_launch_us": round(n_ms / max(n_launch, 1) * 1e3, 2),
                         "algorithmic_bytes_per_launch": round(n_bytes / max(n_launch, 1)),
                         "ntt_share_of_kernel_time": round(bd_ntt_ms / total_prof_ms, 3) if total_prof_ms else None},
            "cpu_baseline": cpu,
            "check": {"mae_image0_vs_cleartext": mae, "mae_over_ranks": "max", "setup_s": round(t_setup, 1)},
            "client_gpu": dict(client_ms, end_to_end_images_per_s=round(
                args.batch / ((dt / args.steps) + (client_ms["encode_encrypt_ms_per_batch"]
                                                   + client_ms["decrypt_decode_ms_per_batch"]) / 1e3) * world, 3)),
            "batch1": {"ms_per_image": round(b1_ms, 3), "images_per_s": round(1e3 / b1_ms, 1)},
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
